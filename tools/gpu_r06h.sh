# round 6: the four-wave LK kernel.  Digests against the one-wave kernel (UVIO_HP_LK_1WAVE=1), the whole GPU suite,
# alternating cfg3 A/B, then the cfg3 per-frame profile.  usage: bash tools/gpu_r06h.sh TAG
set -e
TAG=${1:-r06h}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
for wl in cfg3 cfg2; do
  timeout -k 10 200 python -u tools/ab_state_digest.py $wl 40 > $O/digest_${wl}_lk4.txt 2>&1
  UVIO_HP_LK_1WAVE=1 timeout -k 10 200 python -u tools/ab_state_digest.py $wl 40 > $O/digest_${wl}_lk1.txt 2>&1
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --workload cfg3 --steps 300 --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/lk4_cfg3_$i.json 2> /dev/null
  UVIO_HP_LK_1WAVE=1 timeout -k 10 200 python -u bench.py --workload cfg3 --steps 300 --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/lk1_cfg3_$i.json 2> /dev/null
done
bash tools/gpu_tl_wl.sh $TAG cfg3 200

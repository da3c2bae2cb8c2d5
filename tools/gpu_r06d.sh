# round 6: digests of the six-launch delayed-init chain against the eight-launch one, the whole GPU suite + smoke,
# then alternating cfg3 / cfg3t bench runs of the two chains.  usage: bash tools/gpu_r06d.sh TAG
set -e
TAG=${1:-r06d}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
for wl in cfg3t cfg3; do
  timeout -k 10 200 python -u tools/ab_state_digest.py $wl 40 > $O/digest_${wl}_fused.txt 2>&1
  UVIO_HP_DI_UNFUSED=1 timeout -k 10 200 python -u tools/ab_state_digest.py $wl 40 > $O/digest_${wl}_unfused.txt 2>&1
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
for i in 1 2; do
  for wl in cfg3 cfg3t; do
    timeout -k 10 200 python -u bench.py --workload $wl --steps 200 --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/fused_${wl}_$i.json 2> /dev/null
    UVIO_HP_DI_UNFUSED=1 timeout -k 10 200 python -u bench.py --workload $wl --steps 200 --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/unfused_${wl}_$i.json 2> /dev/null
  done
done

# round 6: fused delayed-init chain checks.  Digests fused vs UVIO_HP_DI_UNFUSED=1, the lock-step subset, a cfg3t
# A/B of the two chains, then the cfg3t timeline / per-frame / gaps / host profile.  usage: bash tools/gpu_r06c.sh TAG
set -e
TAG=${1:-r06c}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
for wl in cfg3t cfg3; do
  timeout -k 10 200 python -u tools/ab_state_digest.py $wl 40 > $O/digest_${wl}_fused.txt 2>&1
  UVIO_HP_DI_UNFUSED=1 timeout -k 10 200 python -u tools/ab_state_digest.py $wl 40 > $O/digest_${wl}_unfused.txt 2>&1
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py tests/test_gpu_updaters.py -x -v -s --timeout 300 --timeout-method thread > $O/lockstep.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --workload cfg3t --steps 100 --cpu-frames 0 --no-host-feed > $O/fused_cfg3t_$i.json 2> /dev/null
  UVIO_HP_DI_UNFUSED=1 timeout -k 10 200 python -u bench.py --workload cfg3t --steps 100 --cpu-frames 0 --no-host-feed > $O/unfused_cfg3t_$i.json 2> /dev/null
done
bash tools/gpu_tl_wl.sh $TAG cfg3t 100

# GPU tests, chi2 phases, host profiles (cfg4 / cfg3), the cfg3 timeline and the cfg4 sharded timeline.
# usage: bash tools/gpu_check2.sh TAG
TAG=${1:-chk}; O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/feat_phases.py cfg3 > $O/feat_phases_cfg3.txt 2>&1 &&
UVIO_HP_HOST_PROF=1 timeout -k 10 300 python -u bench.py --workload cfg4 --steps 300 --cpu-frames 0 --no-host-feed > $O/hp_cfg4.json 2> $O/hp_cfg4.err &&
bash tools/gpu_tl_wl.sh $TAG cfg3 200 &&
bash tools/gpu_tl_wl.sh $TAG cfg4 100 --shard
rc=$?
tail -3 $O/gpu_tests.log; grep -h "chi2" $O/feat_phases_cfg3.txt
exit $rc

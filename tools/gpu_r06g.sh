# round 6: the RCCL-sharded MSCKF update inside the frame chain.  Shard tests (world 1 over RCCL: the chain path;
# worlds 2 / 4 / 8 over gloo: the per-updater path), then cfg4 sharded (world 1) against unsharded.
# usage: bash tools/gpu_r06g.sh TAG
set -e
TAG=${1:-r06g}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_shard.py -x -v -s --timeout 400 --timeout-method thread > $O/shard_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --workload cfg4 --shard --steps 200 --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/shard_cfg4_$i.json 2> $O/shard_$i.err
  timeout -k 10 200 python -u bench.py --workload cfg4 --steps 200 --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/plain_cfg4_$i.json 2> /dev/null
done

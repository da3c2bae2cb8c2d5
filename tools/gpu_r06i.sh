# round 6: the feature-sharded MSCKF update inside the frame chain for both all-reduce backends: the shard tests
# (world 1 over RCCL, worlds 2 / 4 / 8 over gloo on one GPU), then the digests of cfg3 / cfg3t (unsharded, unchanged).
# usage: bash tools/gpu_r06i.sh TAG
set -e
TAG=${1:-r06i}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_shard.py -x -v -s --timeout 400 --timeout-method thread > $O/shard_tests.log 2>&1
for wl in cfg3t cfg3; do
  timeout -k 10 200 python -u tools/ab_state_digest.py $wl 40 > $O/digest_${wl}.txt 2>&1
done

# round 6: the cfg4 frame in its sharded form (world 1 over RCCL, bench.py --shard) and unsharded: per-frame kernel
# summaries, gaps and host sections, for DESIGN.md section 7's bound.  usage: bash tools/gpu_r06s.sh TAG
set -e
TAG=${1:-r06s}
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_tl_wl.sh $TAG cfg4 100 --shard
bash tools/gpu_tl_wl.sh $TAG cfg4 100

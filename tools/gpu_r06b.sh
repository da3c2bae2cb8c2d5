# lock-step subset, then the cfg3t timeline / per-frame / gaps / host profile.  usage: bash tools/gpu_r06b.sh TAG WL
set -e
TAG=${1:-r06b}; WL=${2:-cfg3t}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py -x -v -s --timeout 300 --timeout-method thread > $O/lockstep.log 2>&1
bash tools/gpu_tl_wl.sh $TAG $WL 100

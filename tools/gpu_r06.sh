# round 6: the grid-sort tests first, then the whole GPU suite and smoke.  usage: bash tools/gpu_r06.sh TAG
set -e
TAG=${1:-r06}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_grid_sort.py -x -v -s --timeout 200 --timeout-method thread > $O/grid_tests.log 2>&1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1

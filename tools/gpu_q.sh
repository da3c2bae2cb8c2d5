# quick round check: GPU tests then the default bench line.  usage: bash tools/gpu_q.sh TAG [pytest-args]
set -e
TAG=${1:-rXX}; shift || true
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > $O/gpu_tests.log 2>&1
timeout -k 10 400 python -u bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err

# development check on one MI355X: every GPU test (-s: the steering events print), then short bench lines.
# usage: bash tools/gpu_check.sh TAG [workload:steps ...]
set -e
TAG=${1:-dev}; shift || true
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
for ws in "$@"; do
  wl=${ws%%:*}; st=${ws##*:}
  timeout -k 10 400 python -u bench.py --workload $wl --steps $st --cpu-frames 2 > $O/bench_$wl.json 2> $O/bench_$wl.err
done

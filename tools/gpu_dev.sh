# development check on one MI355X: selected GPU tests, then a kernel-trace profile of the cfg2 bench.
# usage: bash tools/gpu_dev.sh TAG "pytest -k expression" [workload]
set -e
TAG=${1:-dev}; KEXPR=${2:-parity}; WL=${3:-cfg2}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$KEXPR" > $O/gpu_tests.log 2>&1
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --workload $WL --steps 200 --cpu-frames 0 > $O/bench_$WL.json 2> $O/bench.err)
python tools/prof_summary.py $O/prof/run_kernel_trace.csv > $O/per_frame_$WL.txt
rm -f $O/prof/run_kernel_trace.csv

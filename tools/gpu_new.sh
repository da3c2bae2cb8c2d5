# New / changed GPU tests plus the driver-form bench line and its kernel-trace summary.  usage: bash tools/gpu_new.sh TAG [pytest -k expr]
set -e
TAG=${1:-dev}; K=${2:-}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread -k "$K" > $O/gpu_tests.log 2>&1
fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/${TAG}_cfg3_bench_driver_form.json 2> $O/cfg3_driver.err
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfg3 -o run -- python3 $R/bench.py --steps 20 --warmup 5 --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/prof_cfg3.json 2> $O/prof_cfg3.err)
python tools/prof_summary.py $O/prof_cfg3/run_kernel_trace.csv > $O/${TAG}_cfg3_per_frame.txt
cp $O/prof_cfg3/run_kernel_stats.csv $O/${TAG}_cfg3_kernel_stats.csv
rm -f $O/prof_cfg3/run_kernel_trace.csv

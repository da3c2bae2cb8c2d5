# Round profile set on one MI355X, in two parts (each fits one gpurun call):
#   part 1: GPU tests, smoke, the cfg3 (default) and cfg2 bench lines with CPU baselines, the driver form, kernel-trace
#           statistics of the cfg3 and cfg2 benches (per-frame summaries);
#   part 2: the other workloads' bench lines (cfg2l, cfg4i, cfg5i, cfg4, cfg5).
# PMC passes: tools/gpu_pmc.sh.   usage: bash tools/gpu_final.sh TAG [1|2]
set -e
TAG=${1:-rXX}; PART=${2:-1}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
if [ "$PART" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  timeout -k 10 400 python -u bench.py > $O/${TAG}_cfg3_bench.json 2> $O/cfg3.err
  timeout -k 10 400 python -u bench.py --workload cfg2 > $O/${TAG}_cfg2_bench.json 2> $O/cfg2.err
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/${TAG}_cfg3_bench_driver_form.json 2> $O/cfg3_driver.err
  export TMPDIR=/tmp
  for wl in cfg3 cfg2; do
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$wl -o run -- python3 $R/bench.py --workload $wl --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/prof_$wl.log 2>&1)
    python tools/prof_summary.py $O/prof_$wl/run_kernel_trace.csv > $O/${TAG}_${wl}_per_frame.txt
    cp $O/prof_$wl/run_kernel_stats.csv $O/${TAG}_${wl}_kernel_stats.csv
    rm -f $O/prof_$wl/run_kernel_trace.csv
  done
else
  for wl in cfg2l cfg4i cfg5i cfg4 cfg5; do
    timeout -k 10 400 python -u bench.py --workload $wl > $O/${TAG}_${wl}_bench.json 2> $O/$wl.err
  done
fi

# Round-6 profile set, in parts that each fit one gpurun call (run tools/gpu_pmc.sh TAG cfg3 cfg3t first):
#   1: kernel-trace summaries of the cfg3, cfg3t and cfg2 benches (per-frame with the library hash, gaps, timelines)
#      copied into profiles/, then the whole GPU suite and smoke;
#   2: the bench lines: cfg3 (default, with the CPU baseline and the msckf_load companion), cfg2, the driver form,
#      cfg3 over 300 frames;
#   3: the other workloads' lines (cfg3t, cfg2l, cfg4i, cfg5i, cfg5, cfg4 over 300 frames).
# usage: bash tools/gpu_final6.sh TAG PART
set -e
TAG=${1:-rXX}; PART=${2:-1}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O profiles
if [ "$PART" = "1" ]; then
  export TMPDIR=/tmp
  for wl in cfg3 cfg3t cfg2; do
    steps=200; [ $wl = cfg3t ] && steps=60
    cut=k_hist_multi; [ $wl = cfg3t ] && cut=k_prop_clone
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$wl -o run -- python3 $R/bench.py --workload $wl --steps $steps --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/prof_$wl.log 2>&1)
    python tools/prof_summary.py $O/prof_$wl/run_kernel_trace.csv > $O/${TAG}_${wl}_per_frame.txt
    python tools/gap_summary.py $O/prof_$wl/run_kernel_trace.csv > $O/${TAG}_${wl}_gaps.txt
    UVIO_TL_CUT=$cut python tools/frame_timeline.py $O/prof_$wl/run_kernel_trace.csv 40 2 > $O/${TAG}_${wl}_timeline.txt
    cp $O/prof_$wl/run_kernel_stats.csv $O/${TAG}_${wl}_kernel_stats.csv
    rm -f $O/prof_$wl/run_kernel_trace.csv
  done
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
elif [ "$PART" = "2" ]; then
  timeout -k 10 400 python -u bench.py > $O/${TAG}_cfg3_bench.json 2> $O/cfg3.err
  timeout -k 10 400 python -u bench.py --workload cfg2 > $O/${TAG}_cfg2_bench.json 2> $O/cfg2.err
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/${TAG}_cfg3_bench_driver_form.json 2> $O/cfg3_driver.err
  timeout -k 10 300 python -u bench.py --steps 300 --cpu-frames 0 --msckf-load-steps 0 > $O/${TAG}_cfg3_bench_300.json 2> $O/cfg3_300.err
else
  for wl in cfg3t cfg2l cfg4i cfg5i cfg5; do
    timeout -k 10 400 python -u bench.py --workload $wl > $O/${TAG}_${wl}_bench.json 2> $O/$wl.err
  done
  timeout -k 10 400 python -u bench.py --workload cfg4 --steps 300 > $O/${TAG}_cfg4_bench_300.json 2> $O/cfg4.err
fi

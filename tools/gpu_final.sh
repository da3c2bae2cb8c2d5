# Round profile set on one MI355X (run through gpurun): GPU tests, PMC traffic passes (FETCH_SIZE,
# WRITE_SIZE in separate runs) for cfg2 / cfg4, bench lines cfg2..cfg5 with CPU baselines, and the
# kernel-trace statistics of the default bench.  usage: bash tools/gpu_final.sh TAG   (e.g. r01f)
set -e
TAG=${1:-rXX}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
export TMPDIR=/tmp
for wl in cfg2 cfg4; do
  steps=100; [ $wl = cfg4 ] && steps=20
  (cd /tmp && timeout -k 10 -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf_$wl -o run -- python3 $R/bench.py --workload $wl --steps $steps --warmup 20 --cpu-frames 0 > $O/pf_$wl.log 2>&1)
  (cd /tmp && timeout -k 10 -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pw_$wl -o run -- python3 $R/bench.py --workload $wl --steps $steps --warmup 20 --cpu-frames 0 > $O/pw_$wl.log 2>&1)
  python tools/pmc_summary.py $O/pf_$wl/run_counter_collection.csv $O/pw_$wl/run_counter_collection.csv profiles/${TAG}_pmc_traffic_$wl.json
  cp profiles/${TAG}_pmc_traffic_$wl.json $O/
  rm -rf $O/pf_$wl $O/pw_$wl  # per-dispatch counter rows: summarized above, too large to bring back
done
timeout -k 10 400 python -u bench.py > $O/${TAG}_cfg2_bench.json 2> $O/cfg2.err
for wl in cfg3 cfg4 cfg5; do
  timeout -k 10 400 python -u bench.py --workload $wl > $O/${TAG}_${wl}_bench.json 2> $O/$wl.err
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2 -o run -- python3 $R/bench.py --cpu-frames 0 > $O/prof2.log 2>&1)
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof4 -o run -- python3 $R/bench.py --workload cfg4 --cpu-frames 0 > $O/prof4.log 2>&1)
python tools/prof_summary.py $O/prof2/run_kernel_trace.csv > $O/${TAG}_cfg2_per_frame.txt
python tools/prof_summary.py $O/prof4/run_kernel_trace.csv > $O/${TAG}_cfg4_per_frame.txt
rm -f $O/prof2/run_kernel_trace.csv $O/prof4/run_kernel_trace.csv

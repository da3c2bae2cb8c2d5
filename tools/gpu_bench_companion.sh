# The default bench line (driver form, with the msckf_load companion) and a kernel-trace summary of the cfg3t workload.
# usage: bash tools/gpu_bench_companion.sh TAG
set -e
TAG=${1:-dev}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/${TAG}_cfg3_bench_driver_form.json 2> $O/cfg3_driver.err
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfg3t -o run -- python3 $R/bench.py --workload cfg3t --steps 60 --cpu-frames 0 > $O/prof_cfg3t.json 2> $O/prof_cfg3t.err)
python tools/prof_summary.py $O/prof_cfg3t/run_kernel_trace.csv > $O/${TAG}_cfg3t_per_frame.txt
cp $O/prof_cfg3t/run_kernel_stats.csv $O/${TAG}_cfg3t_kernel_stats.csv
rm -f $O/prof_cfg3t/run_kernel_trace.csv

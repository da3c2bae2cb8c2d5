# GPU tests, the cfg3 line and its per-frame kernel summary, then the round-end set's part 2 (other workloads).
# usage: bash tools/gpu_check_final2.sh TAG
TAG=${1:-fin}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/gpu_tests2.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/${TAG}_cfg3_bench2.json 2> $O/cfg3_2.err &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2_cfg3 -o run -- python3 $R/bench.py --cpu-frames 0 --no-host-feed > $O/prof2_cfg3.log 2>&1) &&
python tools/prof_summary.py $O/prof2_cfg3/run_kernel_trace.csv > $O/${TAG}_cfg3_per_frame2.txt &&
cp $O/prof2_cfg3/run_kernel_stats.csv $O/${TAG}_cfg3_kernel_stats2.csv && rm -f $O/prof2_cfg3/run_kernel_trace.csv &&
bash tools/gpu_final.sh $TAG 2
rc=$?
tail -2 $O/gpu_tests2.log; grep -E "prop|clone" $O/${TAG}_cfg3_per_frame2.txt
exit $rc

# The headline evidence in one call: GPU tests, the default bench line (cfg3), its rocprofv3 kernel statistics
# and per-frame summary, the cfg3 PMC passes (profiles/TAG_pmc_traffic_cfg3.json), a cfg4 host profile.
# usage: bash tools/gpu_headline.sh TAG
TAG=${1:-hl}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/${TAG}_cfg3_bench.json 2> $O/cfg3.err &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cfg3 -o run -- python3 $R/bench.py --cpu-frames 0 --no-host-feed > $O/prof_cfg3.log 2>&1) &&
python tools/prof_summary.py $O/prof_cfg3/run_kernel_trace.csv > $O/${TAG}_cfg3_per_frame.txt &&
cp $O/prof_cfg3/run_kernel_stats.csv $O/${TAG}_cfg3_kernel_stats.csv && rm -f $O/prof_cfg3/run_kernel_trace.csv &&
bash tools/gpu_pmc.sh $TAG cfg3 &&
UVIO_HP_HOST_PROF=1 timeout -k 10 300 python -u bench.py --workload cfg4 --steps 300 --cpu-frames 0 --no-host-feed > $O/hp_cfg4.json 2> $O/hp_cfg4.err
rc=$?
tail -2 $O/gpu_tests.log; head -3 $O/${TAG}_cfg3_per_frame.txt
exit $rc

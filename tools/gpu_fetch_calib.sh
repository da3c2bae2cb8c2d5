# FETCH_SIZE / WRITE_SIZE calibration per access width (tools/bench_fetch.hip, prebuilt in build/).
# usage: bash tools/gpu_fetch_calib.sh TAG
set -e
TAG=${1:-fc}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 $R/build/bench_fetch > $O/bench_fetch.csv
(cd /tmp && timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf -o run -- $R/build/bench_fetch > /dev/null 2>&1)
(cd /tmp && timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pw -o run -- $R/build/bench_fetch > /dev/null 2>&1)
python3 tools/fetch_calib.py $O/bench_fetch.csv $O/pf/run_counter_collection.csv $O/pw/run_counter_collection.csv > $O/fetch_calib.txt
cat $O/fetch_calib.txt

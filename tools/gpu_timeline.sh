set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03x; mkdir -p $O; export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 $R/bench.py --steps 60 --cpu-frames 0 > $O/bench.json 2> $O/bench.err)
python $R/tools/frame_timeline.py $O/tr/run_kernel_trace.csv 30 3 > $O/timeline.txt
rm -f $O/tr/run_kernel_trace.csv

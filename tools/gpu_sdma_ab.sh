set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03z; mkdir -p $O; export TMPDIR=/tmp
cd $R
timeout -k 10 200 python -u bench.py --steps 300 --cpu-frames 0 > $O/a.json 2> $O/a.err
HSA_ENABLE_SDMA=0 timeout -k 10 200 python -u bench.py --steps 300 --cpu-frames 0 > $O/b.json 2> $O/b.err
timeout -k 10 200 python -u bench.py --steps 300 --cpu-frames 0 > $O/c.json 2> $O/c.err
HSA_ENABLE_SDMA=0 timeout -k 10 200 python -u bench.py --steps 300 --cpu-frames 0 > $O/d.json 2> $O/d.err
(cd /tmp && HSA_ENABLE_SDMA=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 $R/bench.py --steps 200 --cpu-frames 0 > $O/e.json 2> $O/e.err)
python $R/tools/frame_timeline.py $O/tr/run_kernel_trace.csv 100 2 > $O/timeline.txt
python $R/tools/gap_summary.py $O/tr/run_kernel_trace.csv > $O/gaps_cfg2.txt
rm -f $O/tr/run_kernel_trace.csv

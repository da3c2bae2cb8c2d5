# development check + one-frame timelines: selected GPU tests, then a short traced cfg2 bench.
# usage: bash tools/gpu_dev_tl.sh TAG "pytest -k expression"
set -e
TAG=${1:-dev}; KEXPR=${2:-parity}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$KEXPR" > $O/gpu_tests.log 2>&1
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 $R/bench.py --steps 200 --cpu-frames 0 > $O/bench.json 2> $O/bench.err)
python $R/tools/frame_timeline.py $O/tr/run_kernel_trace.csv 100 3 > $O/timeline.txt
python $R/tools/prof_summary.py $O/tr/run_kernel_trace.csv > $O/per_frame_cfg2.txt
python $R/tools/gap_summary.py $O/tr/run_kernel_trace.csv > $O/gaps_cfg2.txt
rm -f $O/tr/run_kernel_trace.csv

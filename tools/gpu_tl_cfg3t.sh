# one-frame device timelines of the cfg3t workload (TrackSIM feed at cfg3's MSCKF load).  usage: bash tools/gpu_tl_cfg3t.sh TAG
set -e
TAG=${1:-dev}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 $R/bench.py --workload cfg3t --steps 60 --cpu-frames 0 > $O/bench.json 2> $O/bench.err)
UVIO_TL_CUT=k_prop_clone python $R/tools/frame_timeline.py $O/tr/run_kernel_trace.csv 60 2 > $O/timeline.txt
python $R/tools/prof_summary.py $O/tr/run_kernel_trace.csv > $O/per_frame_cfg3t.txt
rm -f $O/tr/run_kernel_trace.csv

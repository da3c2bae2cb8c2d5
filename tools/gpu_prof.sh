# kernel-trace profiles of bench workloads on one MI355X (no tests).  usage: bash tools/gpu_prof.sh TAG workload...
set -e
TAG=${1:-dev}; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
export TMPDIR=/tmp
for wl in "$@"; do
  steps=200; [ $wl != cfg2 ] && [ $wl != cfg3 ] && steps=60
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$wl -o run -- python3 $R/bench.py --workload $wl --steps $steps --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/bench_$wl.json 2> $O/bench_$wl.err)
  python tools/prof_summary.py $O/prof_$wl/run_kernel_trace.csv > $O/per_frame_$wl.txt
  python tools/gap_summary.py $O/prof_$wl/run_kernel_trace.csv > $O/gaps_$wl.txt
  cut=k_hist_multi; case $wl in cfg3t|cfg4|cfg5) cut=k_prop_clone;; esac
  UVIO_TL_CUT=$cut python tools/frame_timeline.py $O/prof_$wl/run_kernel_trace.csv 40 3 > $O/timeline_$wl.txt
  rm -f $O/prof_$wl/run_kernel_trace.csv
done

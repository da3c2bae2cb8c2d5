# Kernel-trace per-frame summaries of bench workloads (tools/prof_summary.py; the trace itself is deleted).
# usage: bash tools/gpu_prof_wl.sh TAG STEPS WORKLOAD...
set -e
T=$1; S=$2; shift 2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for wl in "$@"; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p_$wl -o run -- python3 $R/bench.py --workload $wl --steps $S --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/p_$wl.log 2>&1)
  python tools/prof_summary.py $O/p_$wl/run_kernel_trace.csv > $O/${T}_${wl}_per_frame.txt
  cut=k_hist_multi; case $wl in cfg3t|cfg4) cut=k_prop_clone;; cfg5) cut=k_gemm_HPg_tiled;; esac
  cut=${TL_CUT:-$cut}
  UVIO_TL_CUT=$cut python tools/frame_timeline.py $O/p_$wl/run_kernel_trace.csv 20 2 > $O/${T}_${wl}_timeline.txt
  rm -rf $O/p_$wl
  head -16 $O/${T}_${wl}_per_frame.txt
done

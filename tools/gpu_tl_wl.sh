# one-frame device timelines + per-frame kernel summary + host sections of a workload (no tests).
# usage: bash tools/gpu_tl_wl.sh TAG WORKLOAD [STEPS] [EXTRA BENCH ARGS, e.g. --shard]
set -e
TAG=${1:-tl}; WL=${2:-cfg3}; STEPS=${3:-200}; EXTRA=${4:-}
SFX=$WL$(echo "$EXTRA" | tr -d ' -')
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 $R/bench.py --workload $WL --steps $STEPS --cpu-frames 0 --no-host-feed --msckf-load-steps 0 $EXTRA > $O/bench_$SFX.json 2> $O/bench_$SFX.err)
python $R/tools/frame_timeline.py $O/tr/run_kernel_trace.csv 100 3 > $O/timeline_$SFX.txt
python $R/tools/prof_summary.py $O/tr/run_kernel_trace.csv > $O/per_frame_$SFX.txt
python $R/tools/gap_summary.py $O/tr/run_kernel_trace.csv > $O/gaps_$SFX.txt
rm -f $O/tr/run_kernel_trace.csv
UVIO_HP_HOST_PROF=1 timeout -k 10 300 python -u bench.py --workload $WL --steps 300 --cpu-frames 0 --no-host-feed --msckf-load-steps 0 $EXTRA > $O/hp_$SFX.json 2> $O/hp_$SFX.err

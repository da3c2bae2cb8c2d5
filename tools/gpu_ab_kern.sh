# A/B of two library builds (abl/lib_old.so, abl/lib_new.so) for a kernel change that must keep every value:
# 30-frame digests, each build's per-frame kernel summary lines matching PATTERN, alternating benches.
# usage: bash tools/gpu_ab_kern.sh TAG PATTERN [WORKLOAD...]
set -e
T=$1; PAT=$2; shift 2
WLS=${@:-cfg5 cfg4 cfg3t}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
cd $R && mkdir -p $O
export TMPDIR=/tmp
for lib in old new; do
  for wl in $WLS; do
    echo "$lib $wl $(UVIO_HP_LIB=$R/abl/lib_$lib.so timeout -k 10 200 python -u tools/ab_state_digest.py $wl 30 2>/dev/null | tail -1)" >> $O/digests.txt
  done
done
cat $O/digests.txt
for lib in old new; do
  for wl in $WLS; do
    (cd /tmp && UVIO_HP_LIB=$R/abl/lib_$lib.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p_${lib}_$wl -o run -- python3 $R/bench.py --workload $wl --steps 40 --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/p_${lib}_$wl.log 2>&1)
    python tools/prof_summary.py $O/p_${lib}_$wl/run_kernel_trace.csv > $O/${wl}_${lib}_per_frame.txt
    rm -rf $O/p_${lib}_$wl
    echo "$lib $wl: $(grep -E "$PAT" $O/${wl}_${lib}_per_frame.txt | tr -s ' ' | tr '\n' '|')"
  done
done
for wl in $WLS; do
  bash tools/gpu_libs_ab.sh $T/ab 3 120 $wl abl/lib_old.so abl/lib_new.so
done

# Round 6: k_chi2 instantiated per panel rows (lib_new) against the previous build (lib_old): digests, kernel
# summaries, alternating benches.  usage: bash tools/gpu_r06c2.sh TAG
set -e
T=${1:-r06c2}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
cd $R && mkdir -p $O
export TMPDIR=/tmp
for lib in old new; do
  for wl in cfg3 cfg3t cfg4 cfg5 cfg2; do
    echo "$lib $wl $(UVIO_HP_LIB=$R/abl/lib_$lib.so timeout -k 10 200 python -u tools/ab_state_digest.py $wl 30 2>/dev/null | tail -1)" >> $O/digests.txt
  done
done
cat $O/digests.txt
for wl in cfg5 cfg4 cfg3t cfg3; do
  (cd /tmp && UVIO_HP_LIB=$R/abl/lib_new.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p_$wl -o run -- python3 $R/bench.py --workload $wl --steps 40 --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/p_$wl.log 2>&1)
  python tools/prof_summary.py $O/p_$wl/run_kernel_trace.csv > $O/${wl}_new_per_frame.txt
  python tools/kernel_split.py $O/p_$wl/run_kernel_trace.csv k_chi2 >> $O/${wl}_new_per_frame.txt
  rm -rf $O/p_$wl
  grep -E "span|k_chi2" $O/${wl}_new_per_frame.txt
done
bash tools/gpu_libs_ab.sh $T/ab 3 120 cfg5 abl/lib_old.so abl/lib_new.so
bash tools/gpu_libs_ab.sh $T/ab 3 120 cfg4 abl/lib_old.so abl/lib_new.so
bash tools/gpu_libs_ab.sh $T/ab 3 100 cfg3t abl/lib_old.so abl/lib_new.so
bash tools/gpu_libs_ab.sh $T/ab 2 200 cfg3 abl/lib_old.so abl/lib_new.so

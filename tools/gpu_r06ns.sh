# Round 6: k_feature's reflector application with batched LDS loads (lib_new) against the previous build (lib_old):
# 40-frame state digests of cfg3 / cfg3t / cfg2 for both, a kernel-trace of cfg3t per build, then alternating benches.
# usage: bash tools/gpu_r06ns.sh TAG
set -e
T=${1:-r06ns}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
cd $R && mkdir -p $O
export TMPDIR=/tmp
for lib in old new; do
  for wl in cfg3 cfg3t cfg2; do
    echo "$lib $wl $(UVIO_HP_LIB=$R/abl/lib_$lib.so timeout -k 10 200 python -u tools/ab_state_digest.py $wl 40 2>/dev/null | tail -1)" >> $O/digests.txt
  done
done
cat $O/digests.txt
for lib in old new; do
  (cd /tmp && UVIO_HP_LIB=$R/abl/lib_$lib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$lib -o run -- python3 $R/bench.py --workload cfg3t --steps 60 --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/prof_$lib.log 2>&1)
  python tools/prof_summary.py $O/prof_$lib/run_kernel_trace.csv > $O/cfg3t_${lib}_per_frame.txt
  rm -f $O/prof_$lib/run_kernel_trace.csv
  grep -E "k_feature|span" $O/cfg3t_${lib}_per_frame.txt | head -3
done
bash tools/gpu_libs_ab.sh $T/ab 3 200 cfg3t abl/lib_old.so abl/lib_new.so
bash tools/gpu_libs_ab.sh $T/ab 3 200 cfg3 abl/lib_old.so abl/lib_new.so

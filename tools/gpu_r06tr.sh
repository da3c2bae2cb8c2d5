# Round 6: the prefactor's V solve held back until the chi2 T GEMM has run (lib_new) against the previous build
# (lib_old): 40-frame state digests (cfg3, cfg3t, cfg2, cfg4, cfg5), a cfg5 kernel trace per build, alternating benches.
# usage: bash tools/gpu_r06tr.sh TAG
set -e
T=${1:-r06tr}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
cd $R && mkdir -p $O
export TMPDIR=/tmp
for lib in old new; do
  for wl in cfg3 cfg3t cfg2 cfg4 cfg5; do
    echo "$lib $wl $(UVIO_HP_LIB=$R/abl/lib_$lib.so timeout -k 10 200 python -u tools/ab_state_digest.py $wl 30 2>/dev/null | tail -1)" >> $O/digests.txt
  done
done
cat $O/digests.txt
for lib in old new; do
  (cd /tmp && UVIO_HP_LIB=$R/abl/lib_$lib.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p_$lib -o run -- python3 $R/bench.py --workload cfg5 --steps 40 --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/p_$lib.log 2>&1)
  python tools/prof_summary.py $O/p_$lib/run_kernel_trace.csv > $O/cfg5_${lib}_per_frame.txt
  UVIO_TL_CUT=k_gemm_HPg_tiled python tools/frame_timeline.py $O/p_$lib/run_kernel_trace.csv 20 1 > $O/cfg5_${lib}_timeline.txt
  rm -rf $O/p_$lib
  grep -E "span|HPg_tiled|k_trsm|cholP|cholZ|chi2_S" $O/cfg5_${lib}_per_frame.txt
done
bash tools/gpu_libs_ab.sh $T/ab 3 150 cfg5 abl/lib_old.so abl/lib_new.so
bash tools/gpu_libs_ab.sh $T/ab 3 150 cfg4 abl/lib_old.so abl/lib_new.so
bash tools/gpu_libs_ab.sh $T/ab 2 200 cfg3 abl/lib_old.so abl/lib_new.so

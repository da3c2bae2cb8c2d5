# Round 6: the split information-form factor for n + 1 > the packed LDS triangle (lib_new) against the previous build
# (lib_old) and against itself with UVIO_HP_NO_INFO_SPLIT=1: digests, a cfg5 kernel summary, alternating benches,
# the cfg5-size lock-step tests.  usage: bash tools/gpu_r06sp.sh TAG
set -e
T=${1:-r06sp}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
cd $R && mkdir -p $O
export TMPDIR=/tmp
for wl in cfg5 cfg5i cfg4; do
  echo "old $wl $(UVIO_HP_LIB=$R/abl/lib_old.so timeout -k 10 200 python -u tools/ab_state_digest.py $wl 30 2>/dev/null | tail -1)" >> $O/digests.txt
  echo "new $wl $(UVIO_HP_LIB=$R/abl/lib_new.so timeout -k 10 200 python -u tools/ab_state_digest.py $wl 30 2>/dev/null | tail -1)" >> $O/digests.txt
  echo "new-nosplit $wl $(UVIO_HP_NO_INFO_SPLIT=1 UVIO_HP_LIB=$R/abl/lib_new.so timeout -k 10 200 python -u tools/ab_state_digest.py $wl 30 2>/dev/null | tail -1)" >> $O/digests.txt
done
cat $O/digests.txt
(cd /tmp && UVIO_HP_LIB=$R/abl/lib_new.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p -o run -- python3 $R/bench.py --workload cfg5 --steps 40 --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/p.log 2>&1)
python tools/prof_summary.py $O/p/run_kernel_trace.csv > $O/cfg5_new_per_frame.txt
UVIO_TL_CUT=k_gemm_HPg_tiled python tools/frame_timeline.py $O/p/run_kernel_trace.csv 20 1 > $O/cfg5_new_timeline.txt
rm -rf $O/p
grep -E "span|split|chol|trsm" $O/cfg5_new_per_frame.txt
bash tools/gpu_libs_ab.sh $T/ab 3 120 cfg5 abl/lib_old.so abl/lib_new.so
bash tools/gpu_libs_ab.sh $T/ab 3 150 cfg5i abl/lib_old.so abl/lib_new.so

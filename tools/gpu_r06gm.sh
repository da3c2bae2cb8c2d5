# Round 6: the tiled chi2 T GEMM templated on its gather (lib_new) against the committed build (lib_old), with the
# prefactor placement modes (UVIO_HP_PREFACTOR 0 / 1 / 2): digests, a cfg5 trace, alternating benches.
# usage: bash tools/gpu_r06gm.sh TAG
set -e
T=${1:-r06gm}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
cd $R && mkdir -p $O
export TMPDIR=/tmp
for lib in old new; do
  for wl in cfg3 cfg3t cfg4 cfg5; do
    echo "$lib $wl $(UVIO_HP_LIB=$R/abl/lib_$lib.so timeout -k 10 200 python -u tools/ab_state_digest.py $wl 30 2>/dev/null | tail -1)" >> $O/digests.txt
  done
done
cat $O/digests.txt
(cd /tmp && UVIO_HP_LIB=$R/abl/lib_new.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p -o run -- python3 $R/bench.py --workload cfg5 --steps 40 --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/p.log 2>&1)
python tools/prof_summary.py $O/p/run_kernel_trace.csv > $O/cfg5_new_per_frame.txt
UVIO_TL_CUT=k_gemm_HPg_tiled python tools/frame_timeline.py $O/p/run_kernel_trace.csv 20 1 > $O/cfg5_new_timeline.txt
rm -rf $O/p
grep -E "span|HPg_tiled|k_trsm|cholP|cholZ|chi2_S|k_chi2 " $O/cfg5_new_per_frame.txt
for i in 1 2 3; do
  for arm in old new:0 new:1 new:2; do
    lib=${arm%%:*}; m=${arm#*:}; [ "$m" = "$arm" ] && m=0
    for wl in cfg5 cfg4 cfg3t; do
      UVIO_HP_PREFACTOR=$m UVIO_HP_LIB=$R/abl/lib_$lib.so timeout -k 10 300 python -u bench.py --workload $wl --steps 120 --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/${wl}_${lib}${m}_$i.json 2>/dev/null
    done
  done
done
python - $O <<'PY'
import json, glob, sys, statistics
o = sys.argv[1]
for wl in ("cfg5", "cfg4", "cfg3t"):
    for arm in ("old0", "new0", "new1", "new2"):
        v = [json.loads(open(f).read().strip().splitlines()[-1])["value"] for f in sorted(glob.glob("%s/%s_%s_*.json" % (o, wl, arm)))]
        print(wl, arm, "median %.1f" % statistics.median(v), " ".join("%.1f" % x for x in v))
PY

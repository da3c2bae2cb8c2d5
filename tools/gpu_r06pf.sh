# Round 6: when the information-form prefactor runs (UVIO_HP_PREFACTOR: 0 at once, 1 V after the chi2 T GEMM, 2 all of
# it after the tiled T GEMM): digests of the modes, a cfg5 trace per mode, alternating benches.  usage: bash tools/gpu_r06pf.sh TAG
set -e
T=${1:-r06pf}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
cd $R && mkdir -p $O
export TMPDIR=/tmp
for m in 0 2; do
  for wl in cfg3 cfg4 cfg5; do
    echo "mode $m $wl $(UVIO_HP_PREFACTOR=$m UVIO_HP_LIB=$R/abl/lib_new.so timeout -k 10 200 python -u tools/ab_state_digest.py $wl 30 2>/dev/null | tail -1)" >> $O/digests.txt
  done
done
echo "old cfg5 $(UVIO_HP_LIB=$R/abl/lib_old.so timeout -k 10 200 python -u tools/ab_state_digest.py cfg5 30 2>/dev/null | tail -1)" >> $O/digests.txt
cat $O/digests.txt
for m in 0 2; do
  (cd /tmp && UVIO_HP_PREFACTOR=$m UVIO_HP_LIB=$R/abl/lib_new.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p_$m -o run -- python3 $R/bench.py --workload cfg5 --steps 40 --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/p_$m.log 2>&1)
  python tools/prof_summary.py $O/p_$m/run_kernel_trace.csv > $O/cfg5_mode${m}_per_frame.txt
  UVIO_TL_CUT=k_gemm_HPg_tiled python tools/frame_timeline.py $O/p_$m/run_kernel_trace.csv 20 1 > $O/cfg5_mode${m}_timeline.txt
  rm -rf $O/p_$m
  grep -E "span|HPg_tiled|k_trsm|cholP|cholZ|chi2_S|k_chi2 " $O/cfg5_mode${m}_per_frame.txt
done
for i in 1 2 3; do
  for m in 0 1 2; do
    for wl in cfg5 cfg4; do
      UVIO_HP_PREFACTOR=$m UVIO_HP_LIB=$R/abl/lib_new.so timeout -k 10 300 python -u bench.py --workload $wl --steps 150 --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/${wl}_m${m}_$i.json 2>/dev/null
    done
  done
done
python - $O <<'PY'
import json, glob, sys, statistics
o = sys.argv[1]
for wl in ("cfg5", "cfg4"):
    for m in (0, 1, 2):
        v = [json.loads(open(f).read().strip().splitlines()[-1])["value"] for f in sorted(glob.glob("%s/%s_m%d_*.json" % (o, wl, m)))]
        print(wl, "mode", m, "median %.1f" % statistics.median(v), " ".join("%.1f" % x for x in v))
PY

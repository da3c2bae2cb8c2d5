# Round 6: k_chi2_S2 (one workgroup per feature, T / H rows staged once per 32-column chunk) against k_chi2_S
# (UVIO_HP_CHI2_S_TILES=1), same library: digests, kernel summaries, alternating benches.  usage: bash tools/gpu_r06s2.sh TAG
set -e
T=${1:-r06s2}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
cd $R && mkdir -p $O
export TMPDIR=/tmp
for arm in tiles s2; do
  ev=""; [ $arm = tiles ] && ev="UVIO_HP_CHI2_S_TILES=1"
  for wl in cfg3t cfg4 cfg5; do
    echo "$arm $wl $(env $ev UVIO_HP_LIB=$R/abl/lib_new.so timeout -k 10 200 python -u tools/ab_state_digest.py $wl 30 2>/dev/null | tail -1)" >> $O/digests.txt
  done
done
cat $O/digests.txt
for wl in cfg5 cfg4 cfg3t; do
  (cd /tmp && UVIO_HP_LIB=$R/abl/lib_new.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p_$wl -o run -- python3 $R/bench.py --workload $wl --steps 40 --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/p_$wl.log 2>&1)
  python tools/prof_summary.py $O/p_$wl/run_kernel_trace.csv > $O/${wl}_s2_per_frame.txt
  rm -rf $O/p_$wl
  grep -E "span|chi2_S|k_chi2 |HPg_tiled" $O/${wl}_s2_per_frame.txt
done
for i in 1 2 3; do
  for arm in tiles s2; do
    for wl in cfg5 cfg4 cfg3t; do
      if [ $arm = tiles ]; then export UVIO_HP_CHI2_S_TILES=1; else unset UVIO_HP_CHI2_S_TILES; fi
      UVIO_HP_LIB=$R/abl/lib_new.so timeout -k 10 300 python -u bench.py --workload $wl --steps 120 --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/${wl}_${arm}_$i.json 2>/dev/null
    done
  done
done
unset UVIO_HP_CHI2_S_TILES
python - $O <<'PY'
import json, glob, sys, statistics
o = sys.argv[1]
for wl in ("cfg5", "cfg4", "cfg3t"):
    for arm in ("tiles", "s2"):
        v = [json.loads(open(f).read().strip().splitlines()[-1])["value"] for f in sorted(glob.glob("%s/%s_%s_*.json" % (o, wl, arm)))]
        print(wl, arm, "median %.1f" % statistics.median(v), " ".join("%.1f" % x for x in v))
PY

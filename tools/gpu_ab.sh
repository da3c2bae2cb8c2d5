# Same-box A/B of the current library against build/abprev/libuvio_hp_prev.so: alternating cfg3 / cfg2 bench runs.
# usage: [WLS="cfg3 cfg4i"] bash tools/gpu_ab.sh TAG [PAIRS]
TAG=${1:-ab}; PAIRS=${2:-3}; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
for i in $(seq 1 $PAIRS); do
  for wl in ${WLS:-cfg3 cfg2}; do
    timeout -k 10 200 python -u bench.py --workload $wl --steps 300 --cpu-frames 0 --no-host-feed > $O/new_${wl}_$i.json 2> /dev/null || exit 1
    UVIO_HP_LIB=$R/build/abprev/libuvio_hp_prev.so UVIO_HP_AB_OLD=1 timeout -k 10 200 python -u bench.py --workload $wl --steps 300 --cpu-frames 0 --no-host-feed > $O/old_${wl}_$i.json 2> /dev/null || exit 1
  done
done
python - "$O" "${WLS:-cfg3 cfg2}" <<'PY'
import json, glob, sys, statistics
o = sys.argv[1]
for wl in sys.argv[2].split():
    for arm in ("new", "old"):
        v = [json.loads(open(f).read().strip().splitlines()[-1])["value"] for f in sorted(glob.glob("%s/%s_%s_*.json" % (o, arm, wl)))]
        print("%s %s: %s  median %.1f" % (wl, arm, " ".join("%.1f" % x for x in v), statistics.median(v)))
PY

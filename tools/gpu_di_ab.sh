# Alternating A/B of the delayed-initialization chain: six launches per candidate (default) against the eight-launch
# chain (UVIO_HP_DI_UNFUSED=1); cfg3t and cfg3, three pairs each.  usage: bash tools/gpu_di_ab.sh TAG
set -e
TAG=${1:-diab}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
cd $R && mkdir -p $O
for i in 1 2 3; do
  for wl in cfg3t cfg3; do
    timeout -k 10 200 python -u bench.py --workload $wl --steps 200 --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/six_${wl}_$i.json 2> /dev/null
    UVIO_HP_DI_UNFUSED=1 timeout -k 10 200 python -u bench.py --workload $wl --steps 200 --cpu-frames 0 --no-host-feed --msckf-load-steps 0 > $O/eight_${wl}_$i.json 2> /dev/null
  done
done
python - "$O" <<'PY'
import json, glob, sys, statistics
o = sys.argv[1]
for wl in ("cfg3t", "cfg3"):
    for arm in ("six", "eight"):
        rs = [json.loads(open(f).read().strip().splitlines()[-1]) for f in sorted(glob.glob("%s/%s_%s_*.json" % (o, arm, wl)))]
        v = [r["value"] for r in rs]
        sd = [r["config"]["stage_ms"]["slam_delayed"] for r in rs]
        cw = [r["config"]["stage_ms"]["chain_wait"] for r in rs]
        print("%s %-5s fps %s median %.1f | slam_delayed median %.3f | chain_wait median %.3f" % (
            wl, arm, " ".join("%.1f" % x for x in v), statistics.median(v), statistics.median(sd), statistics.median(cw)))
PY

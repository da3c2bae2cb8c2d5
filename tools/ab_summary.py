"""Summarize an A/B directory written by tools/gpu_ab.sh: frames/s per arm and workload (each run, mean)."""
import glob
import json
import os
import sys

d = sys.argv[1]
rows = {}
for f in sorted(glob.glob(os.path.join(d, "*_*_*.json"))):
    wl, arm, _ = os.path.basename(f)[:-5].rsplit("_", 2)
    try:
        v = json.load(open(f))["value"]
    except (ValueError, KeyError):
        continue
    rows.setdefault(wl, {}).setdefault(arm, []).append(v)
for wl, arms in rows.items():
    parts = []
    for arm in ("new", "old"):
        vs = arms.get(arm, [])
        if vs:
            parts.append("%s %.1f (%s)" % (arm, sum(vs) / len(vs), ", ".join("%.1f" % v for v in vs)))
    print("%-6s %s" % (wl, "   ".join(parts)))

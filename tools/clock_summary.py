"""Effective clock of chosen kernels from a rocprofv3 --pmc GRBM_GUI_ACTIVE pass (MI355X_MICROARCH.md 'DVFS
give-back': GRBM_GUI_ACTIVE / 8 XCDs / wall time).  usage: python tools/clock_summary.py counter_collection.csv NAME..."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
want = sys.argv[2:]
acc = collections.defaultdict(list)
for r in rows:
    if r.get("Counter_Name") != "GRBM_GUI_ACTIVE":
        continue
    k = r["Kernel_Name"]
    if want and not any(w in k for w in want):
        continue
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9 if r.get("End_Timestamp") else 0.0
    acc[k.split("(")[0][:40]].append((float(r["Counter_Value"]), dur))
for k, v in sorted(acc.items()):
    cyc = sum(c for c, _ in v) / len(v)
    dur = sum(d for _, d in v) / len(v)
    print("%-40s n %4d  GRBM_GUI_ACTIVE/8 %10.0f  wall %8.1f us  clock %5.2f GHz" % (
        k, len(v), cyc / 8, dur * 1e6, cyc / 8 / dur * 1e-9 if dur > 0 else float("nan")))

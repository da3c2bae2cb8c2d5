"""Summarize a rocprofv3 kernel trace: per-kernel totals over the timed region (after the last torch kernel)."""
import collections
import csv
import hashlib
import os
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
nframes = int(sys.argv[2]) if len(sys.argv) > 2 else 0
ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'], r['Grid_Size_X']) for r in rows)
last_torch = max([i for i, e in enumerate(ev) if 'at::' in e[2]] + [-1])
seg = ev[last_torch + 1:]
if nframes <= 0:  # image workloads: one equalizeHist launch per frame; TrackSIM workloads: one propagation per frame
    nframes = max(sum(1 for e in seg if 'k_hist_multi' in e[2]),
                  sum(1 for e in seg if 'k_clone' in e[2] or 'k_prop_clone' in e[2]), 1)
t0, t1 = seg[0][0], seg[-1][1]
busy, cur = 0, t0
for s, e, n, g in seg:
    s2 = max(s, cur)
    if e > s2:
        busy += e - s2
    cur = max(cur, e)
print("kernels %d  span %.1f ms  busy %.1f ms (%.0f%%)  per frame: span %.3f ms busy %.3f ms  launches %.1f" % (
    len(seg), (t1 - t0) / 1e6, busy / 1e6, 100 * busy / (t1 - t0), (t1 - t0) / 1e6 / nframes, busy / 1e6 / nframes,
    len(seg) / nframes))
d = collections.defaultdict(list)
for s, e, n, g in seg:
    d[n.split('(')[0].replace('uvhp::', '').replace('void ', '')].append((e - s) / 1e3)
tot = sum(sum(v) for v in d.values())
for k in sorted(d, key=lambda k: -sum(d[k]))[:28]:
    v = d[k]
    print("%-34s n/frame %6.2f  avg %7.1f us  per frame %7.1f us  %5.1f%%" % (k[:34], len(v) / nframes, sum(v) / len(v),
                                                                        sum(v) / nframes, 100 * sum(v) / tot))
# the library the trace ran (bench.py uses this summary only for the same build): sha256 of the .so, 16 hex
lib = os.environ.get("UVIO_HP_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "uvio_amd",
                                                "libuvio_hp.so"))
if os.path.exists(lib):
    print("library sha256 %s" % hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16])

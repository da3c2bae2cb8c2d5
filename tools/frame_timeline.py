"""One frame's device timeline from a rocprofv3 kernel trace: every kernel / blit in launch order with its start
relative to the frame's histogram launch, its duration and the idle gap before it.  Frames are cut at
k_hist_multi (UVIO_TL_CUT=<kernel> cuts at another kernel, e.g. k_prop_clone for TrackSIM workloads).
usage: frame_timeline.py trace.csv [first_frame] [count]"""
import os
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in rows)
last_torch = max([i for i, e in enumerate(ev) if 'at::' in e[2]] + [-1])
seg = ev[last_torch + 1:]
CUT = os.environ.get('UVIO_TL_CUT', 'k_hist_multi')
starts = [i for i, e in enumerate(seg) if CUT in e[2]]
f0 = int(sys.argv[2]) if len(sys.argv) > 2 else len(starts) // 2
cnt = int(sys.argv[3]) if len(sys.argv) > 3 else 2


def short(n):
    return n.split('(')[0].replace('uvhp::', '').replace('void ', '')[:40]


for f in range(f0, min(f0 + cnt, len(starts) - 1)):
    a, b = starts[f], starts[f + 1]
    t0 = seg[a][0]
    busy = 0
    cur = t0
    print("frame %d: span %.1f us" % (f, (seg[b][0] - t0) / 1e3))
    for s, e, n in seg[a:b]:
        gap = max(0, s - cur) / 1e3
        busy += e - s
        print("  %8.1f  %6.1f  gap %6.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap, short(n)))
        cur = max(cur, e)
    print("  busy %.1f us" % (busy / 1e3))

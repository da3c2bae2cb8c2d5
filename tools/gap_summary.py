"""Device idle gaps in a rocprofv3 kernel trace, grouped by the (previous kernel -> next kernel) pair that
brackets each gap, per frame: where the device waits for the host.  usage: gap_summary.py trace.csv [nframes]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in rows)
# the timed region starts after the last torch kernel (bench.py issues one right before it, so the warm-up of
# TrackSIM workloads, which render nothing, stays out as well)
last_torch = max([i for i, e in enumerate(ev) if 'at::' in e[2]] + [-1])
seg = ev[last_torch + 1:]
nframes = int(sys.argv[2]) if len(sys.argv) > 2 else 0
if nframes <= 0:  # image workloads: one equalizeHist launch per frame; TrackSIM workloads: one propagation per frame
    nframes = max(sum(1 for e in seg if 'k_hist_multi' in e[2]),
                  sum(1 for e in seg if 'k_clone' in e[2] or 'k_prop_clone' in e[2]), 1)


def short(n):
    return n.split('(')[0].replace('uvhp::', '').replace('void ', '')[:28]


gaps = collections.defaultdict(list)
cur_end, prev = seg[0][1], short(seg[0][2])
for s, e, n in seg[1:]:
    if s > cur_end:
        gaps[(prev, short(n))].append((s - cur_end) / 1e3)
    if e >= cur_end:
        cur_end, prev = e, short(n)
tot = sum(sum(v) for v in gaps.values())
print("idle %.1f us/frame over %d frames" % (tot / nframes, nframes))
for k in sorted(gaps, key=lambda k: -sum(gaps[k]))[:30]:
    v = gaps[k]
    print("%-28s -> %-28s n/frame %5.2f  avg %6.1f us  per frame %6.1f us" % (k[0], k[1], len(v) / nframes,
                                                                           sum(v) / len(v), sum(v) / nframes))

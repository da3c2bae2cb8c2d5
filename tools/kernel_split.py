"""Per-launch duration of one kernel split by grid size (e.g. k_feature: one workgroup per delayed-initialization
candidate against the multi-feature MSCKF / SLAM batches).  usage: python tools/kernel_split.py TRACE.csv NAME"""
import collections
import csv
import sys

name = sys.argv[2]
by = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if r['Kernel_Name'].split('(')[0].split('<')[0].endswith(name):
        g = int(r['Grid_Size_X']) // max(int(r['Workgroup_Size_X']), 1)
        by['1 wg' if g == 1 else '2-63 wg' if g < 64 else '>=64 wg'].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k in sorted(by):
    v = sorted(by[k])
    print('%-10s %-8s n %5d  avg %7.2f us  median %7.2f us' % (name, k, len(v), sum(v) / len(v), v[len(v) // 2]))

"""Grid sizes and durations of one kernel's launches in a rocprofv3 kernel trace.  usage: python tools/kernel_grid.py TRACE NAME"""
import collections
import csv
import sys

by = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r['Kernel_Name']:
        by[(int(r['Grid_Size_X']) // int(r['Workgroup_Size_X']), r.get('LDS_Block_Size', ''), r.get('VGPR_Count', ''),
            r.get('Accum_VGPR_Count', ''))].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in sorted(by.items()):
    print('workgroups %6d lds %s vgpr %s agpr %s  n %4d  avg %8.1f us  min %8.1f' % (k[0], k[1], k[2], k[3], len(v), sum(v) / len(v), min(v)))

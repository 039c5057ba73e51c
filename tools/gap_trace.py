"""Median kernel durations and inter-kernel gaps (by kernel pair) from a rocprofv3 kernel trace."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'].split('(')[0][-40:])
            for r in rows if 'dqnx' in r['Kernel_Name'])[-800:]
dur, gap = collections.defaultdict(list), collections.defaultdict(list)
for i, (a, b, c) in enumerate(ks):
    dur[c].append(b - a)
    if i:
        gap[(ks[i - 1][2], c)].append(a - ks[i - 1][1])
med = lambda v: sorted(v)[len(v) // 2]
for k, v in dur.items():
    print(f"dur {k:42s} n={len(v):4d} med {med(v)/1e3:7.2f} us")
for k, v in gap.items():
    print(f"gap {k[0][-25:]:26s}->{k[1][-25:]:26s} n={len(v):4d} med {med(v)/1e3:7.2f} us")

"""Kernel timeline (ms from the superstep's first k_lpa_units) of superstep k
from a rocprofv3 kernel trace:  python tools/timeline.py trace.csv k"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
k = int(sys.argv[2])


def short(n):
    m = re.search(r'(k_[A-Za-z0-9_]+(<[^>]*>)?)', n)
    return m.group(1) if m else n[:25]


idx = [i for i, r in enumerate(rows) if 'k_lpa_units' in r['Kernel_Name']]
a, b = idx[k], (idx[k + 1] if k + 1 < len(idx) else len(rows))
t0 = int(rows[a]['Start_Timestamp'])
for r in rows[a:b]:
    s = (int(r['Start_Timestamp']) - t0) / 1e6
    e = (int(r['End_Timestamp']) - t0) / 1e6
    print(f"{short(r['Kernel_Name']):28s} {s:7.3f} {e:7.3f} {e - s:6.3f}")

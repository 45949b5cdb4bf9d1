"""Per-superstep kernel durations (ms) from a rocprofv3 kernel trace.

A superstep starts at each k_lpa_units dispatch (the first tally kernel); every
dispatch until the next one (hub combine, bins, diff, al refresh) belongs to it.
Columns: one per superstep in launch order; rows: kernels; last row: sum.
"""
import collections
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))


def short(name):
    m = re.search(r'(k_[A-Za-z0-9_]+(<[^>]*>)?)', name)
    return m.group(1) if m else name[:30]


steps = []
for r in rows:
    n = short(r['Kernel_Name'])
    if n == 'k_lpa_units':
        steps.append(collections.OrderedDict())
    if not steps:
        continue
    ms = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
    steps[-1][n] = steps[-1].get(n, 0.0) + ms
names = []
for st in steps:
    for n in st:
        if n not in names:
            names.append(n)
for n in names:
    print(f"{n:18s}", ' '.join(f"{st.get(n, 0.0):6.3f}" for st in steps))
print(f"{'sum':18s}", ' '.join(f"{sum(st.values()):6.3f}" for st in steps))

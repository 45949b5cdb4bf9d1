"""Per-superstep kernel timelines from a rocprofv3 kernel trace (csv): every
superstep starts at a k_lpa_units dispatch.  Prints the superstep spans, then the
dispatch timeline (start / end / duration in ms, queue) of the chosen supersteps.

    python tools/timeline2.py trace.csv [idx ...]
"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))


def short(n):
    m = re.search(r'(k_[A-Za-z0-9_]+(<[^>]*>)?)', n)
    return m.group(1) if m else n[:30]


steps = []
for r in rows:
    n = short(r['Kernel_Name'])
    if n == 'k_frontier_lists':
        steps.append([])
    if steps:
        steps[-1].append((n, int(r['Start_Timestamp']), int(r['End_Timestamp']), r.get('Queue_Id', '')))
spans = [(s[-1][2] - s[0][1]) / 1e6 for s in steps]
print('supersteps:', len(steps))
print('spans ms:', ' '.join(f"{x:.3f}" for x in spans[:80]))
for idx in [int(x) for x in sys.argv[2:]]:
    s = steps[idx]
    t0 = s[0][1]
    print(f'--- superstep {idx} span {spans[idx]:.3f} ms')
    for n, a, b, q in s:
        print(f"{n:30s} q{q:>3s} {(a - t0) / 1e6:7.3f} {(b - t0) / 1e6:7.3f} {(b - a) / 1e6:7.3f}")

"""Per-call kernel breakdown from a rocprofv3 kernel trace: calls start at each
dispatch of the named kernel (default k_edge_keys, the outlier stage's first).

    python tools/trace_calls.py trace.csv [first_kernel] [top]
"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
first = sys.argv[2] if len(sys.argv) > 2 else "k_edge_keys"
top = int(sys.argv[3]) if len(sys.argv) > 3 else 14


def short(n):
    m = re.search(r"(k_[A-Za-z0-9_]+(<[^>]*>)?)", n)
    return m.group(1) if m else n[:30]


starts = [i for i, r in enumerate(rows) if short(r["Kernel_Name"]) == first]
for c, a in enumerate(starts):
    b = starts[c + 1] if c + 1 < len(starts) else len(rows)
    seg = rows[a:b]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
    agg = {}
    for r in seg:
        n = short(r["Kernel_Name"])
        agg[n] = agg.get(n, 0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    print(f"call {c}: span {(t1 - t0) / 1e6:.1f} ms, kernel sum {sum(agg.values()):.1f} ms")
    for n, v in sorted(agg.items(), key=lambda x: -x[1])[:top]:
        print(f"   {n:34s} {v:8.2f}")

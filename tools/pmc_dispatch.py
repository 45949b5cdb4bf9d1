"""Per-dispatch counter table from rocprofv3 --pmc passes (glob of pass dirs):
one row per (kernel, dispatch ordinal), counters side by side + derived ratios."""
import collections
import csv
import glob
import re
import sys

vals = collections.defaultdict(dict)   # (kernel, ordinal) -> counter -> value
for d in sorted(glob.glob(sys.argv[1])):
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            m = re.search(r"(k_[A-Za-z0-9_]+(<[^>]*>)?)", r["Kernel_Name"])
            k = m.group(1) if m else r["Kernel_Name"][:30]
            per[(k, r["Counter_Name"])].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
        for (k, c), lst in per.items():
            lst.sort()
            for i, (_, v) in enumerate(lst):
                vals[(k, i)][c] = v
for (k, i) in sorted(vals):
    row = vals[(k, i)]
    g = row.get
    extra = ""
    if g("SQ_WAVE_CYCLES"):
        extra += f" wait_any {g('SQ_WAIT_ANY', 0) / g('SQ_WAVE_CYCLES'):.2f} wait_inst {g('SQ_WAIT_INST_ANY', 0) / g('SQ_WAVE_CYCLES'):.2f} active {g('SQ_ACTIVE_INST_ANY', 0) / g('SQ_WAVE_CYCLES'):.2f}"
    if g("SQ_LDS_IDX_ACTIVE"):
        extra += f" ldsconf {g('SQ_LDS_BANK_CONFLICT', 0) / g('SQ_LDS_IDX_ACTIVE'):.2f}"
    cs = " ".join(f"{c.replace('SQ_', '')}={v:.3g}" for c, v in sorted(row.items()))
    print(f"{k:22s} #{i:<2d}{extra} | {cs}")

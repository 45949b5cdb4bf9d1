"""Per-kernel sums of rocprofv3 --pmc counter CSVs: python tools/sq_summary.py DIR..."""
import csv
import glob
import re
import sys
from collections import defaultdict

tot = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("lpa::(anonymous namespace)::", "").replace("void ", "")
            k = re.sub(r"\(.*", "", k)
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
for k in sorted(tot, key=lambda k: -tot[k].get("SQ_WAVE_CYCLES", 0)):
    c = tot[k]
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    line = f"{k[:40]:40s} n={len(disp[k]):3d} wc={wc:.3g}"
    for n in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
        if n in c:
            line += f" {n[3:]}={c[n] / wc:.2f}"
    for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_LDS_BANK_CONFLICT", "SQ_WAVES"):
        if n in c:
            line += f" {n[3:]}={c[n]:.3g}"
    print(line)

"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc_*/run_counter_collection.csv):
per LPA kernel, counters averaged over the steady-state dispatches (last N)."""
import csv
import collections
import glob
import re
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
last = int(sys.argv[2]) if len(sys.argv) > 2 else 5
vals = collections.defaultdict(lambda: collections.defaultdict(list))  # kernel -> counter -> [per dispatch]
dur = collections.defaultdict(dict)
for f in sorted(glob.glob(f"{root}/pmc_*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("lpa::", "").replace("(anonymous namespace)::", "").replace("void ", "")
        k = re.sub(r"\(.*", "", k)
        key = (f, r["Dispatch_Id"])
        vals[k][r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
        dur[k][key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
out = []
for k, cs in vals.items():
    row = {}
    for c, lst in cs.items():
        lst.sort()
        v = [x for _, x in lst][-last:]
        row[c] = sum(v) / len(v)
    d = sorted(dur[k].values())
    out.append((k, row))
    print(f"== {k}")
    for c in sorted(row):
        print(f"   {c:32s} {row[c]:.4g}")
    g = row.get
    if g("SQ_WAVE_CYCLES"):
        print(f"   wait_any/wave_cycles {g('SQ_WAIT_ANY', 0) / g('SQ_WAVE_CYCLES'):.3f}  "
              f"wait_inst/wave {g('SQ_WAIT_INST_ANY', 0) / g('SQ_WAVE_CYCLES'):.3f}  "
              f"active/wave {g('SQ_ACTIVE_INST_ANY', 0) / g('SQ_WAVE_CYCLES'):.3f}")
    if g("SQ_LDS_IDX_ACTIVE"):
        print(f"   lds bank conflict ratio {g('SQ_LDS_BANK_CONFLICT', 0) / g('SQ_LDS_IDX_ACTIVE'):.3f}")
    if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum") is not None:
        print(f"   L2 hit rate {g('TCC_HIT_sum') / (g('TCC_HIT_sum') + g('TCC_MISS_sum')):.3f}")
    if g("FETCH_SIZE") is not None:
        print(f"   FETCH {g('FETCH_SIZE') * 1024 / 1e9:.3f} GB  WRITE {g('WRITE_SIZE', 0) * 1024 / 1e9:.3f} GB")

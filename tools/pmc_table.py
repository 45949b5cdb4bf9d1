"""Per-dispatch PMC table from rocprofv3 --pmc passes: one line per (kernel, dispatch
ordinal), counters of every pass side by side (passes run the same program, so the
n-th dispatch of a kernel is the same launch in every pass).

    python tools/pmc_table.py gpurun_out/pmcA   (reads gpurun_out/pmcA_*/run_counter_collection.csv)
"""
import collections
import csv
import glob
import re
import sys

prefix = sys.argv[1]
data = collections.defaultdict(dict)   # (kernel, ordinal) -> counter -> value
dur = {}
for f in sorted(glob.glob(f"{prefix}_*/run_counter_collection.csv")):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        m = re.search(r'(k_[A-Za-z0-9_]+(<[^>]*>)?)', r["Kernel_Name"])
        k = m.group(1) if m else r["Kernel_Name"][:30]
        per[(k, int(r["Dispatch_Id"]))][r["Counter_Name"]] = float(r["Counter_Value"])
        per[(k, int(r["Dispatch_Id"]))]["_ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    ords = collections.Counter()
    for (k, did) in sorted(per, key=lambda x: x[1]):
        ords[k] += 1
        data[(k, ords[k])].update(per[(k, did)])
for (k, o), c in sorted(data.items(), key=lambda x: (x[0][0], x[0][1])):
    parts = [f"{k:22s} #{o:<2d} {c.get('_ms', 0):7.3f}ms"]
    if "FETCH_SIZE" in c:
        parts.append(f"fetch {c['FETCH_SIZE'] * 1024 / 1e9 * 2:6.3f}GB(x2)")
    if "WRITE_SIZE" in c:
        parts.append(f"write {c['WRITE_SIZE'] * 1024 / 1e9:6.3f}GB")
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        parts.append(f"L2hit {c['TCC_HIT_sum'] / max(1, c['TCC_HIT_sum'] + c['TCC_MISS_sum']):.3f}")
    if c.get("SQ_WAVE_CYCLES"):
        wc = c["SQ_WAVE_CYCLES"]
        parts.append(f"waitany {c.get('SQ_WAIT_ANY', 0) / wc:.2f} waitinst {c.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} "
                     f"active {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} waves {c.get('SQ_WAVES', 0):.0f} "
                     f"valu {c.get('SQ_INSTS_VALU', 0):.3g} lds {c.get('SQ_INSTS_LDS', 0):.3g}")
    print("  ".join(parts))

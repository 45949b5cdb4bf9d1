"""Per-launch HBM traffic of the measured labelPropagation(10) call (the second call of
tools/pmc_workload5.py) from the tools/pmc_r05.sh passes, per superstep: superstep t ends with its refresh -- the t-th k_giant_pick of the call and
the rebuild launches right after it.  Summaries for the kernels with a byte model:
  k_code_rebuild     the giant-code refresh (round 5): col 4 B/arc, a 2-bit code per arc
                     of the coded rows (above 64 or 8 arcs), a 4-B label per arc of the others, the code
                     array (1/4 B per slot) and the label vector (4 B per slot) once
  k_code_build       each label once (4 B/slot) + its 2-bit code (1/4 B/slot)
  k_al_rebuild_hot   col 4 B/arc + al 4 B/arc + each label once (4 B/vertex)
  k_first_runs       al0 4 B/arc + row-start bits 1/8 B/arc + a label per row
Read factor: the round-2 calibration (4 B/lane streams read FETCH_SIZE = half the bytes).
    python tools/pmc_r05.py gpurun_out/<TAG> <config>  > traffic.json
"""
import csv
import glob
import json
import os
import re
import sys

pre, cfg = sys.argv[1], sys.argv[2]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cal = json.load(open(os.path.join(ROOT, "profiles", "r02", "traffic", "pmc_traffic.json")))["calibration"]
rf, wf = cal["read_factor"], cal["write_factor"]


def launches(d, counter):
    out = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            m = re.search(r"(k_[A-Za-z0-9_]+(<[^>]*>)?)", r["Kernel_Name"])
            out.append((int(r["Dispatch_Id"]), m.group(1) if m else r["Kernel_Name"], 1024.0 * float(r["Counter_Value"])))
    out.sort()
    return out


info = json.load(open(f"{pre}_info.json"))
A, V = info["arcs"], info["V"]
bins = list(info["bin_arcs"].values())
# arcs of the coded rows: above 64 arcs on a label vector of <= 64 MB, else above 8 (lpa_build)
p64 = sum(bins[:5]) if 4 * info["slice"] <= 64 << 20 else sum(bins[:8])
F = launches(f"{pre}_fetch", "FETCH_SIZE")
W = launches(f"{pre}_write", "WRITE_SIZE")


def by_superstep(L):
    """the measured call's launches -> {superstep: {kernel: bytes}}; a superstep ends with
    its refresh: its k_giant_pick and the rebuild launches right after it"""
    firsts = [i for i, (_, k, _) in enumerate(L) if k == "k_first_runs"]
    seg = L[firsts[1]:] if len(firsts) > 1 else L
    out, t, in_refresh = {}, 1, False
    for _, k, b in seg:
        if in_refresh and k.split("<")[0] not in ("k_al_rebuild_hot", "k_code_rebuild", "k_code_build"):
            t += 1
            in_refresh = False
        out.setdefault(t, {}).setdefault(k, 0.0)
        out[t][k] += b
        if k == "k_giant_pick":
            in_refresh = True
    return out


fs, ws = by_superstep(F), by_superstep(W)
model = {
    "k_code_rebuild": (4 * A + p64 // 4 + 4 * (A - p64) + V // 4 + 4 * V,
                       "col 4 B/arc + 2-bit code per arc (the coded rows) + label 4 B/arc (the others) + "
                       "the code array (1/4 B/slot) and the label vector (4 B/slot) once"),
    "k_code_build": (4 * V + V // 4, "each label once + its 2-bit code"),
    "k_al_rebuild_hot": (8 * A + 4 * V, "col 4 B/arc + al 4 B/arc + each label once (4 B/vertex)"),
    "k_first_runs": (4 * A + A // 8 + 4 * V, "al0 4 B/arc + row-start bits 1/8 B/arc + a label per row"),
}
rows = {}
for t in sorted(fs):
    for k, fb in fs[t].items():
        wb = ws.get(t, {}).get(k, 0.0)
        e = {"fetch_bytes": round(rf * fb), "write_bytes": round(wf * wb), "traffic_bytes": round(rf * fb + wf * wb)}
        kb = k.split("<")[0]
        if kb in model and e["traffic_bytes"] > 0.2 * model[kb][0]:   # a launch that did the work
            e["algorithmic_bytes"] = model[kb][0]
            e["traffic_over_algorithmic"] = round(e["traffic_bytes"] / model[kb][0], 3)
            e["algorithmic_note"] = model[kb][1]
        rows.setdefault(k, {})[f"superstep_{t}"] = e
print(json.dumps({"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes (tools/pmc_r05.sh, "
                            "tools/pmc_workload5.py), the measured (second) labelPropagation(10) call",
                  "config": cfg, "read_factor": rf, "write_factor": wf, "arcs": A, "vertices": V,
                  "code_range_arcs": p64, "per_superstep": rows}, indent=1))

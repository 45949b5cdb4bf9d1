"""Per-launch HBM traffic from the pmc_r03.sh passes (C3).

Launch order (tools/pmc_workload3.py): calls 0 and 1 on the shipped schedule, call 2
with the frontier off.  Reported:
  k_al_rebuild_hot  the rebuilding launch of superstep 2 of call 1 (the one in the
                    timed window: bits mode), and that of superstep 1 (labels mode)
  k_lpa_units       call 2's supersteps 2..10 (every unit streamed)
Read factor: the round-2 calibration (4 B/lane streams read FETCH_SIZE = half the bytes).
    python tools/pmc_r03.py gpurun_out/<TAG>  > traffic.json
"""
import csv
import glob
import json
import os
import re
import sys

pre = sys.argv[1]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cal = json.load(open(os.path.join(ROOT, "profiles", "r02", "traffic", "pmc_traffic.json")))["calibration"]
rf, wf = cal["read_factor"], cal["write_factor"]


def per_kernel(d, counter):
    """kernel -> [(dispatch id, bytes)] in dispatch order"""
    out = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            m = re.search(r"(k_[A-Za-z0-9_]+)", r["Kernel_Name"])
            k = m.group(1) if m else r["Kernel_Name"]
            out.setdefault(k, []).append((int(r["Dispatch_Id"]), 1024.0 * float(r["Counter_Value"])))
    for k in out:
        out[k].sort()
    return out


info = json.load(open(f"{pre}_info.json"))
A = info["arcs"]
lf = per_kernel(f"{pre}_pmc_lib_fetch", "FETCH_SIZE")
lw = per_kernel(f"{pre}_pmc_lib_write", "WRITE_SIZE")


def calls(d):
    """dispatch-id boundaries of the three calls: each starts with its k_first_runs"""
    return [i for i, _ in d["k_first_runs"]] + [1 << 62]


def in_call(d, name, c, pred=lambda v: True):
    b = calls(d)
    return [k for k, (i, v) in enumerate(d[name]) if b[c] <= i < b[c + 1] and pred(v)]


def entry(name, idx, algo, note):
    f, w = lf[name], lw[name]
    fb = rf * sum(f[i][1] for i in idx) / len(idx)
    wb = wf * sum(w[i][1] for i in idx) / len(idx)
    return {"launches": len(idx), "fetch_bytes": round(fb), "write_bytes": round(wb), "traffic_bytes": round(fb + wb),
            "algorithmic_bytes": algo, "traffic_over_algorithmic": round((fb + wb) / algo, 3), "algorithmic_note": note}


res = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes (tools/pmc_r03.sh, tools/pmc_workload3.py)",
       "read_factor": rf, "write_factor": wf}
algo_rb = 8 * A + 4 * info["V"]
note = "col read 4 B/arc + al write 4 B/arc + each label once (4 B/vertex)"
big = in_call(lf, "k_al_rebuild_hot", 1, lambda v: v * rf > 1e9)   # rebuilding launches of call 1
res["k_al_rebuild_hot"] = entry("k_al_rebuild_hot", big[1:2], algo_rb, note + "; superstep 2 (bits mode, timed window)")
res["k_al_rebuild_hot_superstep1"] = entry("k_al_rebuild_hot", big[0:1], algo_rb, note + "; superstep 1 (labels mode, untimed)")
u = in_call(lf, "k_lpa_units", 2)
res["k_lpa_units"] = entry("k_lpa_units", u[1:],
                           4 * info["bin_arcs"]["seg"] + 16 * info["segments"] + 4 * info["bin_vertices"]["seg"],
                           "al 4 B/arc + 16 B/unit + 4 B/row; call 2 (frontier off), every launch after its first")
ab = in_call(lf, "k_abits_pass", 1) if "k_abits_pass" in lf else []
if ab:
    na = A - info["bin_arcs"]["seg"]
    res["k_abits_pass"] = entry("k_abits_pass", ab, 4 * na + na // 8,
                                "al 4 B/arc read + 1 bit/arc written over the rows below the hubs; superstep 4")
fr = in_call(lf, "k_first_runs", 1)
if fr:
    S = info["slice"]
    res["k_first_runs"] = entry("k_first_runs", fr, 4 * A + A // 8 + 4 * S,
                                "al0 4 B/arc + row-start bits 1/8 B/arc + the label of every row (4 B); "
                                "superstep 1 (round 4: the 1-bit row-start map replaced crow, 4 B/arc)")
print(json.dumps(res, indent=1))

"""Per-launch HBM traffic from the pmc_r02.sh passes.

Calibration: mb_rebuild's k_floor streams exactly 4 B/arc in (col) and 4 B/arc out
(al), 4 B per lane, non-temporal: the ratio of its FETCH_SIZE to those bytes is the
read-counter factor for this access width (the guide's 1/2 holds for 16 B/lane).
Library launches (tools/pmc_workload.py, C3, frontier off, second labelPropagation(10)
call): k_lpa_units supersteps 2..10, every full k_al_rebuild_hot (fetch > 1 GB).
    python tools/pmc_r02.py gpurun_out/<TAG>  > traffic.json
"""
import csv
import glob
import json
import re
import sys

pre = sys.argv[1]


def per_kernel(d, counter):
    out = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            m = re.search(r"(k_[A-Za-z0-9_]+(<[^>]*>)?)", r["Kernel_Name"])
            k = m.group(1) if m else r["Kernel_Name"]
            out.setdefault(k, []).append((int(r["Dispatch_Id"]), 1024.0 * float(r["Counter_Value"])))
    for k in out:
        out[k].sort()
    return out


info = json.load(open(f"{pre}_info.json"))
A = info["arcs"]
arcs_mb = A // 512 * 512  # mb_rebuild uses the C3 degree sequence rounded to 512
mf, mw = per_kernel(f"{pre}_pmc_mb_fetch", "FETCH_SIZE"), per_kernel(f"{pre}_pmc_mb_write", "WRITE_SIZE")
fl_f = [v for _, v in mf["k_floor"]]
fl_w = [v for _, v in mw["k_floor"]]
read_factor = 4.0 * arcs_mb / (sum(fl_f) / len(fl_f))
write_factor = 4.0 * arcs_mb / (sum(fl_w) / len(fl_w))
res = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes (tools/pmc_r02.sh)",
       "calibration": {"kernel": "mb_rebuild k_floor (4 B/lane non-temporal stream, 4 B/arc in + 4 B/arc out)",
                       "expected_bytes_each_way": 4 * arcs_mb,
                       "fetch_counter_bytes": round(sum(fl_f) / len(fl_f)),
                       "write_counter_bytes": round(sum(fl_w) / len(fl_w)),
                       "read_factor": round(read_factor, 3), "write_factor": round(write_factor, 3)}}
lf, lw = per_kernel(f"{pre}_pmc_lib_fetch", "FETCH_SIZE"), per_kernel(f"{pre}_pmc_lib_write", "WRITE_SIZE")


def merged(d, name):
    """dispatches of every template instance of kernel `name`, in dispatch order"""
    return [v for _, v in sorted(x for k, xs in d.items() if k.split("<")[0] == name for x in xs)]


def summarize(name, sel):
    f = merged(lf, name)
    w = merged(lw, name)
    idx = sel(f)
    if not idx:
        return None
    fb = read_factor * sum(f[i] for i in idx) / len(idx)
    wb = write_factor * sum(w[i] for i in idx) / len(idx) if len(w) == len(f) else None
    return {"launches": len(idx), "fetch_bytes": round(fb), "write_bytes": round(wb) if wb is not None else None,
            "traffic_bytes": round(fb + (wb or 0.0))}


# units: 20 launches (2 calls x 10 supersteps); the measured call's supersteps 2..10
res["k_lpa_units"] = summarize("k_lpa_units", lambda f: list(range(11, 20)) if len(f) >= 20 else [])
res["k_lpa_units"]["algorithmic_bytes"] = 4 * info["bin_arcs"]["seg"] + 16 * info["segments"] + 4 * info["bin_vertices"]["seg"]
res["k_al_rebuild_hot"] = summarize("k_al_rebuild_hot", lambda f: [i for i, v in enumerate(f) if v * read_factor > 1e9])
res["k_al_rebuild_hot"]["algorithmic_bytes"] = 8 * A + 4 * info["V"]
res["k_al_rebuild_hot"]["algorithmic_note"] = "col read 4 B/arc + al write 4 B/arc + each label once (4 B/vertex)"
print(json.dumps(res, indent=1))

"""Per-launch HBM traffic from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

bench.py launches k_lpa_units once per superstep: prime (1), warmup (W), timed (K),
warmup (W), breakdown (K).  The timed pass's K dispatches are averaged.  FETCH_SIZE
is in KiB and, on gfx950, reports half the bytes of a wide coalesced streaming read
(MI355X_MICROARCH.md, HBM section): doubled here.  The doubling is cross-checked on
k_diff, whose int4 streams read exactly 2 x 4 vpad bytes per launch.
    python tools/pmc_traffic.py <fetch dir> <write dir> <bench json> > traffic.json
"""
import csv
import glob
import json
import re
import sys


def per_kernel(d, counter):
    out = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            m = re.search(r"(k_[A-Za-z0-9_]+(<[^>]*>)?)", r["Kernel_Name"])
            k = m.group(1) if m else r["Kernel_Name"]
            out.setdefault(k, []).append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    for k in out:
        out[k].sort()
    return out


fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
write = per_kernel(sys.argv[2], "WRITE_SIZE")
bench = json.load(open(sys.argv[3]))
W, K = bench["warmup"], bench["steps"]
lo, hi = 1 + W, 1 + W + K  # timed dispatches of a once-per-superstep kernel
res = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), bench.py --no-cpu-baseline",
       "timed_dispatches": [lo, hi - 1]}
for k in sorted(fetch):
    f = [v for _, v in fetch.get(k, [])][lo:hi]
    w = [v for _, v in write.get(k, [])][lo:hi]
    if not f:
        continue
    fb = 2 * 1024 * sum(f) / len(f)
    wb = 1024 * sum(w) / len(w) if w else 0.0
    res[k] = {"fetch_bytes": round(fb), "write_bytes": round(wb), "traffic_bytes": round(fb + wb),
              "fetch_bytes_per_superstep": [round(2 * 1024 * v) for v in f],
              "write_bytes_per_superstep": [round(1024 * v) for v in w]}
vpad = bench["config"]["vertices"]
if "k_diff" in res:
    res["k_diff"]["expected_read_bytes"] = 2 * 4 * vpad
print(json.dumps(res, indent=1))

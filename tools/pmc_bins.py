"""Per-bin counter table from tools/pmc_bins.sh's three rocprofv3 --pmc passes.

Dispatches of one kernel line up across passes by ordinal (same program, same launch
sequence).  Each kernel's dispatches are split into "dense" (duration >= half the
kernel's longest dispatch: the label-dense supersteps after L0) and "steady" (the rest:
converged supersteps); counters are averaged per group.
  GB/s      = (2 x FETCH_SIZE + WRITE_SIZE) / duration  (FETCH doubled for gfx950,
              MI355X_MICROARCH.md HBM section; durations are the --pmc runs' own)
  ldsconf   = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE  (extra cycles per LDS cycle)
  waves/CU  = 4 SQ_WAVE_CYCLES (quad-cycles) / (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs)
              = mean resident waves per CU while the kernel runs (cap 32)
  theo      = waves/CU the resources allow: min(32, 4 x 512 / VGPRs, LDS blocks x waves/block)
    python tools/pmc_bins.py "gpurun_out/bins_[0-9]*" > table.txt
"""
import collections
import csv
import glob
import re
import statistics
import sys

rows = collections.defaultdict(dict)       # (kernel, ordinal) -> counter -> value
dur = collections.defaultdict(list)        # (kernel, ordinal) -> [ms per pass]
res = {}                                   # kernel -> (vgpr, lds bytes, wg size)
for d in sorted(glob.glob(sys.argv[1])):
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(dict)  # kernel -> dispatch id -> row values
        for r in csv.DictReader(open(f)):
            m = re.search(r"(k_[A-Za-z0-9_]+(<[^>]*>)?)", r["Kernel_Name"])
            k = m.group(1) if m else r["Kernel_Name"][:30]
            did = int(r["Dispatch_Id"])
            e = per[k].setdefault(did, {"ms": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6})
            e[r["Counter_Name"]] = float(r["Counter_Value"])
            res[k] = (int(r["VGPR_Count"]) + int(r["Accum_VGPR_Count"]), int(r["LDS_Block_Size"]),
                      int(r["Workgroup_Size"]))
        for k, ds in per.items():
            for i, did in enumerate(sorted(ds)):
                e = ds[did]
                dur[(k, i)].append(e.pop("ms"))
                rows[(k, i)].update(e)


def theo(k):
    vgpr, lds, wg = res[k]
    vg = max(8, -(-vgpr // 8) * 8)
    w = min(32, 4 * min(8, 512 // vg))
    if lds:
        w = min(w, (163840 // lds) * max(1, wg // 64))
    return w


kernels = sorted({k for k, _ in rows})
hdr = (f"{'kernel':32s} {'group':6s} {'n':>3s} {'ms':>7s} {'fetchGB':>8s} {'writeGB':>8s} {'GB/s':>7s} "
       f"{'L2hit':>6s} {'ldsconf':>7s} {'waves/CU':>8s} {'theo':>4s} {'vgpr':>4s} {'ldsKB':>6s}")
print(hdr)
for k in kernels:
    ords = sorted(i for kk, i in rows if kk == k)
    ms = {i: statistics.median(dur[(k, i)]) for i in ords}
    mx = max(ms.values())
    groups = {"dense": [i for i in ords if ms[i] >= 0.5 * mx], "steady": [i for i in ords if ms[i] < 0.5 * mx]}
    for gname, sel in groups.items():
        if not sel or mx < 0.003:
            continue
        avg = lambda c: statistics.mean(rows[(k, i)].get(c, 0.0) for i in sel)
        t = statistics.mean(ms[i] for i in sel)
        fetch = 2 * avg("FETCH_SIZE") * 1024 / 1e9
        write = avg("WRITE_SIZE") * 1024 / 1e9
        gbs = (fetch + write) / (t / 1e3) if t > 0 else 0.0
        hit, miss = avg("TCC_HIT_sum"), avg("TCC_MISS_sum")
        l2 = hit / (hit + miss) if hit + miss else float("nan")
        lia = avg("SQ_LDS_IDX_ACTIVE")
        conf = avg("SQ_LDS_BANK_CONFLICT") / lia if lia else float("nan")
        gui = avg("GRBM_GUI_ACTIVE")
        wpc = 4 * avg("SQ_WAVE_CYCLES") / (gui / 8 * 256) if gui else float("nan")
        vgpr, lds, _ = res[k]
        print(f"{k:32s} {gname:6s} {len(sel):3d} {t:7.3f} {fetch:8.3f} {write:8.3f} {gbs:7.0f} "
              f"{l2:6.3f} {conf:7.3f} {wpc:8.1f} {theo(k):4d} {vgpr:4d} {lds / 1024:6.1f}")

"""Per-kernel SQ/GRBM table of the last N supersteps of tools/pmc_dense.sh.

    python tools/pmc_dense.py gpurun_out/<TAG> N

Supersteps start at k_frontier_lists.  Columns: duration (ms, trace timestamps),
waves, mean resident waves per CU (SQ_WAVE_CYCLES / kernel cycles / 256 CUs; both
in the SQ's quad-cycle units vs GRBM cycles / 8 XCDs), the share of wave cycles
parked on a counter (wait), stalled at issue (istall), issuing (act) and issuing
LDS (lds), LDS bank-conflict cycles per LDS-array cycle (conf), and instructions per
wave (valu / salu / lds / vmem), HBM GB/s from FETCH_SIZE x 2 + WRITE_SIZE over the
kernel's duration, and the L2 hit rate.
"""
import csv
import glob
import re
import sys
from collections import defaultdict

pre, N = sys.argv[1], int(sys.argv[2])


def short(n):
    m = re.search(r"(k_[A-Za-z0-9_]+(<[^>]*>)?)", n)
    return m.group(1) if m else n[:28]


disp = defaultdict(dict)   # (pass, dispatch) -> counters
meta = {}
for k, d in enumerate(sorted(glob.glob(f"{pre}_pmc*/"))):
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            key = (k, int(r["Dispatch_Id"]))
            disp[key][r["Counter_Name"]] = disp[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            if key not in meta:
                t = (int(r.get("End_Timestamp", 0) or 0) - int(r.get("Start_Timestamp", 0) or 0)) / 1e6
                meta[key] = (short(r["Kernel_Name"]), t, r.get("LDS_Block_Size", ""), r.get("VGPR_Count", ""))

def gbs(c, ms):
    """FETCH_SIZE (KB, doubled: the gfx950 correction for wide streaming reads, calibrated
    in profiles/r02/traffic for 4 B/lane streams too) + WRITE_SIZE (KB) per ms."""
    kb = 2.0 * c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0)
    return kb * 1024 / (ms * 1e-3) / 1e9 if ms > 0 else 0.0


def hit(c):
    h, m = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
    return h / (h + m) if h + m else 0.0


passes = sorted({k for k, _ in disp})
seqs = []
for p in passes:
    ids = sorted(i for (k, i) in disp if k == p)
    steps = []
    for i in ids:
        name = meta[(p, i)][0]
        if name == "k_frontier_lists":
            steps.append([])
        if steps:
            steps[-1].append((p, i))
    seqs.append(steps[-N:])

hdr = (f"{'ss':>2} {'kernel':32s} {'ms':>7} {'waves':>8} {'w/CU':>5} {'wait':>5} {'istl':>5} {'act':>5} {'lds':>5} "
       f"{'conf':>5} {'valu':>7} {'salu':>7} {'ldsI':>6} {'vmem':>6} {'lds_KB':>6} {'vgpr':>4} {'HBM_GB/s':>8} {'L2hit':>5}")
print(hdr)
for t in range(N):
    rows0 = seqs[0][t]
    others = [s[t] for s in seqs[1:]]
    for j, key in enumerate(rows0):
        c = dict(disp[key])
        for o in others:
            if j < len(o) and meta[o[j]][0] == meta[key][0]:
                c.update(disp[o[j]])
        name, ms, lds, vgpr = meta[key]
        if ms < 0.02:
            continue
        W = c.get("SQ_WAVES", 0) or 1
        wc = c.get("SQ_WAVE_CYCLES", 0)
        cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8.0
        occ = wc * 4 / cyc / 256 if cyc else 0
        f = lambda x: c.get(x, 0) / wc if wc else 0
        conf = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"] if c.get("SQ_LDS_IDX_ACTIVE") else 0
        print(f"{t + 1:>2} {name:32s} {ms:7.3f} {W:8.0f} {occ:5.1f} {f('SQ_WAIT_ANY'):5.2f} {f('SQ_WAIT_INST_ANY'):5.2f} "
              f"{f('SQ_ACTIVE_INST_ANY'):5.2f} {f('SQ_ACTIVE_INST_LDS'):5.2f} {conf:5.2f} "
              f"{c.get('SQ_INSTS_VALU', 0) / W:7.0f} {c.get('SQ_INSTS_SALU', 0) / W:7.0f} "
              f"{c.get('SQ_INSTS_LDS', 0) / W:6.0f} {c.get('SQ_INSTS_VMEM_RD', 0) / W:6.0f} {lds:>6} {vgpr:>4} "
              f"{gbs(c, ms):8.0f} {hit(c):5.2f}")

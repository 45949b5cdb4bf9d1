"""Offline workload analysis of config C3 (R-MAT scale 24) on the CPU oracle:
per superstep, per degree bin: rows, arcs, distinct neighbour labels (the hash
work of the tally) and the vertices / arcs whose label changed (the al refresh).

    python tools/analyse_c3.py [scale] [steps]
"""
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from oracle import oracle  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
V = 1 << scale
t0 = time.time()
s, d = oracle.gen_rmat(scale, 16, 1, True)
rp, col = oracle.build_csr(V, s, d)
del s, d
deg = np.diff(rp)
print(f"built scale {scale}: {col.size} arcs, max deg {deg.max()} ({time.time() - t0:.0f}s)", flush=True)
edges = [0, 1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 4096, 32768, 1 << 40]
binof = np.searchsorted(np.array(edges[1:]), deg, side="left")
for b in range(len(edges) - 1):
    sel = binof == b
    print(f"bin ({edges[b]},{edges[b+1]}]: rows {sel.sum()}, arcs {deg[sel].sum()} "
          f"({deg[sel].sum() / col.size:.3f})")
big = np.nonzero(deg > 64)[0]
rows_big = np.repeat(big, deg[big]).astype(np.int64)
pos_big = np.concatenate([np.arange(rp[v], rp[v + 1]) for v in big[:0]]) if False else None
# arc ranges of the big rows (contiguous per row)
mask = np.zeros(col.size, dtype=bool)
starts, ends = rp[big], rp[big + 1]
idx = np.concatenate([np.arange(a, b) for a, b in zip(starts, ends)])
colb = col[idx]
L = np.arange(V, dtype=np.int32)
for t in range(1, steps + 1):
    lab = L[colb].astype(np.int64)
    key = (rows_big << 32) | lab
    key.sort()
    newk = np.ones(key.size, dtype=bool)
    newk[1:] = key[1:] != key[:-1]
    dist_row = np.bincount((key[newk] >> 32).astype(np.int64), minlength=V)
    for lo, hi in [(64, 512), (512, 4096), (4096, 32768), (32768, 1 << 40)]:
        sel = (deg > lo) & (deg <= hi)
        if sel.any():
            dr = dist_row[sel]
            print(f"  step {t} deg ({lo},{hi}]: rows {sel.sum()}, distinct sum {dr.sum()} "
                  f"(/arcs {dr.sum() / deg[sel].sum():.3f}), max {dr.max()}, "
                  f"rows with distinct>6144: {(dr > 6144).sum()}, >2048: {(dr > 2048).sum()}")
    Ln = oracle.superstep_csr(rp, col, L)
    chg = Ln != L
    print(f"step {t}: changed {chg.sum()} vertices, dirty arcs {deg[chg].sum()} "
          f"({deg[chg].sum() / col.size:.3f}), distinct labels {np.unique(Ln).size} "
          f"({time.time() - t0:.0f}s)", flush=True)
    L = Ln

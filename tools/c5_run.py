"""Config C5 (BASELINE.json configs[4]) on ONE GPU: Chung-Lu power law,
exponent 2.1, 40 M vertices / 1.4 B edges (2.8 B arcs), expected maximum degree 1.25 M,
seed 7, maxIter 10.  The survey quotes C5 at 8 GPUs; one MI355X holds it (288 GB), which
stresses the hub-combine spill path (bucket partition + sub-bucket passes) hardest.
Prints one JSON line: GTEPS over supersteps 2..10 (wall clock, no events), per-superstep
times, degree facts, community count, and (with --oracle) bit-exactness vs the CPU oracle.

    python tools/c5_run.py [--V 40000000] [--m 1400000000] [--max-deg 1.25e6] [--oracle]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import graphframes_amd as gfa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--V", type=int, default=40_000_000)
ap.add_argument("--m", type=int, default=1_400_000_000)
ap.add_argument("--max-deg", type=float, default=1.25e6)
ap.add_argument("--seed", type=int, default=7)
ap.add_argument("--oracle", action="store_true")
a = ap.parse_args()

t0 = time.perf_counter()
s, d = gfa.gen_chunglu(a.V, a.m, 2.1, a.max_deg, seed=a.seed)
torch.cuda.synchronize()
t_gen = time.perf_counter() - t0
t0 = time.perf_counter()
g = gfa.Graph(s, d, a.V)
t_build = time.perf_counter() - t0
deg = g.degrees()
free, total = torch.cuda.mem_get_info()
print(f"built: gen {t_gen:.1f}s build {t_build:.1f}s max deg {int(deg.max())} "
      f"HBM used {(total - free) / 2**30:.1f} GiB", file=sys.stderr, flush=True)
src_np = dst_np = None
if a.oracle:
    src_np, dst_np = s.cpu().numpy(), d.cpu().numpy()
del s, d
torch.cuda.empty_cache()
g.step(1)
g.reset()
g.step(1)
torch.cuda.synchronize()
t0 = time.perf_counter()
g.step(9)
torch.cuda.synchronize()
t = time.perf_counter() - t0
lab = g.labels()
g.reset()
g.step(1)
st = g.step(9, stats=True)
info = g.info()
out = {
    "config": f"C5 Chung-Lu gamma 2.1, V {a.V}, m {a.m}, expected max degree {a.max_deg:g}, seed {a.seed}, "
              f"maxIter 10, 1 GPU",
    "gteps": round(a.m * 9 / t / 1e9, 2), "ms_per_superstep": round(t * 1e3 / 9, 4),
    "iter_ms": [round(x, 4) for x in st["iter_ms"]],
    "arcs": info["arcs"], "max_degree": int(deg.max()), "isolated": int((deg == 0).sum()),
    "rows_deg_gt_100k": int((deg > 100_000).sum()),
    "communities": int(np.unique(lab).size), "gen_s": round(t_gen, 1), "build_s": round(t_build, 1),
    "hbm_used_gib": round((total - free) / 2**30, 1),
}
g.close()
if a.oracle:
    from oracle import oracle
    t0 = time.perf_counter()
    ref = oracle.lpa(a.V, src_np, dst_np, 10)
    out["oracle_s"] = round(time.perf_counter() - t0, 1)
    out["bit_exact_vs_oracle"] = bool(np.array_equal(lab, ref))
print(json.dumps(out), flush=True)

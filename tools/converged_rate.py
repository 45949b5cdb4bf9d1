"""Converged-superstep rate on C3: wall time of N supersteps after the labels
settle (host launch overhead vs device time), with and without captured graphs.

    python tools/converged_rate.py [--scale 24] [--n 100]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import graphframes_amd as gfa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scale", type=int, default=24)
ap.add_argument("--n", type=int, default=100)
a = ap.parse_args()
s, d = gfa.gen_rmat(a.scale, 16, seed=1)
g = gfa.Graph(s, d, 1 << a.scale)
del s, d
for frontier in (1, 0):
    g.set_frontier(bool(frontier))
    g.reset()
    g.step(10)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.step(a.n)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    st = g.step(20, stats=True)
    dev = sorted(st["iter_ms"])[10]
    print(f"frontier={frontier} graphs={os.environ.get('LPA_GRAPHS', '1')}: wall {t * 1e3 / a.n:.4f} ms/superstep, "
          f"device median {dev:.4f} ms", flush=True)
g.close()

"""Config C2 on one GPU: planted-partition SBM, 1 M vertices / 20 M
edges / 100 blocks, maxIter 10.  Prints one JSON line: GTEPS over supersteps 2..10
(wall clock, no events), per-superstep times, community count, NMI / ARI vs the planted
blocks, and bit-exactness vs the CPU oracle."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from sklearn.metrics import adjusted_rand_score, normalized_mutual_info_score  # noqa: E402

import graphframes_amd as gfa  # noqa: E402
from oracle import oracle  # noqa: E402

V, B, m = 1_000_000, 100, 20_000_000
s, d = gfa.gen_sbm(V, B, m)
g = gfa.Graph(s, d, V)
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
ref = oracle.lpa(V, s.cpu().numpy(), d.cpu().numpy(), 10)
truth = np.minimum(np.arange(V) // (V // B), B - 1)
print(json.dumps({
    "config": "C2 SBM 1M/20M/100 blocks, maxIter 10", "gteps": round(m * 9 / t / 1e9, 2),
    "ms_per_superstep": round(t * 1e3 / 9, 4), "iter_ms": [round(x, 4) for x in st["iter_ms"]],
    "communities": int(np.unique(lab).size), "nmi": round(float(normalized_mutual_info_score(truth, lab)), 4),
    "ari": round(float(adjusted_rand_score(truth, lab)), 4), "bit_exact_vs_oracle": bool(np.array_equal(lab, ref))}))
g.close()

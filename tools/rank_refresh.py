"""Per-rank time of the refresh after superstep 1 (the giant-code refresh, or the
labels-mode rebuild when it is not taken) against the single-GPU handle's (VERDICT r05
item 1: "the per-rank superstep-1 refresh time at C4/P=8 next to the P = 1 figure").

Run under `rocprofv3 --kernel-trace` and read with tools/refresh_trace.py: every kernel
then has its standalone duration, because the P caller-driven ranks are stepped and
refreshed ONE AFTER ANOTHER from this thread (lpa_step, then the full exchange
lpa_exchange_put, whose refresh is the one the in-library exchange runs after
superstep 1).  Order of the refresh groups in the trace: REPS single-GPU refreshes, then
REPS x P rank refreshes (rank order within a repetition).  Prints one JSON line (the
code_refresh flag of every handle, labels checked against the single-GPU handle).

    rocprofv3 --kernel-trace --output-format csv -d DIR -- python3 tools/rank_refresh.py [C4] [P]
"""
import json
import sys

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
import graphframes_amd as gfa  # noqa: E402
import torch  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C4"
P = int(sys.argv[2]) if len(sys.argv) > 2 else 8
REPS = 3
src, dst, V = bench.make_edges(gfa, bench.CONFIGS[name], 0)

with gfa.Graph(src, dst, V) as g:
    for _ in range(REPS):
        g.reset()
        g.step(1)
    one_code = g.info()["code_refresh"]
    g.step(1)
    ref2 = g.labels()   # superstep 2 (read from the refreshed arc labels / codes)
torch.cuda.synchronize()
torch.cuda.empty_cache()

ranks = [gfa.Graph(src, dst, V, rank=r, nranks=P) for r in range(P)]
del src, dst
torch.cuda.empty_cache()
codes = []
for _ in range(REPS):
    for g in ranks:
        g.reset()
        g.step(1)
    full = np.concatenate([g.exchange_get() for g in ranks])
    for g in ranks:
        g.exchange_put(full)
    codes.append([g.info()["code_refresh"] for g in ranks])
# one more superstep on every rank, exchanged: the replicas equal the single-GPU L2
for g in ranks:
    g.step(1)
full = np.concatenate([g.exchange_get() for g in ranks])
for g in ranks:
    g.exchange_put(full)
ok = all(np.array_equal(g.labels(), ref2) for g in ranks)
for g in ranks:
    g.close()
print(json.dumps(dict(config=name, P=P, reps=REPS, single_code_refresh=one_code, rank_code_refresh=codes,
                      superstep2_equal_single_gpu=ok)), flush=True)

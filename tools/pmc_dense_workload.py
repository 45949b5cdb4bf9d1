"""Workload for tools/pmc_dense.sh: config C3 (or the one named), serialized
schedule (every tally kernel alone on the main stream, so each dispatch's counters
are its own), frontier on as shipped; labelPropagation supersteps 1..N twice, the
second pass is the measured one (dispatches are tagged by order in the trace).

    python tools/pmc_dense_workload.py [C3] [N]
"""
import sys

sys.path.insert(0, ".")
import bench  # noqa: E402
import graphframes_amd as gfa  # noqa: E402
import torch  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4
src, dst, V = bench.make_edges(gfa, bench.CONFIGS[name], 0)
g = gfa.Graph(src, dst, V)
del src, dst
torch.cuda.empty_cache()
g.set_serial(True)
for _ in range(2):
    g.reset()
    for t in range(n):
        g.step(1)
torch.cuda.synchronize()
g.close()

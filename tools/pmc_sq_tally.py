"""Workload for SQ counter passes over the superstep-2 tally kernels: CFG (C3 default),
two reset + step(2) calls.  python tools/pmc_sq_tally.py C3"""
import sys

sys.path.insert(0, ".")
import bench  # noqa: E402
import graphframes_amd as gfa  # noqa: E402
import torch  # noqa: E402

cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "C3"]
src, dst, V = bench.make_edges(gfa, cfg, 0)
g = gfa.Graph(src, dst, V)
del src, dst
torch.cuda.empty_cache()
for _ in range(2):
    g.reset()
    g.step(2)
torch.cuda.synchronize()
print(g.info())
g.close()

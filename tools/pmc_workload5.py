"""Workload for the round-5 PMC traffic passes (tools/pmc_r05.sh): one bench config,
one warm-up labelPropagation(10) call, then the measured call on the shipped schedule
(frontier on).  Writes the handle info for the byte model.

    python tools/pmc_workload5.py <C3|C4|C5> <info.json>
"""
import json
import sys

sys.path.insert(0, ".")
import bench  # noqa: E402
import graphframes_amd as gfa  # noqa: E402
import torch  # noqa: E402

cfg = bench.CONFIGS[sys.argv[1]]
src, dst, V = bench.make_edges(gfa, cfg, 0)
g = gfa.Graph(src, dst, V)
del src, dst
torch.cuda.empty_cache()
for _ in range(2):          # call 0 warms up, call 1 is the measured call
    g.reset()
    g.step(10)
torch.cuda.synchronize()
info = g.info()
json.dump({k: info[k] for k in ("V", "arcs", "slice", "segments", "hub_vertices", "bin_vertices", "bin_arcs")},
          open(sys.argv[2], "w"))
g.close()

"""Workload for the round-3 PMC traffic passes (tools/pmc_r03.sh): config C3, two
labelPropagation(10) calls on the shipped schedule (frontier on), then one call with
the frontier off (every superstep tallies every unit, so each k_lpa_units launch moves
its full algorithmic bytes).  Writes the handle info for the byte model.

    python tools/pmc_workload3.py <info.json>
"""
import json
import sys

sys.path.insert(0, ".")
import bench  # noqa: E402
import graphframes_amd as gfa  # noqa: E402
import torch  # noqa: E402

cfg = bench.CONFIGS["C3"]
src, dst, V = bench.make_edges(gfa, cfg, 0)
g = gfa.Graph(src, dst, V)
del src, dst
torch.cuda.empty_cache()
for _ in range(2):          # call 0 warms up, call 1 is the measured shipped call
    g.reset()
    g.step(10)
g.set_frontier(False)
g.reset()
g.step(10)                  # call 2: frontier off
torch.cuda.synchronize()
info = g.info()
json.dump({k: info[k] for k in ("V", "arcs", "slice", "segments", "hub_vertices", "bin_vertices", "bin_arcs")},
          open(sys.argv[1], "w"))
g.close()

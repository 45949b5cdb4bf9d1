"""Workload for the PMC traffic passes (tools/pmc_r02.sh): config C3, one
labelPropagation(10) with the frontier OFF (every superstep tallies every row, so
each k_lpa_units launch moves its full algorithmic bytes), after one untimed warm
call.  Writes the handle info (arcs, units, bins) for the byte model.

    python tools/pmc_workload.py <info.json>
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
g.set_frontier(False)
for _ in range(2):          # call 0 warms up, call 1 is the measured one
    g.reset()
    g.step(10)
torch.cuda.synchronize()
info = g.info()
json.dump({k: info[k] for k in ("V", "arcs", "slice", "segments", "hub_vertices", "bin_vertices", "bin_arcs")},
          open(sys.argv[1], "w"))
g.close()

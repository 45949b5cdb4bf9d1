"""Standalone (serialized) kernel times of each superstep 1..10 of one
labelPropagation(10) on a bench config, frontier on (as shipped) or off.

    python tools/superstep_breakdown.py [C3|C5|...] [--frontier-off]
"""
import json
import sys

sys.path.insert(0, ".")
import bench  # noqa: E402
import graphframes_amd as gfa  # noqa: E402
import torch  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else "C3"
cfg = bench.CONFIGS[cfg_name]
src, dst, V = bench.make_edges(gfa, cfg, 0)
g = gfa.Graph(src, dst, V)
del src, dst
torch.cuda.empty_cache()
info = g.info()
print(json.dumps({k: info[k] for k in ("arcs", "hub_vertices", "segments", "bin_vertices")}))
if "--frontier-off" in sys.argv:
    g.set_frontier(False)
g.set_serial(True)
for rep in range(2):
    g.reset()
    for t in range(1, 11):
        st = g.step(1, stats=True)
        if rep == 1:
            km = {k: round(v, 3) for k, v in st["kernel_ms"].items() if v >= 0.005}
            print(f"s{t} iter {st['iter_ms'][0]:.3f} ms  sum {sum(st['kernel_ms'].values()):.3f}  {km}", flush=True)
g.close()

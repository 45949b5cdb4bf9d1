"""Write a bench config's degree sequence (descending, int32) for mb_rebuild."""
import sys

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
import graphframes_amd as gfa  # noqa: E402

cfg = bench.CONFIGS[sys.argv[1]]
src, dst, V = bench.make_edges(gfa, cfg, 0)
with gfa.Graph(src, dst, V) as g:
    deg = g.degrees()
np.sort(deg)[::-1].astype(np.int32).tofile(sys.argv[2])
print(sys.argv[1], V, int(deg.sum()))

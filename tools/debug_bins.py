"""Which degree bins hold the vertices whose superstep-1 label differs from the golden fixture."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import graphframes_amd as gfa
z = np.load("tests/golden/r9_golden.npz")
V = z["ids"].size
with gfa.Graph(z["src"], z["dst"], V) as g:
    g.step(1)
    lab = g.labels()
    deg = g.degrees()
    print(g.info()["bin_vertices"])
bad = np.flatnonzero(lab != z["labels_iter"][0])
print("bad", bad.size, "degs", sorted(deg[bad].tolist())[:40])
print("got", lab[bad][:10], "want", z["labels_iter"][0][bad][:10])

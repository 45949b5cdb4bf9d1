import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import graphframes_amd as gfa
z = np.load("tests/golden/r9_golden.npz")
s, d, V = z["src"], z["dst"], z["ids"].size
deg = np.bincount(s, minlength=V) + np.bincount(d, minlength=V)
g = gfa.Graph(s, d, V)
print(g.info())
for t in range(3):
    g.step(1)
    lab = g.labels()
    exp = z["labels_iter"][t]
    bad = lab != exp
    print("step", t + 1, "bad", bad.sum())
    for lo, hi in ((0, 1), (1, 2), (2, 4), (4, 8), (8, 16), (16, 512), (512, 5000)):
        m = (deg > lo) & (deg <= hi)
        print(f"  deg ({lo},{hi}] n={m.sum()} bad={(bad & m).sum()}", "sample got", lab[m & bad][:5], "exp", exp[m & bad][:5], "ident?", (lab[m & bad][:5] == np.flatnonzero(m & bad)[:5]))

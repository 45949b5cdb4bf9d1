import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import graphframes_amd as gfa
z = np.load("tests/golden/r9_golden.npz")
s, d, V = z["src"], z["dst"], z["ids"].size
g = gfa.Graph(s, d, V)
g.step(1)
a = g.labels(); b = g.labels()
print("twice after step1:", (a != z["labels_iter"][0]).sum(), (b != z["labels_iter"][0]).sum())
lab = g.run(2)
print("run(2):", (lab != z["labels_iter"][1]).sum(), lab[:8])
lab = g.run(1)
print("run(1):", (lab != z["labels_iter"][0]).sum(), lab[:8])
g2 = gfa.Graph(s, d, V)
g2.step(2)
lab = g2.labels()
print("fresh step(2):", (lab != z["labels_iter"][1]).sum(), lab[:8])
import torch
out = torch.empty(V, dtype=torch.int32, device="cuda")
g2.labels(out); torch.cuda.synchronize()
print("device out:", (out.cpu().numpy() != z["labels_iter"][1]).sum())

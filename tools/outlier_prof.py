"""Outlier stage (Graphframes.py:92-137) on a bench config: the
maxIter=10 labels, then L1 and L2 twice each, wall time per call (host labels in,
host arrays out, as bench.py measures).  Run under rocprofv3 for the kernel / copy
split.

    python tools/outlier_prof.py [C3]
"""
import sys
import time

sys.path.insert(0, ".")
import bench  # noqa: E402
import graphframes_amd as gfa  # noqa: E402
import torch  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C3"
src, dst, V = bench.make_edges(gfa, bench.CONFIGS[name], 0)
t0 = time.perf_counter()
g = gfa.Graph(src, dst, V)
print(f"build {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
del src, dst
torch.cuda.empty_cache()
lab = g.run(10)
dlab = torch.from_numpy(lab).cuda()
for mode, labels_in, form in (("L1", lab, "host"), ("L1", lab, "host"), ("L1", dlab, "device"),
                              ("L1", dlab, "device"), ("L2", lab, "host"), ("L2", lab, "host"),
                              ("L2", dlab, "device"), ("L2", dlab, "device")):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = g.outlier(labels_in, mode, sub_iter=5)
    torch.cuda.synchronize()
    print(f"{mode} {form} {1e3 * (time.perf_counter() - t0):.1f} ms flagged {int(r['flags'].sum())} "
          f"groups {r['summary']['n_groups']}", flush=True)
g.close()

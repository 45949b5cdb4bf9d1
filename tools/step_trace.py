"""Workload for a HIP API + kernel trace of the timed call (supersteps 2..10): CFG (C3
default), three reset / step(1) / step(9) rounds after a warm-up."""
import sys
import time

sys.path.insert(0, ".")
import bench  # noqa: E402
import graphframes_amd as gfa  # noqa: E402
import torch  # noqa: E402

cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "C3"]
src, dst, V = bench.make_edges(gfa, cfg, 0)
g = gfa.Graph(src, dst, V)
del src, dst
torch.cuda.empty_cache()
g.step(1)
for _ in range(2):
    g.reset()
    g.step(10)
for _ in range(3):
    g.reset()
    g.step(1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.step(9)
    torch.cuda.synchronize()
    print(f"step(9) {1e3 * (time.perf_counter() - t0):.3f} ms", flush=True)
g.close()

"""P in-process ranks on ONE GPU (loopback collective): wall time of supersteps
2..10 of labelPropagation(10), all ranks' handles driven from their own threads.
Measures the multi-rank control path (exchange, host syncs, launches), not scaling.

    python tools/loopback_bench.py [P] [scale] [reps] [posted]

posted: lpa_set_posted capacity (-1 adaptive, the default; 0 off).
"""
import sys
import time

sys.path.insert(0, ".")
import graphframes_amd as gfa  # noqa: E402
import torch  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 2
scale = int(sys.argv[2]) if len(sys.argv) > 2 else 22
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
posted = int(sys.argv[4]) if len(sys.argv) > 4 else -1
V = 1 << scale
s, d = gfa.gen_rmat(scale, 16, seed=1)
lb = gfa.Loopback(P)
gs = [gfa.Graph(s, d, V, rank=r, loopback=lb) for r in range(P)]
del s, d
for g in gs:
    g.set_posted(posted)
torch.cuda.empty_cache()


def one(r, g):
    g.reset()
    g.step(1)
    torch.cuda.synchronize()
    return None


ts = []
for k in range(reps + 1):
    gfa.run_ranks(gs, one)
    t0 = time.perf_counter()
    gfa.run_ranks(gs, lambda r, g: g.step(9))
    torch.cuda.synchronize()
    if k:
        ts.append(time.perf_counter() - t0)
ts.sort()
med = ts[len(ts) // 2]
info = gs[0].info()
print(f"P={P} scale={scale} posted={posted}: supersteps 2..10 median {med * 1e3:.2f} ms "
      f"({med / 9 * 1e3:.3f} ms/superstep), exchanges full {info['exchanges_full']} delta {info['exchanges_delta']} "
      f"posted {info['exchanges_posted']} missed {info['exchanges_post_missed']}")
for g in gs:
    g.close()
lb.close()

"""Per-superstep times of whole labelPropagation(10) calls (lpa_run from reset, the
concurrent schedule, HIP events per superstep) on a bench config; the environment
selects the variant (LPA_* switches).  One JSON line: medians over K calls.

    python tools/run_ab.py [C3|C4|C5|C2] [K] [label]
"""
import json
import statistics
import sys
import time

sys.path.insert(0, ".")
import bench  # noqa: E402
import graphframes_amd as gfa  # noqa: E402
import torch  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "C3"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 7
label = sys.argv[3] if len(sys.argv) > 3 else ""
cfg = bench.CONFIGS[cfg_name]
src, dst, V = bench.make_edges(gfa, cfg, 0)
g = gfa.Graph(src, dst, V)
del src, dst
torch.cuda.empty_cache()
out = torch.empty(V, dtype=torch.int32, device="cuda")
g.run(10, out=out)
ref = out.clone()
per, wall = [], []
for _ in range(K):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _, st = g.run(10, stats=True, out=out)
    torch.cuda.synchronize()
    wall.append(1e3 * (time.perf_counter() - t0))
    per.append(st["iter_ms"][:10])
    assert torch.equal(out, ref), "labels differ between calls"
med = [round(statistics.median(p[t] for p in per), 4) for t in range(10)]
print(json.dumps({"config": cfg_name, "label": label, "run10_ms": round(statistics.median(wall), 3),
                  "ss_ms": med, "ss1_ms": med[0], "ss2_10_ms": round(sum(med[1:]), 3),
                  "labels_crc": int(ref.to(torch.int64).sum().item())}), flush=True)
g.close()

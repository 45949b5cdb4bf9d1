"""Per-block timing of the class-blocked superstep-1 rebuild (diagnostic build:
csrc/Makefile blktime -> tools/diag_lib/liblpa_hip.so, loaded with LPA_LIB_PATH).
Prints, per block group (blocks b = x mod 8), the pieces phase and the plain-stream
phase end times relative to the earliest block start (wall clock, 100 MHz).

    LPA_LIB_PATH=tools/diag_lib/liblpa_hip.so python tools/blk_times.py [C3|C4|C5]
"""
import ctypes
import json
import sys

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
import graphframes_amd as gfa  # noqa: E402
import torch  # noqa: E402

cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "C3"]
src, dst, V = bench.make_edges(gfa, cfg, 0)
g = gfa.Graph(src, dst, V)
del src, dst
torch.cuda.empty_cache()
lib = g._lib
buf = (ctypes.c_ulonglong * (3 * 512))()
out = {"info": {k: g.info()[k] for k in ("arcs", "blocked_rows", "blocked_pieces")}}
for call in range(2):
    g.reset()
    g.step(1)            # superstep 1 + its labels-mode rebuild
    torch.cuda.synchronize()
    assert lib.lpa_diag_blk_times(buf) == 0
    t = np.array(buf, dtype=np.int64).reshape(512, 3)
    nb = int((t[:, 0] > 0).sum())
    if nb == 0:          # no blocked rebuild in this call (e.g. an ablation changed the labels)
        out[f"call{call}"] = {"blocks": 0}
        continue
    t = t[:nb]
    t0 = t[:, 0].min()
    rel = (t - t0) / 100.0  # us
    grp = {}
    for x in range(8):
        r = rel[x::8]
        grp[x] = {"start_max": round(float(r[:, 0].max()), 1), "pieces_end_med": round(float(np.median(r[:, 1])), 1),
                  "pieces_end_max": round(float(r[:, 1].max()), 1), "end_max": round(float(r[:, 2].max()), 1)}
    out[f"call{call}"] = {"blocks": nb, "groups": grp, "kernel_us": round(float(rel[:, 2].max()), 1)}
print(json.dumps(out, indent=1))
g.close()

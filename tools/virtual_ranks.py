"""Per-rank rehearsal of an N-GPU run on ONE GPU (the RCCL exchange replaced by the
caller-driven exchange through the host): builds the P rank handles of R-MAT scale S
(the weak-scaled bench config of N = P GPUs is scale 24 + log2 P), runs the supersteps
(full exchange in the label-dense supersteps or when a delta exceeds slice/4, changed-
label deltas otherwise -- the protocol of lpa_exchange.hip), reports each rank's tally
time per superstep and checks the labels bit-exact against a single-handle run.

    python tools/virtual_ranks.py --scale 26 --P 4 --steps 5
"""
import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import graphframes_amd as gfa  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--P", type=int, default=4)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--no-reference", action="store_true")
    a = ap.parse_args()
    V = 1 << a.scale
    t0 = time.time()
    src, dst = gfa.gen_rmat(a.scale, 16, seed=1, device=0)
    torch.cuda.synchronize()
    out = {"scale": a.scale, "P": a.P, "edges": int(src.numel())}
    ref = None
    if not a.no_reference:
        g = gfa.Graph(src, dst, V, device=0)
        g.step(a.steps)
        ref = g.labels()
        g.close()
        torch.cuda.empty_cache()
        print(f"reference single-handle run done ({time.time() - t0:.0f}s)", flush=True)
    tb = time.time()
    ranks = [gfa.Graph(src, dst, V, device=0, rank=r, nranks=a.P) for r in range(a.P)]
    torch.cuda.synchronize()
    out["build_s_per_rank"] = round((time.time() - tb) / a.P, 2)
    info = [g.info() for g in ranks]
    out["arcs_per_rank"] = [int(i["arcs"]) for i in info]
    out["device_gb_per_rank"] = [round(i["device_bytes"] / 1e9, 2) for i in info]
    slice_ = info[0]["slice"]
    print(f"built {a.P} ranks ({time.time() - tb:.0f}s): arcs {out['arcs_per_rank']}", flush=True)
    tally_ms, put_ms, modes = [], [], []
    for t in range(a.steps):
        ms = [g.step(1, stats=True)["iter_ms"][0] for g in ranks]
        tally_ms.append([round(x, 3) for x in ms])
        tp = time.time()
        deltas = None if t < 2 else [g.exchange_get_delta() for g in ranks]
        if deltas is not None and max(e.size for e in deltas) <= slice_ // 4:
            for g in ranks:
                g.exchange_put_delta(deltas)
            modes.append("delta")
        else:
            full = np.concatenate([g.exchange_get() for g in ranks])
            for g in ranks:
                g.exchange_put(full)
            modes.append("full")
        torch.cuda.synchronize()
        put_ms.append(round((time.time() - tp) * 1e3 / a.P, 1))
        print(f"superstep {t + 1}: tally ms per rank {tally_ms[-1]} ({modes[-1]})", flush=True)
    out["tally_ms_per_rank"] = tally_ms
    out["exchange_mode"] = modes
    out["host_exchange_plus_refresh_ms_per_rank"] = put_ms
    if ref is not None:
        lab = ranks[-1].labels()
        out["bit_exact_vs_single_handle"] = bool(np.array_equal(lab, ref))
    for g in ranks:
        g.close()
    out["wall_s"] = round(time.time() - t0, 1)
    print(json.dumps(out), flush=True)
    if ref is not None and not out["bit_exact_vs_single_handle"]:
        sys.exit(1)


if __name__ == "__main__":
    main()

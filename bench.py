"""Benchmark: LPA supersteps on R-MAT, GTEPS + HBM roofline.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scale S]

A "step" is one synchronous LPA superstep (GraphX Pregel iteration) over the
whole graph.  N = 1: config C3, R-MAT scale 24, edgefactor 16 (16.7 M vertices,
268 M input edges).  N > 1 (one process per GPU, torch.distributed.run): weak
scaling, scale 24 + log2(N) with every rank owning ~268 M edges' worth of arcs
(N = 4 is config C4, R-MAT scale 26); labels refreshed by one RCCL allgather per
superstep inside liblpa_hip.so.

Timed region: W untimed supersteps after a label reset (W = 1 makes the timed
supersteps iterations 2..K+1, the survey's "median over iterations 2..maxIter"),
then barrier + device sync, K supersteps, device sync + barrier; max over ranks.
The per-superstep / per-kernel breakdown (HIP events) comes from a second,
identical pass after another reset, so its events do not perturb `value`.
value = m * K / t / 1e9 (GTEPS, m = input edges of the whole job).
Inputs are generated in HBM before timing; CSR construction is not timed.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "LPA GTEPS per iteration at 1/2/4/8 MI355X; % of HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md: 8.0 TB/s spec)
# measured HBM traffic per launch of the dominant kernel: rocprofv3 --pmc FETCH_SIZE /
# WRITE_SIZE passes over this same bench command (tools/pmc_traffic.sh; FETCH doubled
# per the gfx950 correction, cross-checked on k_diff's known byte count)
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "r01", "e_traffic", "pmc_traffic.json")


def measured_traffic(kernel, scale):
    """HBM bytes per launch of `kernel` from the committed PMC summary (C3 only)."""
    try:
        with open(TRAFFIC_FILE) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None, None
    if scale != 24 or kernel not in t:
        return None, None
    return t[kernel]["traffic_bytes"], os.path.relpath(TRAFFIC_FILE, ROOT)


def kernel_bytes(info, name):
    """Algorithmic bytes per launch of one tally kernel.  The tally streams the
    replicated neighbour labels al[] (4 B per arc) instead of col + label gather
    (SURVEY.md §8(d) counts 8 B per arc for that formulation); per vertex it reads
    8 B of row offsets (seg: a 16 B segment descriptor per segment) and writes a
    4 B label."""
    from graphframes_amd import _lib

    b = _lib.KERNEL_BIN.get(name)
    if b is None:
        return None
    A = info["bin_arcs"][b]
    n = info["bin_vertices"][b]
    if b == "seg":
        return 4 * A + 16 * info["segments"] + 4 * n
    return 4 * A + 8 * (n + 1) + 4 * n


def cpu_baseline(src_np, dst_np, V, gpu_graph, warmup, budget_s=25.0):
    """Oracle (OpenMP C restatement, 'port') timed on this host on the same graph:
    supersteps starting from the GPU's labels after `warmup` supersteps, CSR build
    excluded; also checks the CPU result against the GPU's next superstep."""
    import numpy as np

    from oracle import oracle

    rp, col = oracle.build_csr(V, src_np, dst_np)
    gpu_graph.reset()
    gpu_graph.step(warmup)
    cur = gpu_graph.labels()
    times = []
    nxt = cur
    t_start = time.perf_counter()
    while True:
        t0 = time.perf_counter()
        nxt = oracle.superstep_csr(rp, col, cur)   # dense-id CSR, same semantics
        times.append(time.perf_counter() - t0)
        if len(times) >= 2 or time.perf_counter() - t_start > budget_s:
            break
        cur = nxt
    # parity of the last CPU superstep vs the GPU
    gpu_graph.reset()
    gpu_graph.step(warmup + len(times))
    ok = bool(np.array_equal(gpu_graph.labels(), nxt))
    t = sum(times) / len(times)
    return dict(value=round(src_np.size / t / 1e9, 4), unit="GTEPS", cores=oracle.num_threads(),
                kind="port",
                sample=f"oracle/lpa_oracle.c (OpenMP) supersteps {warmup + 1}..{warmup + len(times)} "
                       f"of the same graph (full size), mean {t * 1e3:.1f} ms/superstep, CSR build excluded",
                parity_vs_gpu=ok)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=9)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scale", type=int, default=None, help="R-MAT scale (default 24 + log2(N))")
    ap.add_argument("--edgefactor", type=int, default=16)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")
        args.gpus = world

    import numpy as np
    import torch
    import torch.distributed as dist

    import graphframes_amd as gfa

    scale = args.scale if args.scale is not None else 24 + int(round(math.log2(world)))
    if world > 1:
        # control plane only (barriers, RCCL id broadcast, max-over-ranks); the
        # per-superstep label allgather is RCCL inside liblpa_hip.so
        dist.init_process_group("gloo", rank=rank, world_size=world)
    device = local_rank
    torch.cuda.set_device(device)

    def barrier():
        if world > 1:
            dist.barrier()

    src, dst = gfa.gen_rmat(scale, args.edgefactor, seed=args.seed, device=device)
    V = 1 << scale
    m = src.numel()
    if world > 1:
        obj = [gfa.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        g = gfa.Graph(src, dst, V, device=device, rank=rank, nranks=world, comm_id=obj[0])
    else:
        g = gfa.Graph(src, dst, V, device=device)
    info = g.info()
    if world == 1 and not args.no_cpu_baseline:
        src_np, dst_np = src.cpu().numpy(), dst.cpu().numpy()
    del src, dst
    torch.cuda.empty_cache()

    g.step(1)          # prime: code objects loaded, caches warm
    g.reset()
    if args.warmup > 0:
        g.step(args.warmup)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.step(args.steps)     # timed: no per-kernel timing events in this run
    torch.cuda.synchronize()
    barrier()
    t = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([t], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt.item())
    # breakdown: the same supersteps again, with HIP events around every kernel and
    # the tally kernels serialized on one stream, so each kernel's time is its
    # standalone duration (the roofline of that kernel, not of its co-runners); the
    # events and the serialization change the schedule, so `value` is not from here
    g.reset()
    if args.warmup > 0:
        g.step(args.warmup)
    g.set_serial(True)
    st = g.step(args.steps, stats=True)
    g.set_serial(False)
    g.reset()
    if args.warmup > 0:
        g.step(args.warmup)
    st_conc = g.step(args.steps, stats=True)   # per-superstep times of the concurrent schedule

    value = m * args.steps / t / 1e9
    kms = st["kernel_ms"]
    ksteps = min(args.steps, 64)
    dom = max((k for k in kms if kernel_bytes(info, k) is not None), key=lambda k: kms[k])
    dom_ms = kms[dom] / ksteps
    dom_bytes = kernel_bytes(info, dom)
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
    traffic, traffic_src = measured_traffic(dom, scale)
    it_ms = sorted(st_conc["iter_ms"])
    med_iter_ms = it_ms[len(it_ms) // 2]
    iter_bytes = 8 * info["arcs"] + 12 * info["slice"] + 8
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GTEPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(t * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic",
        "config": {
            "workload": f"R-MAT scale-{scale} edgefactor {args.edgefactor} (Graph500 .57/.19/.19/.05, "
                        f"scrambled ids, seed {args.seed}, duplicates+self-loops kept), "
                        f"synchronous LPA supersteps (GraphFrames labelPropagation semantics)",
            "config_id": "C3" if (world == 1 and scale == 24) else ("C4" if scale == 26 else "weak-scaled"),
            "vertices": V, "edges": m, "arcs_rank0": info["arcs"],
            "parallelism": f"1D degree-ranked vertex partition x{world}, RCCL label allgather",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": dom,
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "bytes_per_launch": dom_bytes,
            "avg_launch_ms": round(dom_ms, 4),
        },
        "iteration_roofline": {
            "bytes": iter_bytes, "median_iter_ms": round(med_iter_ms, 4),
            "achieved_GBs": round(iter_bytes / (med_iter_ms * 1e-3) / 1e9, 1),
            "frac": round(iter_bytes / (med_iter_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "iter_ms": [round(x, 4) for x in st_conc["iter_ms"]],
        },
        "kernel_ms_per_step": {k: round(v / ksteps, 4) for k, v in kms.items()},
        "kernel_ms_note": "standalone (tally kernels serialized on one stream, HIP events)",
        "exchange_ms_per_step": round(st["exchange_ms"] / ksteps, 4),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(src_np, dst_np, V, g, args.warmup)
    if rank == 0:
        print(json.dumps(out), flush=True)
    g.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

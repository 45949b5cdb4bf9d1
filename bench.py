"""Benchmark: LPA on the BASELINE.json configs, GTEPS + HBM roofline.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C3|C4|C5] [--scale S]

Workloads (synthetic, generated in HBM; CSR construction not timed):
  C3  R-MAT scale 24, edgefactor 16 (16.7 M V / 268 M E)          default at N = 1
  C4  R-MAT scale 26, edgefactor 16 (67 M V / 1.07 B E)            default at N > 1
      (BASELINE config 4: "vertex-partitioned across 2/4/8 MI355X"), strong scaling:
      the same graph split over the N ranks, every rank holding ~1/N of the arcs
  C5  Chung-Lu gamma 2.1, 40 M V / 1.4 B E, max degree ~1.25 M (--config C5; BASELINE
      config 5 is quoted at 8 GPUs)
  C2  planted-partition SBM, 1 M V / 20 M E, 100 blocks            (--config C2)
  --weak (N a power of two): R-MAT scale 24 + log2 N instead, 268 M edges per GPU
  (N = 4 is C4; scale 27 at N = 8 has no at-size parity test: unvalidated).

--gpus N > 1 without a torch.distributed environment re-launches this script under
torch.distributed.run (one rank per GPU) as a child process, before any GPU call.
All run labelPropagation(maxIter=10) semantics (Graphframes.py:81).

A "step" is ONE labelPropagation(maxIter=10) call as a user makes it, timed over
its supersteps 2..10: per step the labels are reset to L0 and superstep 1 runs
untimed; then barrier + device sync, supersteps 2..10, device sync + barrier.
The K steps' windows are summed, max over ranks.  This is SURVEY.md §8(d)'s
"iterations 2..maxIter" window: it contains the label-dense supersteps 2-3 that
decide the real call's time, not only converged ones, whatever K / W the caller
passes.  value = m * 9 * K / t_sum / 1e9 GTEPS (m = input edges of the job).
W warm-up calls run untimed before.

Extra keys: the BASELINE.md:48 method (median superstep time over iterations
2..maxIter across >= 5 runs, HIP events, concurrent schedule), the wall time of a
whole lpa_run(10) from reset (`run_maxiter10_ms`, supersteps 1..10 + label gather),
the per-kernel breakdown of a serialized pass (`roofline`: the al[] rebuild, the longest
kernel of the timed window; `roofline_tally`: the dominant tally kernel),
`moved_bytes_frac` (bytes the replicated-label formulation actually moves in a
converged superstep), the outlier stage (`outlier_l1_ms`, `outlier_l2_ms`) and the
CPU baseline (OpenMP oracle on this host) at N = 1, and `quality`: community count
and modularity of the GPU labels for C1 (the reference's sample graph, maxIter=5),
the bench graph and C2 (plus C2's NMI against its planted blocks).
"""
import argparse
import json
import math
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "LPA GTEPS per iteration at 1/2/4/8 MI355X; % of HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md: 8.0 TB/s spec)
# measured HBM traffic per launch of the dominant kernels: rocprofv3 --pmc FETCH_SIZE /
# WRITE_SIZE passes over the C3 workload (tools/pmc_r03.sh; FETCH doubled per the gfx950
# correction, calibrated on a known-byte stream in profiles/r02/traffic)
TRAFFIC_FILES = [os.path.join(ROOT, "profiles", "r04", "traffic", "pmc_traffic.json"),
                 os.path.join(ROOT, "profiles", "r03", "traffic", "pmc_traffic.json"),
                 os.path.join(ROOT, "profiles", "r02", "traffic", "pmc_traffic.json"),
                 os.path.join(ROOT, "profiles", "r01", "e_traffic", "pmc_traffic.json")]

CONFIGS = {
    "C2": dict(kind="sbm", V=1_000_000, blocks=100, m=20_000_000, seed=20261015,
               text="planted-partition SBM 1M vertices / 20M edges / 100 blocks, p_in 0.9, seed 20261015"),
    "C3": dict(kind="rmat", scale=24, ef=16, seed=1),
    "C4": dict(kind="rmat", scale=26, ef=16, seed=1),
    "C5": dict(kind="chunglu", V=40_000_000, m=1_400_000_000, gamma=2.1, max_deg=1.25e6, seed=7,
               text="Chung-Lu power law gamma 2.1, 40M vertices / 1.4B edges, expected max degree 1.25M, seed 7"),
}
MAX_ITER = 10


def superstep_traffic(kernel, superstep, config_id):
    """HBM bytes of `kernel`'s launch(es) in superstep `superstep` of a labelPropagation(10)
    call from the newest per-config PMC summary (tools/pmc_r05.sh ->
    profiles/r06/traffic/ or profiles/r05/traffic/pmc_traffic_<config>.json), or (None, None)."""
    for rnd in ("r06", "r05"):
        path = os.path.join(ROOT, "profiles", rnd, "traffic", f"pmc_traffic_{config_id}.json")
        try:
            with open(path) as f:
                t = json.load(f)
            per = t["per_superstep"]
            # keys carry template arguments ("k_al_rebuild_hot<true, false>"): match the base name
            key = next(k for k in per if k.split("<")[0] == kernel)
            e = per[key][f"superstep_{superstep}"]
        except (OSError, ValueError, KeyError, StopIteration):
            continue
        return e["traffic_bytes"], os.path.relpath(path, ROOT)
    return None, None


def measured_traffic(kernel, config_id):
    """HBM bytes per launch of `kernel` from the committed PMC summaries: the round-5
    per-config files for the rebuild kernels (superstep 2's refresh in the timed window,
    superstep 1's outside it), else the older C3 files."""
    if kernel == "k_al_rebuild_hot":
        # the refreshes that rebuilt inside the timed window (supersteps 2..10), labels /
        # bits mode or the giant codes: their mean, as the roofline's launches average
        got, src = [], None
        for t in range(2, MAX_ITER + 1):
            for k in ("k_al_rebuild_hot", "k_code_rebuild"):
                b, sx = superstep_traffic(k, t, config_id)
                if b is not None and b > 1e8:
                    got.append(b)
                    src = sx
        if got:
            return round(sum(got) / len(got)), src
    if kernel == "k_al_rebuild_hot_superstep1":
        for k in ("k_code_rebuild", "k_al_rebuild_hot"):
            b, src = superstep_traffic(k, 1, config_id)
            if b is not None and b > 0.2 * 1e6:
                return b, src
    if config_id != "C3":
        return None, None
    for path in TRAFFIC_FILES:
        try:
            with open(path) as f:
                t = json.load(f)
        except (OSError, ValueError):
            continue
        if kernel in t:
            return t[kernel]["traffic_bytes"], os.path.relpath(path, ROOT)
    return None, None


def kernel_bytes(info, name):
    """Algorithmic bytes per launch of one tally kernel.  The tally streams the
    replicated neighbour labels al[] (4 B per arc) instead of col + label gather
    (SURVEY.md §8(d) counts 8 B per arc for that formulation); per vertex it reads
    8 B of row offsets (seg: a 16 B unit descriptor per 512-arc unit) and writes a
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


def moved_bytes_converged(info):
    """Bytes a converged superstep of the replicated-label formulation must move
    at least: the al[] stream (4 B/arc), unit descriptors, row offsets, the label
    write, the unit words staged for the hub combine (8 B written + read, about one
    per unit when converged) and the diff's two label-vector reads."""
    S, vpad = info["slice"], info["slice"] * info["nranks"]
    return 4 * info["arcs"] + 16 * info["segments"] + 8 * (S + 1) + 4 * S + 16 * info["segments"] + 8 * vpad


def make_edges(gfa, cfg, device):
    if cfg["kind"] == "rmat":
        s, d = gfa.gen_rmat(cfg["scale"], cfg["ef"], seed=cfg["seed"], device=device)
        return s, d, 1 << cfg["scale"]
    if cfg["kind"] == "sbm":
        s, d = gfa.gen_sbm(cfg["V"], cfg["blocks"], cfg["m"], seed=cfg["seed"], device=device)
        return s, d, cfg["V"]
    s, d = gfa.gen_chunglu(cfg["V"], cfg["m"], cfg["gamma"], cfg["max_deg"], seed=cfg["seed"], device=device)
    return s, d, cfg["V"]


def workload_text(cfg, config_id):
    if cfg["kind"] == "rmat":
        return (f"R-MAT scale-{cfg['scale']} edgefactor {cfg['ef']} (Graph500 .57/.19/.19/.05, scrambled ids, "
                f"seed {cfg['seed']}, duplicates+self-loops kept)")
    return cfg["text"]


def cpu_baseline(src_np, dst_np, V, gpu_graph, budget_s=25.0):
    """Oracle (OpenMP C restatement, 'port') timed on this host on the same graph:
    supersteps 2.. of the same labelPropagation run, starting from the GPU's
    superstep-1 labels, CSR build excluded; the last CPU superstep is checked
    against the GPU's."""
    import numpy as np

    from oracle import oracle

    rp, col = oracle.build_csr(V, src_np, dst_np)
    gpu_graph.reset()
    gpu_graph.step(1)
    cur = gpu_graph.labels()
    times = []
    nxt = cur
    t_start = time.perf_counter()
    while True:
        t0 = time.perf_counter()
        nxt = oracle.superstep_csr(rp, col, cur)   # dense-id CSR, same semantics
        times.append(time.perf_counter() - t0)
        if len(times) >= 3 or time.perf_counter() - t_start > budget_s:
            break
        cur = nxt
    gpu_graph.reset()
    gpu_graph.step(1 + len(times))
    ok = bool(np.array_equal(gpu_graph.labels(), nxt))
    t = sum(times) / len(times)
    return dict(value=round(src_np.size / t / 1e9, 4), unit="GTEPS", cores=oracle.num_threads(),
                kind="port",
                sample=f"oracle/lpa_oracle.c (OpenMP) supersteps 2..{1 + len(times)} of the same graph "
                       f"(full size), mean {t * 1e3:.1f} ms/superstep, CSR build excluded",
                parity_vs_gpu=ok)


_T0 = time.perf_counter()


def progress(msg):
    """A stderr progress line per phase (the JSON result is the only stdout line)."""
    print(f"[bench {time.perf_counter() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def self_launch(n):
    """Run this script under torch.distributed.run with n ranks (one per GPU) as a
    child process; returns its exit code.  Called before torch is imported."""
    import socket
    import subprocess

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def quality_entry(g, lab, extra=None):
    """Community count + modularity of labels `lab` on handle g's graph (lpa_quality:
    exact integer sums on the GPU; the symmetrised multigraph LPA votes on)."""
    q = g.quality(lab)
    out = dict(communities=q["n_communities"], modularity=round(q["modularity"], 6),
               intra_arc_fraction=round(q["intra_arcs"] / q["arcs"], 6) if q["arcs"] else 0.0)
    if extra:
        out.update(extra)
    return out


def quality_report(gfa, device, bench_entry):
    """C1 (the reference's sample graph, maxIter=5 as Graphframes.py:81), the bench
    graph (maxIter=10) and C2 (maxIter=10, NMI vs the planted blocks): community
    count + modularity of the GPU labels."""
    import numpy as np

    rep = {"agreement_note": "GraphFrames/GraphX itself cannot run here (no JVM, no pyspark): agreement "
                             "with its own output is unpinned; labels are bit-exact vs the oracle's "
                             "smallest-label tie-break (tests/)",
           "bench_graph": bench_entry}
    z = np.load(os.path.join(ROOT, "tests", "golden", "r9_golden.npz"), allow_pickle=False)
    V1 = int(z["ids"].size)
    with gfa.Graph(z["src"], z["dst"], V1, device=device) as g1:
        lab1 = g1.run(5)
        rep["C1"] = quality_entry(g1, lab1, dict(max_iter=5, vertices=V1, edges=int(z["src"].size)))
    c2 = CONFIGS["C2"]
    s2, d2 = gfa.gen_sbm(c2["V"], c2["blocks"], c2["m"], seed=c2["seed"], device=device)
    with gfa.Graph(s2, d2, c2["V"], device=device) as g2:
        del s2, d2
        lab2 = g2.run(MAX_ITER)
        extra = dict(max_iter=MAX_ITER)
        try:
            from sklearn.metrics import normalized_mutual_info_score as nmi
            truth = np.minimum(np.arange(c2["V"]) // (c2["V"] // c2["blocks"]), c2["blocks"] - 1)
            extra["nmi_vs_planted_blocks"] = round(float(nmi(truth, lab2)), 4)
        except ImportError:
            extra["nmi_vs_planted_blocks"] = None
        rep["C2"] = quality_entry(g2, lab2, extra)
    return rep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5, help="timed labelPropagation(10) calls")
    ap.add_argument("--warmup", type=int, default=1, help="untimed labelPropagation(10) calls")
    ap.add_argument("--config", choices=sorted(CONFIGS), default=None,
                    help="default C3 at N = 1, C4 at N > 1")
    ap.add_argument("--weak", action="store_true",
                    help="N > 1: weak scaling from C3 (R-MAT scale 24 + log2 N; N a power of two)")
    ap.add_argument("--scale", type=int, default=None, help="R-MAT scale override (custom config)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-outlier", action="store_true")
    ap.add_argument("--no-quality", action="store_true", help="skip the community count / modularity report")
    ap.add_argument("--launch-check", action="store_true", help=argparse.SUPPRESS)  # tests: ranks + config only
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # the driver's `bench.py --gpus N`: one rank process per GPU, started here
        # before anything touches the GPU (a child process, never an exec)
        sys.exit(self_launch(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    args.gpus = world
    scaling = "strong"
    if args.weak and world > 1 and args.config is None and args.scale is None:
        # weak scaling from C3: 2^24 * N vertices, 268 M edges per GPU (N = 4: C4)
        if world & (world - 1):
            raise SystemExit(f"--weak needs a power-of-two rank count (268 M edges per GPU), got {world}")
        args.scale = 24 + world.bit_length() - 1
        scaling = "weak"
    # N > 1 default: BASELINE config 4, R-MAT-26 partitioned over the N ranks
    config_id = args.config or ("C4" if world > 1 and args.scale is None else "C3")
    cfg = dict(CONFIGS[config_id])
    if args.scale is not None:
        if cfg["kind"] != "rmat":
            raise SystemExit("--scale applies to the R-MAT configs")
        cfg["scale"] = args.scale
        config_id = {24: "C3", 26: "C4"}.get(args.scale, f"R-MAT-{args.scale}")
    if args.launch_check:   # no GPU: what each rank would run (tests/test_bench_launch.py)
        # one write(2) per rank: ranks share the pipe, and print() may split a line
        line = json.dumps(dict(rank=rank, world=world, local_rank=local_rank, config_id=config_id,
                               scaling=scaling, cfg=cfg)) + "\n"
        sys.stdout.flush()
        os.write(1, line.encode())
        return

    import numpy as np
    import torch
    import torch.distributed as dist

    import graphframes_amd as gfa

    if world > 1:
        # control plane only (barriers, RCCL id broadcast, max-over-ranks); the
        # per-superstep label allgather is RCCL inside liblpa_hip.so
        dist.init_process_group("gloo", rank=rank, world_size=world)
    device = local_rank
    torch.cuda.set_device(device)

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(x):
        if world == 1:
            return x
        tt = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item())

    src, dst, V = make_edges(gfa, cfg, device)
    m = src.numel()
    if world > 1:
        obj = [gfa.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        g = gfa.Graph(src, dst, V, device=device, rank=rank, nranks=world, comm_id=obj[0])
    else:
        g = gfa.Graph(src, dst, V, device=device)
    info = g.info()
    keep_host = world == 1 and not args.no_cpu_baseline
    if keep_host:
        src_np, dst_np = src.cpu().numpy(), dst.cpu().numpy()
    del src, dst
    torch.cuda.empty_cache()

    progress(f"{config_id}: built (arcs {info['arcs']}), warm-up")
    g.step(1)          # prime: code objects loaded, caches warm
    for _ in range(args.warmup):
        g.reset()
        g.step(MAX_ITER)

    progress("timed calls")
    # ---- timed: K labelPropagation(10) calls, supersteps 2..10 of each ----
    t_sum = 0.0
    call_ms = []
    for _ in range(args.steps):
        g.reset()
        g.step(1)                      # superstep 1 (from L0), untimed
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.step(MAX_ITER - 1)           # supersteps 2..10: no per-kernel events
        torch.cuda.synchronize()
        barrier()
        dt = time.perf_counter() - t0
        t_sum += dt
        call_ms.append(dt * 1e3)
    t_sum = max_over_ranks(t_sum)
    n_timed = (MAX_ITER - 1) * args.steps
    value = m * n_timed / t_sum / 1e9

    cs = sorted(call_ms)
    progress(f"timed: {value:.1f} GTEPS (per call ms: min {cs[0]:.3f} median {cs[len(cs) // 2]:.3f} "
             f"max {cs[-1]:.3f}); per-superstep method")
    # ---- BASELINE.md:48 method: median superstep time of iterations 2..10 over >= 5
    # runs (HIP events around each superstep, concurrent schedule, graphs replayed) ----
    runs = max(5, args.steps)
    iter_ms = []     # [run][superstep 2..10]
    for _ in range(runs):
        g.reset()
        g.step(1)
        iter_ms.append(g.step(MAX_ITER - 1, stats=True)["iter_ms"])
    flat = [x for r in iter_ms for x in r]
    med_ms = max_over_ranks(statistics.median(flat))
    per_step_med = [round(statistics.median(r[i] for r in iter_ms), 4) for i in range(MAX_ITER - 1)]
    # the same with the frontier off: converged supersteps then stream every al[] arc,
    # the bytes moved_bytes_converged counts (with the frontier they move far fewer)
    g.set_frontier(False)
    off_ms = []
    for _ in range(3):
        g.reset()
        g.step(1)
        off_ms.append(g.step(MAX_ITER - 1, stats=True)["iter_ms"])
    g.set_frontier(True)
    conv_ms = max_over_ranks(statistics.median(x for r in off_ms for x in r[2:]))  # supersteps 4..10
    # full-work figure: supersteps 2..10 with the frontier off (every row tallied every
    # superstep; only the exact giant-label settles of supersteps 3-4 still skip reads)
    full_ms = max_over_ranks(statistics.median(sum(r) for r in off_ms))

    progress("lpa_run(10) wall time")
    # ---- whole call: lpa_run(10) from reset, labels gathered into a device tensor ----
    out = torch.empty(V, dtype=torch.int32, device=f"cuda:{device}")
    run_ms = []
    for _ in range(3):
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.run(MAX_ITER, out=out)
        torch.cuda.synchronize()
        barrier()
        run_ms.append((time.perf_counter() - t0) * 1e3)
    run_ms = max_over_ranks(statistics.median(run_ms))
    # superstep 1 (from L0, column runs + the first al[] rebuild) of those calls, events
    ss1 = []
    for _ in range(3):
        g.reset()
        ss1.append(g.step(1, stats=True)["iter_ms"][0])
    ss1_ms = max_over_ranks(statistics.median(ss1))
    # partition quality of the labels of that call (rank 0: the full dense vector)
    quality = None
    if rank == 0 and not args.no_quality:
        quality = dict(bench_graph=quality_entry(g, out, dict(max_iter=MAX_ITER, config_id=config_id)))

    progress("serialized breakdown")
    # ---- breakdown: supersteps 2..10 again with the tally kernels serialized on one
    # stream and HIP events around every kernel (standalone durations: the roofline
    # of that kernel, not of its co-runners; not used for `value`) ----
    # frontier off here: every row is tallied, so each kernel's time covers the
    # bytes `kernel_bytes` counts (the frontier skips most rows once labels settle)
    g.set_frontier(False)
    g.reset()
    g.step(1)
    g.set_serial(True)
    per_ss = [g.step(1, stats=True) for _ in range(MAX_ITER - 1)]   # supersteps 2..10
    # the untimed superstep 1's al[] rebuild (labels mode; the serialized schedule tallies
    # superstep 1 by hash instead of column runs, to the same labels, so its rebuild is
    # the shipped one), median of 3, HIP events
    ss1_rb = []
    for _ in range(3):
        g.reset()
        ss1_rb.append(g.step(1, stats=True)["kernel_ms"]["k_al_rebuild_hot"])
    # did that refresh take the giant codes (2-bit codes per arc instead of a label rebuild)?
    ss1_code = bool(g.info()["code_refresh"])
    g.set_serial(False)
    g.set_frontier(True)
    kms = {k: sum(st["kernel_ms"][k] for st in per_ss) for k in per_ss[0]["kernel_ms"]}
    exch_ms = sum(st["exchange_ms"] for st in per_ss)
    dom = max((k for k in kms if kernel_bytes(info, k) is not None), key=lambda k: kms[k])
    # launches that moved kernel_bytes: every one, except that k_lpa_units streams
    # only the units of rows > 4096 arcs in the supersteps where k_lpa_block tallied
    # the shorter hub rows (label-dense supersteps; timed separately as k_lpa_block)
    full = [st for st in per_ss if dom != "k_lpa_units" or st["kernel_ms"]["k_lpa_block"] == 0.0]
    dom_ms = sum(st["kernel_ms"][dom] for st in full) / max(1, len(full))
    dom_bytes = kernel_bytes(info, dom)
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
    traffic, traffic_src = measured_traffic(dom, config_id)
    # the al[] rebuild: the single longest kernel of the shipped (frontier) window,
    # launched every superstep but gathering only when > rebuild_frac of the arcs
    # changed (label-dense supersteps); its launches that rebuilt
    rb = [st["kernel_ms"]["k_al_rebuild_hot"] for st in per_ss]
    rb_work = [x for x in rb if x > 0.1]
    rb_bytes = 8 * info["arcs"] + 4 * info["V"]
    rb_traffic, rb_src = measured_traffic("k_al_rebuild_hot", config_id)
    # this rank's vertices (the slice is padded to a power of two at P > 1, lpa_build.hip)
    S = -(-info["V"] // info["nranks"])
    iter_bytes = 8 * info["arcs"] + 12 * S + 8     # SURVEY §8(d) contract, this rank's share
    moved = moved_bytes_converged(info)
    # contract roofline of the whole job: every rank moves its share at 8 TB/s at once
    roof_gteps = m / (iter_bytes / (HBM_PEAK_GBS * 1e9)) / 1e9
    full_gteps = m * (MAX_ITER - 1) / (full_ms * 1e-3) / 1e9
    call_gteps = m * MAX_ITER / (run_ms * 1e-3) / 1e9

    tally_obj = {
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
        "launches": f"{len(full)} launches in supersteps 2..{MAX_ITER} that stream every unit (serialized "
                    f"schedule, frontier off: every row tallied, so each launch moves bytes_per_launch), "
                    f"HIP events on the handle's stream",
    }
    rb_obj = None if not rb_work else {
        "bound": "hbm",
        "kernel": "k_al_rebuild_hot",
        "achieved": round(rb_bytes / (statistics.mean(rb_work) * 1e-3) / 1e9, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(rb_bytes / (statistics.mean(rb_work) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        "traffic": rb_traffic,
        "traffic_source": rb_src,
        "bytes_per_launch": rb_bytes,
        "bytes_note": "col 4 B/arc + al 4 B/arc + each label once (4 B/vertex); superstep 2's rebuild runs in "
                      "bits mode (giant-label bits, gathers only for the other labels: PMC traffic 1.13x)",
        "avg_launch_ms": round(statistics.mean(rb_work), 4),
        "launches": f"{len(rb_work)} rebuilding launch(es) in supersteps 2..{MAX_ITER} (serialized schedule, "
                    f"HIP events on the handle's stream)",
    }

    ss1_rb_ms = max_over_ranks(statistics.median(ss1_rb))
    ss1_traffic, ss1_src = measured_traffic("k_al_rebuild_hot_superstep1", config_id)
    if ss1_code:
        # the giant-code refresh: col 4 B/arc, a 2-bit code per arc of the coded rows, a
        # 4-B label per arc of the others, the code array (1/4 B per slot) and the label
        # vector once
        # the coded rows: above 64 arcs on a label vector of <= 64 MB, else above 8 (lpa_build)
        lbin = 5 if 4 * info["slice"] * info["nranks"] <= 64 << 20 else 8
        pcut = sum(list(info["bin_arcs"].values())[:lbin])
        ss1_bytes = 4 * info["arcs"] + pcut // 4 + 4 * (info["arcs"] - pcut) + info["V"] // 4 + 4 * info["V"]
    else:
        ss1_bytes = rb_bytes
    ss1_obj = None if ss1_rb_ms <= 0.1 else {
        "bound": "hbm",
        "kernel": "k_code_rebuild" if ss1_code else "k_al_rebuild_hot",
        "achieved": round(ss1_bytes / (ss1_rb_ms * 1e-3) / 1e9, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(ss1_bytes / (ss1_rb_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        "traffic": ss1_traffic,
        "traffic_source": ss1_src,
        "bytes_per_launch": ss1_bytes,
        "avg_launch_ms": round(ss1_rb_ms, 4),
        "note": ("superstep 1's refresh (outside the timed window, inside lpa_run(10)), the giant-code form: "
                 "2-bit label codes per arc for superstep 2's settle instead of a 4-B label rebuild; bound by "
                 "its gather lanes (DESIGN.md section 4, Giant codes)") if ss1_code else
                ("superstep 1's rebuild (labels mode; outside the timed window, inside lpa_run(10)): "
                 "bound by its L2-missing gathers (PMC traffic / algorithmic in traffic), DESIGN.md section 4"),
    }

    out_json = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GTEPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(t_sum * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic",
        "config": {
            "workload": workload_text(cfg, config_id) + "; labelPropagation(maxIter=10) "
                        "(GraphFrames semantics, smallest-label ties)",
            "config_id": config_id,
            "vertices": V, "edges": m, "arcs_rank0": info["arcs"],
            "parallelism": f"1D degree-ranked vertex partition x{world}, RCCL label allgather",
            "scaling_note": ("weak: R-MAT scale 24 + log2 N, 268 M edges per GPU" if scaling == "weak" else
                             "strong: the same graph at every N (N = 1 default C3, the north-star config; "
                             "N > 1 default C4, BASELINE's partitioned config)"),
        },
        "timed_window": f"supersteps 2..{MAX_ITER} of each of {args.steps} labelPropagation(maxIter={MAX_ITER}) "
                        f"calls ({n_timed} supersteps); step = one call",
        "ms_per_superstep": round(t_sum * 1e3 / n_timed, 4),
        "call_ms_min_median_max": [round(cs[0], 4), round(cs[len(cs) // 2], 4), round(cs[-1], 4)],
        "baseline_method": {
            "what": f"BASELINE.md:48: median superstep time over iterations 2..{MAX_ITER}, {runs} runs, HIP events",
            "median_iter_ms": round(med_ms, 4),
            "gteps": round(m / (med_ms * 1e-3) / 1e9, 3),
            "median_ms_per_superstep_2_to_10": per_step_med,
        },
        "run_maxiter10_ms": round(run_ms, 3),
        "run_maxiter10_note": "lpa_run(10) wall time from reset: supersteps 1..10 + labels gathered to HBM",
        # the single longest kernel of the shipped (frontier) window is the al[] rebuild
        # of superstep 2 (when one ran); the dominant tally kernel follows as
        # roofline_tally
        "roofline": rb_obj if rb_obj is not None else tally_obj,
        "roofline_tally": tally_obj,
        "roofline_superstep1_rebuild": ss1_obj,
        "iteration_roofline": {
            "what": ("north_star 'fraction of HBM-roofline TEPS' against the SURVEY §8(d) contract: B_iter = "
                     "16m+12V+8 bytes per superstep (col 4 B/arc + gathered label 4 B/arc + row offsets + label "
                     "write), roofline TEPS = m / (B_iter / 8 TB/s).  frac = the full-work figure (every row "
                     "tallied every superstep) over that roofline"),
            "bytes": iter_bytes,
            "roofline_gteps": round(roof_gteps, 1),
            "frac": round(full_gteps / roof_gteps, 4),
            "full_work": {
                "what": f"supersteps 2..{MAX_ITER} with the frontier OFF (every row re-tallied; the exact "
                        f"giant-label row settles of supersteps 3-4 stay on), median of 3 calls, HIP events",
                "ms": round(full_ms, 4),
                "gteps": round(full_gteps, 2),
                "frac": round(full_gteps / roof_gteps, 4),
            },
            "whole_call": {
                "what": f"lpa_run({MAX_ITER}) wall time from reset: supersteps 1..{MAX_ITER} + labels gathered "
                        f"to HBM (median of 3)",
                "ms": round(run_ms, 4),
                "superstep1_ms": round(ss1_ms, 4),
                "gteps": round(call_gteps, 2),
                "frac": round(call_gteps / roof_gteps, 4),
            },
            "shipped_vs_contract_roofline": round(value / roof_gteps, 4),
            "shipped_note": ("value (frontier on) over the contract roofline TEPS: a time-to-result ratio, NOT a "
                             "bandwidth fraction -- the exact frontier and the giant-label settle skip most rows "
                             "after superstep 4, so the shipped window moves far fewer bytes than B_iter per "
                             "superstep"),
        },
        "moved_bytes_frac": round(moved / (conv_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        "moved_bytes_note": (f"{moved} B the replicated-label formulation moves per converged superstep "
                             f"(al[] 4 B/arc + units + row offsets + labels + staged words + diff) / "
                             f"median converged superstep {conv_ms:.4f} ms (supersteps 4..10, frontier OFF so "
                             f"that every arc is streamed) / 8 TB/s"),
        "kernel_ms_per_step": {k: round(v / (MAX_ITER - 1), 4) for k, v in kms.items()},
        "kernel_ms_note": "per superstep, standalone (tally kernels serialized on one stream, HIP events)",
        "exchange_ms_per_superstep": round(exch_ms / (MAX_ITER - 1), 4),
    }
    if world == 1 and not args.no_outlier:
        progress("outlier stage")
        lab = g.run(MAX_ITER)
        dlab = torch.from_numpy(lab).to(f"cuda:{device}")
        for mode, key in (("L1", "outlier_l1"), ("L2", "outlier_l2")):
            # device form (labels and every output in HBM, as `value`'s inputs are), then
            # the host-array form of the drop-in API (host labels in, numpy arrays out)
            for form, labels_in in (("", dlab), ("_host", lab)):
                ts = []
                for _ in range(3):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    res = g.outlier(labels_in, mode, sub_iter=5)
                    torch.cuda.synchronize()
                    ts.append((time.perf_counter() - t0) * 1e3)
                    progress(f"outlier {mode}{form}: {ts[-1]:.1f} ms")
                out_json[f"{key}{form}_ms"] = round(statistics.median(ts), 2)
                if form == "":
                    out_json[f"{key}_first_ms"] = round(ts[0], 2)
            if mode == "L2":
                out_json["outlier_l2_flagged"] = int(res["flags"].sum())
        out_json["outlier_note"] = ("lpa_outlier on the maxIter=10 labels, median of 3 calls; outlier_l*_ms: device "
                                    "labels in, device arrays out (lpa_outlier_device); outlier_l*_host_ms: host "
                                    "labels in, host numpy arrays out (lpa_outlier); L2 = second LPA of 5 supersteps "
                                    "on the intra-community distinct edges.  The handle's distinct directed edge "
                                    "set (and, for L2, its (d, s) order) is topology, built by the first call of "
                                    "each kind and kept (outlier_l*_first_ms include it)")
    if keep_host and rank == 0:
        progress("CPU baseline")
        out_json["cpu_baseline"] = cpu_baseline(src_np, dst_np, V, g)
    if quality is not None:
        progress("quality report")
        out_json["quality"] = quality_report(gfa, device, quality["bench_graph"])
    if rank == 0:
        print(json.dumps(out_json), flush=True)
    g.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

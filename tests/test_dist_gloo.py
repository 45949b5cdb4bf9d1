"""World-size-2 gloo run of the multi-GPU label-exchange protocol on CPU
(SURVEY.md §8(e) fake backend).

Each rank owns the degree ranks k with k % P == rank (the layout lpa_build.hip
uses: slot = (k % P) * slice + k // P, equal slice lengths), computes the next
labels of its owned slots only, and the replicated vector is refreshed with ONE
all_gather of the owned slices in rank order -- the same collective the library
issues (ncclAllGather of `slice` int32 per rank).  The oracle superstep stands in
for the device tally (test infrastructure); the test checks that the protocol
reproduces the single-process supersteps bit for bit.

Also: all three exchange forms of lpa_exchange.hip (full, changed-label delta,
giant-compressed), chosen per superstep by the library's byte rule, across two gloo
processes (CPU); and (-m gpu) the library's own caller-driven full / delta entry
points driven from two processes, one rank handle each, payloads moved by gloo.
"""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from graphs import degree_mix

STEPS = 4


def _layout(deg, P):
    V = deg.size
    order = np.lexsort((np.arange(V), -deg))           # degree desc, id asc
    S = ((V + P - 1) // P + 63) // 64 * 64
    slot_of = np.empty(V, np.int64)
    k = np.arange(V)
    slot_of[order] = (k % P) * S + k // P
    return S, slot_of


def _worker(rank, P, port, V, s, d, ref, q):
    from oracle import oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=P)
    try:
        deg = np.bincount(s, minlength=V) + np.bincount(d, minlength=V)
        S, slot_of = _layout(deg, P)
        vertex_of_slot = np.full(P * S, -1, np.int64)
        vertex_of_slot[slot_of] = np.arange(V)
        own = vertex_of_slot[rank * S:(rank + 1) * S]
        rp, col = oracle.build_csr(V, s, d)
        full = np.full(P * S, -1, np.int32)               # replicated vector (slot order)
        full[slot_of] = np.arange(V, dtype=np.int32)      # L0[v] = v
        ok = True
        for t in range(STEPS):
            cur = full[slot_of]                            # dense view of the replica
            nxt = oracle.superstep_csr(rp, col, cur)       # stand-in for the device tally
            mine = np.full(S, -1, np.int32)
            m = own >= 0
            mine[m] = nxt[own[m]]                          # only the owned slots are written
            parts = [torch.empty(S, dtype=torch.int32) for _ in range(P)]
            dist.all_gather(parts, torch.from_numpy(mine))
            full = torch.cat(parts).numpy()
            ok = ok and bool(np.array_equal(full[slot_of], ref[t]))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("P", [2])
def test_gloo_allgather_protocol_matches_single_process(oracle, P):
    V, s, d = degree_mix(3)
    _, ref, _ = oracle.lpa(V, s, d, STEPS, per_iter=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 2000)
    procs = [ctx.Process(target=_worker, args=(r, P, port, V, s, d, ref, q)) for r in range(P)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(P))
    for p in procs:
        p.join(timeout=60)
    assert all(res[r] for r in range(P)), res


# ---------------------------------------------------------------------------
# The three exchange forms of lpa_exchange.hip exchange_collective across real
# process boundaries: full slices (the superstep after L0), changed-label deltas and the
# giant-compressed form (bitmap of label == G + changed non-G entries), chosen per
# superstep by the same byte rule from one all_gather of every rank's (delta, giant)
# count pair; variable-length payloads padded to the largest rank's count as the
# library's allgather does.  The oracle superstep stands in for the device tally.
# ---------------------------------------------------------------------------
FORM_STEPS = 6


def _gather(x):
    parts = [torch.empty_like(x) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, x)
    return parts


def _giant_pick(full, slot_of, order):
    """k_giant_pick: the most frequent label among the 1,024 highest-degree vertices
    (ties to the smallest label)."""
    top = full[slot_of[order[:1024]]]
    vals, cnt = np.unique(top, return_counts=True)
    return int(vals[np.argmax(cnt)])


def _forms_worker(rank, P, port, V, s, d, ref, q):
    from oracle import oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=P)
    try:
        deg = np.bincount(s, minlength=V) + np.bincount(d, minlength=V)
        order = np.lexsort((np.arange(V), -deg))
        S, slot_of = _layout(deg, P)
        wpr, dcap = S // 64, max(1, S // 4)
        vertex_of_slot = np.full(P * S, -1, np.int64)
        vertex_of_slot[slot_of] = np.arange(V)
        own = vertex_of_slot[rank * S:(rank + 1) * S]
        rp, col = oracle.build_csr(V, s, d)
        full = np.full(P * S, -1, np.int32)
        full[slot_of] = np.arange(V, dtype=np.int32)
        ok, forms = True, []
        for t in range(FORM_STEPS):
            nxt = oracle.superstep_csr(rp, col, full[slot_of])
            prev_own = full[rank * S:(rank + 1) * S]
            mine = prev_own.copy()
            m = own >= 0
            mine[m] = nxt[own[m]]
            if t == 0:
                form = "full"
            else:
                G = _giant_pick(full, slot_of, order)
                chg = np.nonzero(mine != prev_own)[0]
                ent = (chg.astype(np.uint64) << np.uint64(32)) | mine[chg].astype(np.uint32).astype(np.uint64)
                ng = chg[mine[chg] != G]
                gent = (ng.astype(np.uint64) << np.uint64(32)) | mine[ng].astype(np.uint32).astype(np.uint64)
                pairs = _gather(torch.tensor([ent.size, gent.size], dtype=torch.int64))
                capd = max(int(p[0]) for p in pairs)
                capg = max(int(p[1]) for p in pairs)
                full_b = 4 * S
                delta_b = 8 * capd if capd <= dcap else 1 << 62
                giant_b = 8 * wpr + 8 * capg if capg <= dcap else 1 << 62
                form = ("delta" if delta_b <= giant_b and delta_b < full_b
                        else "giant" if giant_b < full_b else "full")
            new = full.copy()
            if form == "full":
                for r, p in enumerate(_gather(torch.from_numpy(mine))):
                    new[r * S:(r + 1) * S] = p.numpy()
            else:
                cap, e = (capd, ent) if form == "delta" else (capg, gent)
                if form == "giant":
                    bits = np.packbits((mine == G).astype(np.uint8), bitorder="little")
                    for r, p in enumerate(_gather(torch.from_numpy(bits))):
                        if r != rank:
                            isg = np.unpackbits(p.numpy(), bitorder="little")[:S].astype(bool)
                            sl = new[r * S:(r + 1) * S]
                            sl[isg] = G
                counts = [int(p[0] if form == "delta" else p[1]) for p in pairs]
                pad = np.zeros(max(cap, 1), np.uint64)
                pad[:e.size] = e
                for r, p in enumerate(_gather(torch.from_numpy(pad.view(np.int64)))):
                    got = p.numpy().view(np.uint64)[:counts[r]]
                    slots = (got >> np.uint64(32)).astype(np.int64)
                    new[r * S + slots] = (got & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32)
                new[rank * S:(rank + 1) * S] = mine
            full = new
            forms.append(form)
            ok = ok and bool(np.array_equal(full[slot_of], ref[t]))
        q.put((rank, ok, forms))
    finally:
        dist.destroy_process_group()


def test_gloo_three_exchange_forms_match_single_process(oracle):
    """World size 2: every superstep's replica after the exchange equals the single-process
    labels, and the run uses all three forms (R-MAT-12: full, giant, giant, delta ...)."""
    P = 2
    s, d = oracle.gen_rmat(12, 16, 1, True)
    V = 1 << 12
    _, ref, _ = oracle.lpa(V, s, d, FORM_STEPS, per_iter=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31500 + (os.getpid() % 2000)
    procs = [ctx.Process(target=_forms_worker, args=(r, P, port, V, s, d, ref, q)) for r in range(P)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(P):
        r, ok, forms = q.get(timeout=180)
        res[r] = (ok, forms)
    for p in procs:
        p.join(timeout=60)
    assert all(res[r][0] for r in range(P)), res
    assert res[0][1] == res[1][1], res          # every rank took the same form
    assert set(res[0][1]) == {"full", "delta", "giant"}, res[0][1]


# ---------------------------------------------------------------------------
# The library's own caller-driven exchange (lpa_exchange_get / put and
# lpa_exchange_get_delta / put_delta, the delta protocol the in-library collective
# runs) across two real processes: each process holds one rank's handle of a
# two-rank partition on the GPU and the host moves the payloads with gloo.
# ---------------------------------------------------------------------------
LIB_STEPS = 8


def _lib_worker(rank, P, port, V, s, d, ref, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=P)
    try:
        import graphframes_amd as gfa

        g = gfa.Graph(s, d, V, rank=rank, nranks=P)
        dcap = max(1, g.info()["slice"] // 4)
        ok, forms = True, []
        for t in range(LIB_STEPS):
            g.step(1)
            if t > 0:
                e = g.exchange_get_delta()
                pairs = _gather(torch.tensor([e.size], dtype=torch.int64))
                counts = [int(p[0]) for p in pairs]
            if t > 0 and max(counts) <= dcap:
                pad = np.zeros(max(max(counts), 1), np.uint64)
                pad[:e.size] = e
                parts = _gather(torch.from_numpy(pad.view(np.int64)))
                g.exchange_put_delta([p.numpy().view(np.uint64)[:counts[r]] for r, p in enumerate(parts)])
                forms.append("delta")
            else:
                parts = _gather(torch.from_numpy(g.exchange_get()))
                g.exchange_put(torch.cat(parts).numpy())
                forms.append("full")
            ok = ok and bool(np.array_equal(g.labels(), ref[t]))
        g.close()
        q.put((rank, ok, forms))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_gloo_library_delta_exchange_two_processes(oracle):
    """Two processes, one rank handle each (R-MAT-14 on the one GPU): the library's full
    and delta exchange entry points, payloads moved by gloo, labels bit-exact per
    superstep on both ranks and both forms used."""
    P = 2
    s, d = oracle.gen_rmat(14, 16, 2, True)
    V = 1 << 14
    _, ref, _ = oracle.lpa(V, s, d, LIB_STEPS, per_iter=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 33500 + (os.getpid() % 2000)
    procs = [ctx.Process(target=_lib_worker, args=(r, P, port, V, s, d, ref, q)) for r in range(P)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(P):
        r, ok, forms = q.get(timeout=240)
        res[r] = (ok, forms)
    for p in procs:
        p.join(timeout=60)
    assert all(res[r][0] for r in range(P)), res
    assert set(res[0][1]) == {"full", "delta"}, res[0][1]


# ---------------------------------------------------------------------------
# The library's IN-LIBRARY exchange (lpa_exchange.hip exchange_collective -- the code an
# RCCL rank runs: the per-rank count triple, the full / delta / giant-compressed forms,
# the posted delta and its stand-down) across two real processes: each handle is built
# with lpa_graph_create_hostcoll and its allgathers are done by torch.distributed gloo
# on the host (the giant and posted forms across a
# process boundary, and a posted capacity set on ONE rank only).
# ---------------------------------------------------------------------------
HC_STEPS = 10


def _gloo_allgather_bytes(send):
    """Every rank's `send` bytes in rank order (gloo all_gather on int32 words)."""
    n = send.size
    x = torch.from_numpy(send.view(np.int32) if n % 4 == 0 else send)
    parts = _gather(x)
    return b"".join(p.numpy().tobytes() for p in parts)


def _hostcoll_worker(rank, P, port, V, s, d, ref, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=P)
    try:
        import graphframes_amd as gfa

        out = {}
        with gfa.Graph(s, d, V, rank=rank, nranks=P, allgather=_gloo_allgather_bytes) as g:
            ok = True
            for t in range(HC_STEPS):
                g.step(1)
                ok = ok and bool(np.array_equal(g.labels(), ref[t]))
            out["steps_ok"] = ok
            out["forms"] = {k: g.info()[k] for k in ("exchanges_full", "exchanges_delta", "exchanges_giant",
                                                     "exchanges_posted", "exchanges_post_missed",
                                                     "host_allgathers")}
            # a posted capacity of 1 requested by rank 0 ONLY: the ranks agree on the
            # smallest request (it travels with the count triple), so both post the same
            # allgather size and the queued apply stands down on both
            before = g.info()
            if rank == 0:
                g.set_posted(1)
            runs_ok = bool(np.array_equal(g.run(HC_STEPS), ref[HC_STEPS - 1]))
            after = g.info()
            out["missed_p1"] = after["exchanges_post_missed"] - before["exchanges_post_missed"]
            # back to adaptive on rank 0: posted exchanges that fit
            if rank == 0:
                g.set_posted(-1)
            before = g.info()
            runs_ok = runs_ok and bool(np.array_equal(g.run(HC_STEPS), ref[HC_STEPS - 1]))
            after = g.info()
            out["posted_adaptive"] = after["exchanges_posted"] - before["exchanges_posted"]
            out["runs_ok"] = runs_ok
        q.put((rank, out))
    except BaseException as e:  # noqa: BLE001 -- reported to the parent
        q.put((rank, {"error": repr(e)}))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_gloo_host_collective_in_library_exchange_two_processes(oracle):
    """Two processes, one hostcoll rank handle each (R-MAT-16 on the one GPU): every
    superstep bit-exact on both ranks through the library's own exchange schedule with
    gloo as the transport; the full, delta, giant and posted forms all ran, a posted
    capacity set on one rank alone stood down identically on both, and lpa_run(10)
    is bit-exact after each setting."""
    P = 2
    s, d = oracle.gen_rmat(16, 16, 3, True)
    V = 1 << 16
    _, ref, _ = oracle.lpa(V, s, d, HC_STEPS, per_iter=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 35500 + (os.getpid() % 2000)
    procs = [ctx.Process(target=_hostcoll_worker, args=(r, P, port, V, s, d, ref, q)) for r in range(P)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(P):
        r, out = q.get(timeout=240)
        res[r] = out
    for p in procs:
        p.join(timeout=60)
    assert all("error" not in res[r] for r in range(P)), res
    assert all(res[r]["steps_ok"] and res[r]["runs_ok"] for r in range(P)), res
    f = res[0]["forms"]
    assert f == res[1]["forms"], res            # every rank took the same forms
    assert f["exchanges_full"] >= 1 and f["exchanges_delta"] >= 1 and f["exchanges_giant"] >= 1, f
    assert f["exchanges_posted"] >= 1 and f["host_allgathers"] > 0, f
    assert res[0]["missed_p1"] == res[1]["missed_p1"] >= 1, res
    assert res[0]["posted_adaptive"] == res[1]["posted_adaptive"] >= 1, res

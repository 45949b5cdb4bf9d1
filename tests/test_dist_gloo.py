"""World-size-2 gloo run of the multi-GPU label-exchange protocol on CPU
(SURVEY.md §8(e) fake backend).

Each rank owns the degree ranks k with k % P == rank (the layout lpa_build.hip
uses: slot = (k % P) * slice + k // P, equal slice lengths), computes the next
labels of its owned slots only, and the replicated vector is refreshed with ONE
all_gather of the owned slices in rank order -- the same collective the library
issues (ncclAllGather of `slice` int32 per rank).  The oracle superstep stands in
for the device tally (test infrastructure); the test checks that the protocol
reproduces the single-process supersteps bit for bit.
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

"""The RCCL transport of the multi-GPU label exchange on the one-GPU box.

Two RCCL ranks cannot share one device, so the distributed path is driven as a
ONE-rank job: lpa_comm_unique_id -> lpa_graph_create_dist(nranks=1, comm_id) runs
ncclCommInitRank, and every superstep goes through exchange_collective exactly as
at P > 1 (full ncclAllGather in place after L0, then per superstep the (delta, giant)
count pairs allgathered and read on the host and the smaller form sent: the delta
entries, whose gathered change list queues the refresh, or the giant-label bitmap
plus the changed non-giant entries).  Bit-exact against the oracle per
superstep (reference: Graphframes.py:81 labelPropagation, the Spark shuffle
behind aggregateMessages replaced by the allgather).
"""
import os

import numpy as np
import pytest

from graphs import degree_mix

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gfa():
    # a single-node box: RCCL's bootstrap may only find the loopback interface
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    import graphframes_amd

    return graphframes_amd


def _one_rank(gfa, s, d, V):
    cid = gfa.comm_unique_id()
    assert isinstance(cid, (bytes, bytearray)) and len(cid) == 128
    return gfa.Graph(s, d, V, rank=0, nranks=1, comm_id=cid)


@pytest.mark.parametrize("graph", ["rmat16", "degree_mix"])
def test_rccl_one_rank_every_superstep(gfa, oracle, graph):
    if graph == "rmat16":
        s, d = gfa.gen_rmat(16, 16, seed=3)
        V = 1 << 16
        s, d = s.cpu().numpy(), d.cpu().numpy()
    else:
        V, s, d = degree_mix(5)
    _, hist, _ = oracle.lpa(V, s, d, 10, per_iter=True)
    with _one_rank(gfa, s, d, V) as g:
        info = g.info()
        assert info["nranks"] == 1 and info["exchanges_full"] == 0
        for t in range(10):
            g.step(1)
            bad = int((g.labels() != hist[t]).sum())
            assert bad == 0, f"{graph} superstep {t + 1}: {bad} labels differ"
        info = g.info()
        # every transport branch ran: the in-place full allgather after L0, then deltas,
        # and (R-MAT, once its giant label dominates) the giant-compressed form with its
        # bitmap allgather; one exchange per superstep
        assert info["exchanges_full"] >= 1 and info["exchanges_delta"] >= 2, info
        assert info["exchanges_full"] + info["exchanges_delta"] + info["exchanges_giant"] == 10, info
        if graph == "rmat16":
            assert info["exchanges_giant"] >= 1, info
        # lpa_run from reset (captured tally graphs replayed) twice: the same answer
        for _ in range(2):
            assert np.array_equal(g.run(10), hist[9])


def test_rccl_one_rank_matches_local(gfa):
    """The one-rank distributed handle and the single-GPU handle agree on a graph
    large enough for the rebuild, the frontier and the hub paths (R-MAT 20)."""
    s, d = gfa.gen_rmat(20, 16, seed=5)
    V = 1 << 20
    with gfa.Graph(s, d, V) as g:
        ref = g.run(10)
    with _one_rank(gfa, s, d, V) as g:
        got = g.run(10)
        assert g.info()["exchanges_delta"] >= 2
    assert np.array_equal(got, ref)

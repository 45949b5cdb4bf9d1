"""Multi-rank label exchange executed by the library itself.

P handles of an in-process loopback group share one device; each is driven by its
own host thread, exactly as P processes drive their ranks under
torch.distributed.run.  Every superstep goes through the library's own exchange
(lpa_exchange.hip exchange_collective: full allgather in the label-dense
supersteps, then the changed-label delta protocol with its host count read, the
in-place allgather offsets and the previous/next delta chain); only the transport
differs from RCCL (stream-ordered D2D copies, lpa_comm.cpp).  Bit-exact against
the oracle per superstep; reference call: Graphframes.py:81.
"""
import threading
import time

import numpy as np
import pytest

from graphs import degree_mix

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gfa():
    import graphframes_amd

    return graphframes_amd


def _group(gfa, s, d, V, P):
    lb = gfa.Loopback(P)
    return lb, [gfa.Graph(s, d, V, rank=r, loopback=lb) for r in range(P)]


def _close(lb, ranks):
    for g in ranks:
        g.close()
    lb.close()


def _per_step_all_ranks(gfa, ranks, n):
    def work(r, g):
        out = []
        for _ in range(n):
            g.step(1)
            out.append(g.labels())
        return out

    return gfa.run_ranks(ranks, work)


@pytest.mark.parametrize("P", [2, 4, 8])
def test_loopback_rmat18_every_superstep(gfa, oracle, P):
    s, d = gfa.gen_rmat(18, 16, seed=1)
    V = 1 << 18
    s, d = s.cpu().numpy(), d.cpu().numpy()
    _, hist, _ = oracle.lpa(V, s, d, 10, per_iter=True)
    lb, ranks = _group(gfa, s, d, V, P)
    try:
        infos = [g.info() for g in ranks]
        assert sum(i["arcs"] for i in infos) == 2 * s.size
        got = _per_step_all_ranks(gfa, ranks, 10)
        for r in range(P):
            for t in range(10):
                bad = int((got[r][t] != hist[t]).sum())
                assert bad == 0, f"P={P} rank {r} superstep {t + 1}: {bad} labels differ"
        infos = [g.info() for g in ranks]
        # full slices after L0, the giant-compressed form once G dominates (R-MAT
        # supersteps 2-3), deltas when converged
        assert all(i["exchanges_full"] >= 1 and i["exchanges_delta"] >= 2 and i["exchanges_giant"] >= 1
                   for i in infos), infos
        # lpa_run (reset + 10 supersteps) on every rank concurrently: same answer
        runs = gfa.run_ranks(ranks, lambda r, g: g.run(10))
        for r in range(P):
            assert np.array_equal(runs[r], hist[9]), f"P={P} rank {r} lpa_run(10)"
    finally:
        _close(lb, ranks)


@pytest.mark.parametrize("P", [2, 4, 8])
def test_loopback_degree_mix_every_superstep(gfa, oracle, P):
    V, s, d = degree_mix(11)
    _, hist, _ = oracle.lpa(V, s, d, 10, per_iter=True)
    lb, ranks = _group(gfa, s, d, V, P)
    try:
        got = _per_step_all_ranks(gfa, ranks, 10)
        for r in range(P):
            for t in range(10):
                assert np.array_equal(got[r][t], hist[t]), f"P={P} rank {r} superstep {t + 1}"
        assert all(g.info()["exchanges_delta"] >= 2 for g in ranks)
    finally:
        _close(lb, ranks)


@pytest.mark.parametrize("P", [2, 4])
def test_loopback_posted_delta_settings(gfa, oracle, P):
    """The posted delta exchange (lpa_set_posted; converged supersteps send the changed
    labels at a capacity fixed before the host reads the counts): adaptive (default),
    off, a capacity of 1 (nearly every posted exchange overflows: the queued apply
    stands down on the device and the host exchanges again) and a fixed large one --
    every superstep bit-exact on every rank."""
    s, d = gfa.gen_rmat(18, 16, seed=2)
    V = 1 << 18
    s, d = s.cpu().numpy(), d.cpu().numpy()
    _, hist, _ = oracle.lpa(V, s, d, 10, per_iter=True)
    lb, ranks = _group(gfa, s, d, V, P)
    try:
        for cap in (-1, 0, 1, 1 << 20):
            before = [g.info() for g in ranks]
            for g in ranks:
                g.set_posted(cap)
                g.reset()
            got = _per_step_all_ranks(gfa, ranks, 10)
            for r in range(P):
                for t in range(10):
                    bad = int((got[r][t] != hist[t]).sum())
                    assert bad == 0, f"posted={cap} P={P} rank {r} superstep {t + 1}: {bad} labels differ"
            after = [g.info() for g in ranks]
            posted = [a["exchanges_posted"] - b["exchanges_posted"] for a, b in zip(after, before)]
            missed = [a["exchanges_post_missed"] - b["exchanges_post_missed"] for a, b in zip(after, before)]
            assert len(set(posted)) == 1 and len(set(missed)) == 1, (cap, posted, missed)  # same on every rank
            if cap == 0:
                assert posted[0] == 0 and missed[0] == 0
            elif cap == 1:
                assert missed[0] >= 1, (posted, missed)
            else:
                assert posted[0] >= 1, (cap, posted, missed)
    finally:
        _close(lb, ranks)


def test_loopback_abort_releases_waiting_rank(gfa):
    """A rank whose peer never arrives is released by lpa_loopback_abort and fails
    with an error instead of blocking its thread."""
    V, s, d = degree_mix(2)
    lb, ranks = _group(gfa, s, d, V, 2)
    try:
        err = []

        def lone():
            try:
                ranks[0].run(3)
            except Exception as e:  # noqa: BLE001
                err.append(e)

        th = threading.Thread(target=lone)
        th.start()
        time.sleep(1.0)
        assert th.is_alive()            # blocked in the superstep-1 allgather
        lb.abort()
        th.join(timeout=60)
        assert not th.is_alive() and err and "loopback" in str(err[0])
    finally:
        _close(lb, ranks)


def test_loopback_p8_rmat22_every_superstep(gfa, oracle):
    """P = 8 at R-MAT scale 22 (4 M V / 67 M E): the delta chain runs with realistic
    change counts (tens of thousands per rank in the converging supersteps) and the
    ranked (power-of-two) hot-set rebuild with its bits mode, every superstep bit-exact."""
    s, d = gfa.gen_rmat(22, 16, seed=1)
    V = 1 << 22
    s, d = s.cpu().numpy(), d.cpu().numpy()
    _, hist, _ = oracle.lpa(V, s, d, 10, per_iter=True)
    lb, ranks = _group(gfa, s, d, V, 8)
    try:
        got = _per_step_all_ranks(gfa, ranks, 10)
        for r in range(8):
            for t in range(10):
                bad = int((got[r][t] != hist[t]).sum())
                assert bad == 0, f"P=8 rank {r} superstep {t + 1}: {bad} labels differ"
        infos = [g.info() for g in ranks]
        assert all(i["exchanges_full"] >= 1 and i["exchanges_delta"] >= 2 and i["exchanges_giant"] >= 1
                   for i in infos), infos
        assert all(i["exchanges_full"] + i["exchanges_delta"] + i["exchanges_giant"] == 10 for i in infos)
    finally:
        _close(lb, ranks)


def test_loopback_close_before_graphs(gfa):
    """Loopback.close() while its handles are still open defers the free to the last
    handle's destroy (no use-after-free); the handles' later close() works."""
    V, s, d = degree_mix(3)
    lb, ranks = _group(gfa, s, d, V, 2)
    lb.close()
    for g in ranks:
        g.close()

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

from graphs import code_mix, degree_mix

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


@pytest.fixture(scope="module")
def codemix22(gfa, oracle):
    s, d = gfa.gen_rmat(22, 16, seed=11)
    V, sn, dn = code_mix(s.cpu().numpy(), d.cpu().numpy(), 1 << 22)
    _, hist, _ = oracle.lpa(V, sn, dn, 5, per_iter=True)
    return V, sn, dn, hist


@pytest.mark.parametrize("P,lbin", [(2, None), (4, None), (2, "8")])
def test_loopback_giant_codes_every_rank(gfa, codemix22, monkeypatch, P, lbin):
    """Round 6: the giant-code refresh after superstep 1 and superstep 2's settle from the
    2-bit codes on EVERY rank of a partitioned job (each rank codes its own arcs against
    the G of the replicated vector, the rank-strided LDS hot sets), with every exact
    fallback populated (tests/graphs.py code_mix: wave-bin rows, block-tier hub rows and
    > 8192-arc hub rows whose mode is not G) -- bit-exact on every rank at supersteps 1..5,
    the code refresh asserted on every rank.  lbin "8": the cut that codes the rows of
    9-64 arcs too (LPA_CODE_LBIN; C4 / C5 take it by size), whose coded row bins walk
    the code settle's lists on the third stream."""
    if lbin:
        monkeypatch.setenv("LPA_CODE_LBIN", lbin)
    V, sn, dn, hist = codemix22
    lb, ranks = _group(gfa, sn, dn, V, P)
    try:
        assert all(g.info()["slice"] & (g.info()["slice"] - 1) == 0 for g in ranks)   # power-of-two slices

        def work(r, g):
            out, codes = [], []
            for t in range(5):
                g.step(1)
                if t == 0:
                    codes.append(g.info()["code_refresh"])
                out.append(int((g.labels() != hist[t]).sum()))
            return out, codes

        res = gfa.run_ranks(ranks, work)
        for r in range(P):
            assert res[r][0] == [0] * 5, f"P={P} rank {r} labels differing per superstep {res[r][0]}"
            assert res[r][1] == [1], f"P={P} rank {r}: the giant-code refresh was not taken"
        runs = gfa.run_ranks(ranks, lambda r, g: g.run(5))
        for r in range(P):
            assert np.array_equal(runs[r], hist[4]), f"P={P} rank {r} lpa_run(5)"
    finally:
        _close(lb, ranks)


def test_code_cut_g8_single_gpu(gfa, codemix22, monkeypatch):
    """the code_lbin = g8 schedule (the rows of 9-64 arcs coded; their row
    bins walk the code settle's lists after ev_join2[2], k_code_partial_rows fills their
    al[]) on a graph small enough for the fast suite -- forced by LPA_CODE_LBIN=8 --
    bit-exact at supersteps 1..5, then lpa_run(5) twice (replayed graphs)."""
    monkeypatch.setenv("LPA_CODE_LBIN", "8")
    V, sn, dn, hist = codemix22
    with gfa.Graph(sn, dn, V) as g:
        for t in range(5):
            g.step(1)
            if t == 0:
                assert g.info()["code_refresh"] == 1
            bad = int((g.labels() != hist[t]).sum())
            assert bad == 0, f"g8 cut superstep {t + 1}: {bad} labels differ"
        for _ in range(2):
            g.reset()
            assert np.array_equal(g.run(5), hist[4])


@pytest.mark.parametrize("env", [{"LPA_GIANT_CODES": "0"}, {"LPA_POW2_SLICES": "0"}])
def test_round6_switches_bit_exact(gfa, codemix22, monkeypatch, env):
    """The round-6 switches: no giant-code refresh (LPA_GIANT_CODES=0:
    the labels- / bits-mode rebuilds only), and tight slices at P > 1 (LPA_POW2_SLICES=0:
    ceil(V / P) slots per rank, so the plain rebuild and no codes) -- bit-exact at
    supersteps 1..5 on one GPU and on a P = 2 loopback group."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    V, sn, dn, hist = codemix22
    with gfa.Graph(sn, dn, V) as g:
        for t in range(5):
            g.step(1)
            if t == 0 and "LPA_GIANT_CODES" in env:
                assert g.info()["code_refresh"] == 0
            assert np.array_equal(g.labels(), hist[t]), f"{env} one GPU superstep {t + 1}"
    lb, ranks = _group(gfa, sn, dn, V, 2)
    try:
        S = ranks[0].info()["slice"]
        assert (S & (S - 1) == 0) == ("LPA_POW2_SLICES" not in env), S
        got = _per_step_all_ranks(gfa, ranks, 5)
        for r in range(2):
            for t in range(5):
                assert np.array_equal(got[r][t], hist[t]), f"{env} P=2 rank {r} superstep {t + 1}"
        assert all(g.info()["code_refresh"] == 0 for g in ranks)
    finally:
        _close(lb, ranks)

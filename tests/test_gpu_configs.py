"""BASELINE.json configs at their FULL sizes, bit-exact against the CPU oracle at every
superstep (SURVEY.md §8(d) workloads; reference call: Graphframes.py:81
``labelPropagation(maxIter)``; the partitioned forms stand in for the Spark
``local[*]`` parallelism of Graphframes.py:12 and the shuffle behind :81).

  C3  R-MAT scale 24, edgefactor 16 (16.7 M V / 268 M E): supersteps 1..10 from L0,
      plus lpa_run(10) as a user calls it
  C4  R-MAT scale 26, edgefactor 16 (67 M V / 1.07 B E, 2.1 B arcs): one GPU, and as
      configured -- vertex-partitioned over P = 2, 4 and 8 ranks (an in-process
      loopback group on the one GPU: the library's own exchange code, full allgather
      and changed-label deltas, with D2D copies in place of ncclAllGather)
  C5  Chung-Lu gamma 2.1, 40 M V / 1.4 B E (2.8 B arcs, max degree ~1.25 M): one GPU,
      and as configured -- partitioned over P = 8 ranks
  C2  SBM 1 M V / 20 M E: the outlier stage (L1 / L2)

Every superstep of every rank is compared with the oracle's history; the oracle here
is oracle/lpa_oracle.c (OpenMP), the checker only.  Each oracle history is computed
once per module (a fixture) and shared by the single-GPU and the partitioned tests.
"""
import time

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

MAX_ITER = 10


@pytest.fixture(scope="module")
def gfa():
    import graphframes_amd

    return graphframes_amd


def _host(t):
    return t.cpu().numpy()


def _mismatch_per_step(g, hist, n, codes=None):
    """Steps the handle n times; the number of labels that differ at each superstep.
    codes (a list): gets code_refresh after supersteps 1 and 2 (whether that refresh
    took the giant codes)."""
    bad = []
    for t in range(n):
        g.step(1)
        if codes is not None and t < 2:
            codes.append(int(g.info()["code_refresh"]))
        bad.append(int((g.labels() != hist[t]).sum()))
    return bad


class _Config:
    """Host edge list + the oracle's per-superstep history of one config."""

    def __init__(self, V, src, dst, oracle):
        self.V, self.src, self.dst = V, src, dst
        t0 = time.perf_counter()
        _, self.hist, _ = oracle.lpa(V, src, dst, MAX_ITER, per_iter=True)
        self.oracle_s = time.perf_counter() - t0


@pytest.fixture(scope="module")
def c4(gfa, oracle):
    s, d = gfa.gen_rmat(26, 16, seed=1)
    src, dst = _host(s), _host(d)
    del s, d
    return _Config(1 << 26, src, dst, oracle)


@pytest.fixture(scope="module")
def c5(gfa, oracle):
    s, d = gfa.gen_chunglu(40_000_000, 1_400_000_000, 2.1, 1.25e6, seed=7)
    src, dst = _host(s), _host(d)
    del s, d
    return _Config(40_000_000, src, dst, oracle)


def _empty_cache():
    import torch

    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def _partitioned_every_superstep(gfa, cfg, P, what, code_after):
    """A loopback group of P ranks on the one GPU, built from the same edge list (as
    P processes of `bench.py --gpus P` build theirs), every rank checked against the
    oracle at every superstep 1..10, then lpa_run(10) on every rank concurrently.
    code_after (1 or 2): every rank's refresh after that superstep took the giant codes
    (round 6: the code refresh and settle on every rank of a partitioned job)."""
    import torch

    lb = gfa.Loopback(P)
    ranks = []
    try:
        dev_s = torch.from_numpy(cfg.src).cuda()
        dev_d = torch.from_numpy(cfg.dst).cuda()
        for r in range(P):
            ranks.append(gfa.Graph(dev_s, dev_d, cfg.V, rank=r, loopback=lb))
        del dev_s, dev_d
        _empty_cache()
        infos = [g.info() for g in ranks]
        assert sum(i["arcs"] for i in infos) == 2 * cfg.src.size
        codes = [[] for _ in range(P)]
        bad = gfa.run_ranks(ranks, lambda r, g: _mismatch_per_step(g, cfg.hist, MAX_ITER, codes[r]))
        for r in range(P):
            for t in range(MAX_ITER):
                assert bad[r][t] == 0, f"{what} P={P} rank {r} superstep {t + 1}: {bad[r][t]} labels differ"
        assert all(c[code_after - 1] == 1 for c in codes), f"{what} P={P} code refresh per rank: {codes}"
        infos = [g.info() for g in ranks]
        # full slices after L0, giant-compressed (bitmap + changed non-giant labels) once
        # G dominates, changed-label deltas when converged: one exchange per superstep
        assert all(i["exchanges_full"] >= 1 and i["exchanges_delta"] >= 2 and i["exchanges_giant"] >= 1
                   for i in infos), infos
        assert all(i["exchanges_full"] + i["exchanges_delta"] + i["exchanges_giant"] == MAX_ITER for i in infos)
        # the converged supersteps replayed each rank's captured tally graph (the path an
        # RCCL rank runs; a loopback group captures too since round 5)
        assert all(i["graph_replays"] >= 1 for i in infos), [i["graph_replays"] for i in infos]
        runs = gfa.run_ranks(ranks, lambda r, g: int((g.run(MAX_ITER) != cfg.hist[MAX_ITER - 1]).sum()))
        assert runs == [0] * P, f"{what} P={P} lpa_run(10) mismatches per rank: {runs}"
    finally:
        for g in ranks:
            g.close()
        lb.close()
        _empty_cache()


def test_c3_rmat24_every_superstep(gfa, oracle):
    import torch

    scale = 24
    V = 1 << scale
    s, d = gfa.gen_rmat(scale, 16, seed=1)
    with gfa.Graph(s, d, V) as g:
        sn, dn = _host(s), _host(d)
        del s, d
        torch.cuda.empty_cache()
        got = []
        for _ in range(MAX_ITER):
            g.step(1)
            got.append(g.labels())
        run10 = g.run(MAX_ITER)
    t0 = time.perf_counter()
    _, hist, _ = oracle.lpa(V, sn, dn, MAX_ITER, per_iter=True)
    t_or = time.perf_counter() - t0
    for t in range(MAX_ITER):
        bad = int((got[t] != hist[t]).sum())
        assert bad == 0, f"C3 superstep {t + 1}: {bad} labels differ (oracle {t_or:.1f}s)"
    assert np.array_equal(run10, hist[MAX_ITER - 1]), "C3 lpa_run(10) differs from superstep-by-superstep"


def test_c4_rmat26_every_superstep(gfa, c4):
    import torch

    dev_s = torch.from_numpy(c4.src).cuda()
    dev_d = torch.from_numpy(c4.dst).cuda()
    with gfa.Graph(dev_s, dev_d, c4.V) as g:
        assert g.info()["arcs"] == 2 * (16 << 26)   # > 2^31: int64 row offsets
        del dev_s, dev_d
        _empty_cache()
        codes = []
        bad = _mismatch_per_step(g, c4.hist, MAX_ITER, codes)
    _empty_cache()
    assert bad == [0] * MAX_ITER, f"C4 one GPU: labels differing per superstep {bad}"
    assert codes[0] == 1, codes


@pytest.mark.parametrize("P", [2, 4, 8])
def test_c4_rmat26_partitioned_every_superstep(gfa, c4, P):
    """BASELINE C4 as configured: R-MAT-26 vertex-partitioned over P ranks."""
    _partitioned_every_superstep(gfa, c4, P, "C4", code_after=1)


def test_c5_chunglu_every_superstep(gfa, c5):
    """C5 on one GPU, every superstep (the giant decision, the hub bucket path and the
    settles of supersteps 2-4 on 1 M-arc hub rows)."""
    import torch

    dev_s = torch.from_numpy(c5.src).cuda()
    dev_d = torch.from_numpy(c5.dst).cuda()
    with gfa.Graph(dev_s, dev_d, c5.V) as g:
        assert g.info()["max_degree"] > 1_000_000   # the hub-bin spill path is exercised
        del dev_s, dev_d
        _empty_cache()
        codes = []
        bad = _mismatch_per_step(g, c5.hist, MAX_ITER, codes)
        run10 = int((g.run(MAX_ITER) != c5.hist[MAX_ITER - 1]).sum())
    _empty_cache()
    assert bad == [0] * MAX_ITER, f"C5 one GPU: labels differing per superstep {bad}"
    assert codes[1] == 1, codes   # Chung-Lu: L2 is the first vector with a giant on the hubs
    assert run10 == 0, f"C5 lpa_run(10): {run10} labels differ"


def test_c5_chunglu_partitioned_p8_every_superstep(gfa, c5):
    """BASELINE C5 as configured: the heavy-hub graph over 8 ranks."""
    _partitioned_every_superstep(gfa, c5, 8, "C5", code_after=2)


def test_c2_outlier_l1_l2_vs_oracle(gfa, oracle):
    """Outlier stage (Graphframes.py:92-137) at config C2 size (SBM
    1 M V / 20 M E, labels after maxIter=10): size / incident histograms, thresholds,
    L2 sub-labels and flags identical to the oracle."""
    V, B, m = 1_000_000, 100, 20_000_000
    s, d = gfa.gen_sbm(V, B, m)
    sn, dn = _host(s), _host(d)
    with gfa.Graph(s, d, V) as g:
        lab = g.run(10)
        o1 = g.outlier(lab, "L1")
        o2 = g.outlier(lab, "L2", sub_iter=5)
    size, inc, flags, summ = oracle.outlier_l1(V, sn, dn, lab)
    assert np.array_equal(o1["size"], size) and np.array_equal(o1["incident"], inc)
    assert np.array_equal(o1["flags"], flags) and o1["summary"]["threshold"] == summ["thr"]
    assert o1["summary"]["n_groups"] == summ["n_groups"] and o1["summary"]["n_flagged"] == summ["n_flagged"]
    sub, flags2, summ2 = oracle.outlier_l2(V, sn, dn, lab, 5)
    assert np.array_equal(o2["sub_labels"], sub) and np.array_equal(o2["flags"], flags2)
    assert o2["summary"]["n_flagged"] == summ2["n_flagged"]
    assert o2["summary"]["n_groups"] == summ2["n_subgroups"]
    assert o2["summary"]["n_communities_flagged"] == summ2["n_communities_flagged"]

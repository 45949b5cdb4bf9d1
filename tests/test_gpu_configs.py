"""BASELINE.json configs at their FULL sizes on one MI355X, bit-exact against the CPU
oracle (SURVEY.md §8(d) workloads; reference call: Graphframes.py:81
``labelPropagation(maxIter)``).

  C3  R-MAT scale 24, edgefactor 16 (16.7 M V / 268 M E): supersteps 1..10 from L0,
      every superstep, plus lpa_run(10) as a user calls it
  C4  R-MAT scale 26, edgefactor 16 (67 M V / 1.07 B E, 2.1 B arcs) on ONE GPU (the
      config is quoted on 2/4/8 GPUs; the partitioned path is bit-identical by
      construction and tested separately): supersteps 1..10 from L0 (the giant
      decision, the row settle, the frontier and the scatter paths at 2.1 B arcs)
  C5  Chung-Lu gamma 2.1, 40 M V / 1.4 B E (2.8 B arcs, max degree ~1.25 M) on ONE
      GPU: lpa_run(maxIter=10) final labels

The oracle here is oracle/lpa_oracle.c (OpenMP), the checker only.
"""
import time

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


@pytest.fixture(scope="module")
def gfa():
    import graphframes_amd

    return graphframes_amd


def _host(t):
    return t.cpu().numpy()


def _steps(g, n):
    out = []
    for _ in range(n):
        g.step(1)
        out.append(g.labels())
    return out


def test_c3_rmat24_every_superstep(gfa, oracle):
    import torch

    scale = 24
    V = 1 << scale
    s, d = gfa.gen_rmat(scale, 16, seed=1)
    with gfa.Graph(s, d, V) as g:
        sn, dn = _host(s), _host(d)
        del s, d
        torch.cuda.empty_cache()
        got = _steps(g, 10)
        run10 = g.run(10)
    t0 = time.perf_counter()
    _, hist, _ = oracle.lpa(V, sn, dn, 10, per_iter=True)
    t_or = time.perf_counter() - t0
    for t in range(10):
        bad = int((got[t] != hist[t]).sum())
        assert bad == 0, f"C3 superstep {t + 1}: {bad} labels differ (oracle {t_or:.1f}s)"
    assert np.array_equal(run10, hist[9]), "C3 lpa_run(10) differs from superstep-by-superstep"


def test_c4_rmat26_every_superstep(gfa, oracle):
    import torch

    scale = 26
    V = 1 << scale
    s, d = gfa.gen_rmat(scale, 16, seed=1)
    with gfa.Graph(s, d, V) as g:
        assert g.info()["arcs"] == 2 * (16 << scale)   # > 2^31: int64 row offsets
        sn, dn = _host(s), _host(d)
        del s, d
        torch.cuda.empty_cache()
        got = _steps(g, 10)
    _, hist, _ = oracle.lpa(V, sn, dn, 10, per_iter=True)
    del sn, dn
    for t in range(10):
        bad = int((got[t] != hist[t]).sum())
        assert bad == 0, f"C4 superstep {t + 1}: {bad} labels differ"


def test_c5_chunglu_full_maxiter10(gfa, oracle):
    import torch

    V, m = 40_000_000, 1_400_000_000
    s, d = gfa.gen_chunglu(V, m, 2.1, 1.25e6, seed=7)
    with gfa.Graph(s, d, V) as g:
        info = g.info()
        assert info["max_degree"] > 1_000_000   # the hub-bin spill path is exercised
        sn, dn = _host(s), _host(d)
        del s, d
        torch.cuda.empty_cache()
        lab = g.run(10)
    ref = oracle.lpa(V, sn, dn, 10)
    del sn, dn
    bad = int((lab != ref).sum())
    assert bad == 0, f"C5 maxIter=10: {bad} labels differ"


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

"""GPU parity: liblpa_hip.so (through its C ABI) vs the CPU oracle and the
committed golden fixture.  Bit-exact labels per superstep (integer path)."""
import numpy as np
import pandas as pd
import pytest

from graphs import (adversarial_hub, degree_mix, giant_hub, random_multigraph, settled_hubs, stale_units, star,
                    two_cliques)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gfa():
    import graphframes_amd

    return graphframes_amd


def _per_step(gfa, V, s, d, iters):
    out = []
    with gfa.Graph(s, d, V) as g:
        for _ in range(iters):
            g.step(1)
            out.append(g.labels())
    return np.stack(out) if out else np.empty((0, V), np.int32)


def test_r9_golden_every_superstep(gfa, golden):
    V = golden["ids"].size
    got = _per_step(gfa, V, golden["src"], golden["dst"], 10)
    for t in range(10):
        bad = int((got[t] != golden["labels_iter"][t]).sum())
        assert bad == 0, f"superstep {t + 1}: {bad} labels differ"


def test_r9_run_matches_step(gfa, golden):
    V = golden["ids"].size
    with gfa.Graph(golden["src"], golden["dst"], V) as g:
        lab, st = g.run(5, stats=True)
        assert st["iters"] == 5 and len(st["iter_ms"]) == 5
        assert np.array_equal(lab, golden["labels_iter"][4])
        # run() resets: a second call gives the same answer
        assert np.array_equal(g.run(5), lab)


def test_two_cliques_kat(gfa):
    V, s, d = two_cliques()
    with gfa.Graph(s, d, V) as g:
        lab = g.run(20)
    assert lab.tolist() == [0] * 5 + [5] * 6


def test_star_oscillates(gfa):
    V, s, d = star(40)
    got = _per_step(gfa, V, s, d, 4)
    assert (got[0][1:] == 0).all() and got[0][0] == 1
    assert (got[1][1:] == 1).all() and got[1][0] == 0
    assert np.array_equal(got[2], got[0]) and np.array_equal(got[3], got[1])


def test_edge_cases(gfa, oracle):
    # self-loop = 2 votes for own label; duplicates counted; isolated keep label
    V = 6
    s = np.array([0, 0, 1, 1, 1, 2], np.int32)
    d = np.array([0, 1, 2, 2, 3, 4], np.int32)
    with gfa.Graph(s, d, V) as g:
        for it in (1, 2, 3, 7):
            assert np.array_equal(g.run(it), oracle.lpa(V, s, d, it))
    # edgeless graph: every label stays
    with gfa.Graph(np.zeros(0, np.int32), np.zeros(0, np.int32), 4) as g:
        assert g.run(3).tolist() == [0, 1, 2, 3]
    # single vertex with a self loop
    with gfa.Graph(np.zeros(1, np.int32), np.zeros(1, np.int32), 1) as g:
        assert g.run(2).tolist() == [0]


@pytest.mark.parametrize("seed", [0, 1])
def test_first_superstep_runs_cross_tiles(gfa, oracle, seed):
    """Superstep 1 by column runs (k_first_runs): duplicate-edge runs of up to a few
    thousand arcs that cross the 512-arc run tiles, ties between equal-length runs (the
    smallest label wins), self-loop runs, rows of every length from 1 to ~20 K arcs
    crossing tiles at every offset.  Bit-exact vs the oracle for supersteps 1-3, and
    identical with the column-run path off (LPA_FIRST_RUNS=0)."""
    rng = np.random.default_rng(seed)
    V = 30_000
    parts = []
    hubs = rng.choice(V, 12, replace=False)
    for h in hubs:
        nb = rng.choice(V, int(rng.integers(50, 20_000)), replace=True)   # some repeats
        parts.append(np.stack([np.full(nb.size, h), nb]))
        for _ in range(4):                                              # long duplicate runs
            u = int(rng.integers(0, V))
            k = int(rng.integers(300, 3_000))
            parts.append(np.stack([np.full(k, h), np.full(k, u)]))
        parts.append(np.stack([np.full(700, h), np.full(700, h)]))      # self-loop run
    # two equal-length runs: the smaller label must win
    parts.append(np.stack([np.full(900, hubs[0]), np.full(900, 7)]))
    parts.append(np.stack([np.full(900, hubs[0]), np.full(900, 5)]))
    m_rand = 200_000
    parts.append(rng.integers(0, V, size=(2, m_rand)))
    e = np.concatenate(parts, axis=1).astype(np.int32)
    s, d = e[0].copy(), e[1].copy()
    _, hist, _ = oracle.lpa(V, s, d, 3, per_iter=True)
    got = _per_step(gfa, V, s, d, 3)
    for t in range(3):
        assert np.array_equal(got[t], hist[t]), f"seed {seed} superstep {t + 1}"


def test_frontier_after_column_runs(gfa, oracle):
    """Superstep 1 by column runs stages no hub unit words; when it changes < 0.5 % of
    the arcs, superstep 2 must still tally every unit of a dirty hub row.
    Fresh handle per superstep, then lpa_run twice on one handle (the second run would
    otherwise merge the first run's stale unit words)."""
    V, s, d = stale_units()
    _, hist, _ = oracle.lpa(V, s, d, 5, per_iter=True)
    got = _per_step(gfa, V, s, d, 5)
    for t in range(5):
        assert np.array_equal(got[t], hist[t]), f"superstep {t + 1}"
    with gfa.Graph(s, d, V) as g:
        assert g.info()["max_degree"] > 8192
        for _ in range(2):
            for it in (2, 5):
                assert np.array_equal(g.run(it), hist[it - 1]), f"run({it})"


def test_first_runs_off_identical(gfa, monkeypatch):
    s, d = gfa.gen_rmat(16, 16, seed=9)
    V = 1 << 16
    on = _per_step(gfa, V, s, d, 2)
    monkeypatch.setenv("LPA_FIRST_RUNS", "0")
    off = _per_step(gfa, V, s, d, 2)
    assert np.array_equal(on, off)


def test_bad_arguments(gfa):
    with gfa.Graph(np.array([0], np.int32), np.array([1], np.int32), 2) as g:
        with pytest.raises(ValueError, match="Maximum of steps must be greater than 0"):
            g.run(0)
    with pytest.raises(ValueError, match="outside"):
        gfa.Graph(np.array([0], np.int32), np.array([5], np.int32), 2)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_degree_mix_all_bins(gfa, oracle, seed):
    V, s, d = degree_mix(seed)
    with gfa.Graph(s, d, V) as g:
        info = g.info()
        assert info["hub_vertices"] >= 2 and info["bin_vertices"]["seg"] == info["hub_vertices"]
        assert all(info["bin_vertices"][b] > 0 for b in
                   ("w16", "w8", "w4", "w2", "g64", "g32", "g16", "g8", "g4", "g2", "g1")), info["bin_vertices"]
    _, hist, _ = oracle.lpa(V, s, d, 6, per_iter=True)
    got = _per_step(gfa, V, s, d, 6)
    for t in range(6):
        assert np.array_equal(got[t], hist[t]), f"seed {seed} superstep {t + 1}"


@pytest.mark.parametrize("seed", [0, 1])
def test_hub_combine_buckets_and_subpasses(gfa, oracle, seed):
    """A 220K-arc hub whose staged words are all distinct in superstep 1 (128
    combine buckets, one of them overloaded -> sub-bucket passes); the mode sits
    in the overloaded bucket.  Bit-exact per superstep."""
    V, s, d = giant_hub(seed)
    _, hist, _ = oracle.lpa(V, s, d, 4, per_iter=True)
    got = _per_step(gfa, V, s, d, 4)
    for t in range(4):
        bad = np.flatnonzero(got[t] != hist[t])
        assert bad.size == 0, f"superstep {t + 1}: {bad.size} differ, first {bad[:5]}"


@pytest.mark.parametrize("V,m,seed", [(50, 2000, 3), (3000, 60000, 4), (20000, 40000, 5)])
def test_random_multigraphs(gfa, oracle, V, m, seed):
    V, s, d = random_multigraph(V, m, seed)
    with gfa.Graph(s, d, V) as g:
        for it in (1, 4):
            assert np.array_equal(g.run(it), oracle.lpa(V, s, d, it))


def test_generators_match_cpu_restatement(gfa, oracle):
    s, d = gfa.gen_rmat(14, 16, seed=1)
    cs, cd = oracle.gen_rmat(14, 16, seed=1)
    assert np.array_equal(s.cpu().numpy(), cs) and np.array_equal(d.cpu().numpy(), cd)
    s, d = gfa.gen_sbm(10000, 100, 200000, seed=20261015)
    cs, cd = oracle.gen_sbm(10000, 100, 200000, seed=20261015)
    assert np.array_equal(s.cpu().numpy(), cs) and np.array_equal(d.cpu().numpy(), cd)


@pytest.mark.parametrize("scale", [12, 16, 18])
def test_rmat_bit_exact(gfa, oracle, scale):
    s, d = gfa.gen_rmat(scale, 16, seed=1)
    V = 1 << scale
    with gfa.Graph(s, d, V) as g:   # device input path
        got = []
        for _ in range(10):
            g.step(1)
            got.append(g.labels())
    _, hist, _ = oracle.lpa(V, s.cpu().numpy(), d.cpu().numpy(), 10, per_iter=True)
    for t in range(10):
        assert np.array_equal(got[t], hist[t]), f"R-MAT {scale} superstep {t + 1}"


@pytest.mark.parametrize("locality", ["0", "1", "3"])
def test_vertex_order_invariance(gfa, oracle, monkeypatch, locality):
    """The slot order inside the degree bins (LPA_LOCALITY: plain degree order, or the
    locality order by K smallest neighbour ranks) is internal: labels per superstep are
    bit-exact against the oracle under every order (R-MAT scale 16, hubs and all bins)."""
    monkeypatch.setenv("LPA_LOCALITY", locality)   # read when the handle is created
    s, d = gfa.gen_rmat(16, 16, seed=3)
    V = 1 << 16
    with gfa.Graph(s, d, V) as g:
        got = []
        for _ in range(6):
            g.step(1)
            got.append(g.labels())
    _, hist, _ = oracle.lpa(V, s.cpu().numpy(), d.cpu().numpy(), 6, per_iter=True)
    for t in range(6):
        assert np.array_equal(got[t], hist[t]), f"LPA_LOCALITY={locality} superstep {t + 1}"


def test_c2_sbm_full_size(gfa, oracle):
    """Config C2: planted partition, 1 M vertices / 20 M edges /
    100 blocks, maxIter 10: bit-exact vs the oracle at EVERY superstep (the shipped
    schedule, then the frontier off), lpa_run(10) likewise, and the communities recover
    the planted blocks (NMI vs ground truth; oracle value at seed 20261015: 0.916)."""
    from sklearn.metrics import normalized_mutual_info_score as nmi
    V, B, m = 1_000_000, 100, 20_000_000
    s, d = gfa.gen_sbm(V, B, m)
    _, hist, _ = oracle.lpa(V, s.cpu().numpy(), d.cpu().numpy(), 10, per_iter=True)
    ref = hist[9]
    with gfa.Graph(s, d, V) as g:
        assert g.info()["gather_mode"] == 1   # 4 MB label vector, rows <= 128 arcs
        for frontier in (True, False):
            g.set_frontier(frontier)
            g.reset()
            for t in range(10):
                g.step(1)
                bad = int((g.labels() != hist[t]).sum())
                assert bad == 0, f"frontier={frontier} superstep {t + 1}: {bad} labels differ"
        g.set_frontier(True)
        lab = g.run(10)
    assert np.array_equal(lab, ref)
    truth = np.minimum(np.arange(V) // (V // B), B - 1)
    assert nmi(truth, lab) > 0.9


@pytest.mark.parametrize("graph", ["rmat17", "mix"])
def test_schedules_identical(gfa, graph):
    """The concurrent four-stream schedule (forked hub combine in the label-dense
    supersteps) and the serialized profiling schedule give identical labels (the
    degree mix has rows in both block tiers and a bucketed hub)."""
    if graph == "rmat17":
        s, d = gfa.gen_rmat(17, 16, seed=3)
        V = 1 << 17
    else:
        V, s, d = degree_mix(0)
    with gfa.Graph(s, d, V) as g:
        conc = [g.labels() for _ in range(6) if g.step(1) is not None or True]
        g.reset()
        g.set_serial(True)
        ser = [g.labels() for _ in range(6) if g.step(1) is not None or True]
    for t in range(6):
        assert np.array_equal(conc[t], ser[t]), f"superstep {t + 1}"


@pytest.mark.parametrize("env", [{"LPA_SERIAL": "1"}, {"LPA_FIRST_RUNS": "0"}, {"LPA_GRAPHS": "0"},
                                 {"LPA_REBUILD_HOT": "0"}, {"LPA_FRONTIER": "0"}, {"LPA_LOCALITY": "0"},
                                 {"LPA_FUSED_BINS": "0"}, {"LPA_FUSED_BINS": "2", "LPA_CONV_STREAMS": "3"},
                                 {"LPA_CONV_STREAMS": "1"}, {"LPA_KEEP_BITS": "0"}, {"LPA_UNITS_PURE": "0"}])
def test_schedule_options_bit_exact(gfa, oracle, monkeypatch, env):
    """The switches read at graph creation (the serialized profiling
    schedule, superstep 1 by hash tallies, no captured graphs, the plain rebuild, no
    frontier, plain degree order, one launch per bin in the converged supersteps): labels bit-exact per superstep on the degree mix
    (both block tiers + a bucketed hub), R-MAT-16 and an SBM in gather mode."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    V, s, d = degree_mix(1)
    _, hist, _ = oracle.lpa(V, s, d, 6, per_iter=True)
    got = _per_step(gfa, V, s, d, 6)
    for t in range(6):
        assert np.array_equal(got[t], hist[t]), f"mix {env} superstep {t + 1}"
    rs, rd = gfa.gen_rmat(16, 16, seed=5)
    sn, dn = rs.cpu().numpy(), rd.cpu().numpy()
    _, hist, _ = oracle.lpa(1 << 16, sn, dn, 6, per_iter=True)
    got = _per_step(gfa, 1 << 16, rs, rd, 6)
    for t in range(6):
        assert np.array_equal(got[t], hist[t]), f"rmat16 {env} superstep {t + 1}"
    # SBM 200 K / 4 M: gather mode (tallies read L[col[i]], no al[] refresh)
    ss, sd = gfa.gen_sbm(200_000, 20, 4_000_000)
    with gfa.Graph(ss, sd, 200_000) as gg:
        assert gg.info()["gather_mode"] == 1
    _, hist, _ = oracle.lpa(200_000, ss.cpu().numpy(), sd.cpu().numpy(), 8, per_iter=True)
    got = _per_step(gfa, 200_000, ss, sd, 8)
    for t in range(8):
        assert np.array_equal(got[t], hist[t]), f"sbm {env} superstep {t + 1}"


def test_chunglu_generator_matches_oracle(gfa, oracle):
    s, d = gfa.gen_chunglu(100_000, 1_000_000, 2.1, 30_000.0, seed=7)
    cs, cd = oracle.gen_chunglu(100_000, 1_000_000, 2.1, 30_000.0, 7)
    assert np.array_equal(s.cpu().numpy(), cs) and np.array_equal(d.cpu().numpy(), cd)


def test_chunglu_heavy_hub_every_superstep(gfa, oracle):
    """Config C5's shape scaled down (Chung-Lu exponent 2.1): a hub
    of ~250 K arcs among 300 K vertices -- the superstep-1 combine sees ~200 K
    distinct labels in one row (bucket path, sub-bucket passes).  Bit-exact per superstep."""
    V, m = 300_000, 3_000_000
    s, d = gfa.gen_chunglu(V, m, 2.1, 250_000.0, seed=7)
    sn, dn = s.cpu().numpy(), d.cpu().numpy()
    deg = np.bincount(sn, minlength=V) + np.bincount(dn, minlength=V)
    assert deg.max() > 200_000
    got = _per_step(gfa, V, s, d, 10)
    _, hist, _ = oracle.lpa(V, sn, dn, 10, per_iter=True)
    for t in range(10):
        assert np.array_equal(got[t], hist[t]), f"Chung-Lu superstep {t + 1}"


def test_sbm_bit_exact(gfa, oracle):
    s, d = gfa.gen_sbm(20000, 20, 400000)
    with gfa.Graph(s, d, 20000) as g:
        lab = g.run(10)
    assert np.array_equal(lab, oracle.lpa(20000, s.cpu().numpy(), d.cpu().numpy(), 10))


@pytest.mark.parametrize("P", [2, 3, 4])
def test_virtual_partitions_bit_exact(gfa, oracle, P):
    """P ranks on one device with the caller-driven exchange: the partitioned
    build + kernels give the single-GPU answer bit for bit."""
    V, s, d = degree_mix(7)
    ranks = [gfa.Graph(s, d, V, rank=r, nranks=P) for r in range(P)]
    try:
        infos = [g.info() for g in ranks]
        assert sum(i["arcs"] for i in infos) == 2 * s.size
        _, hist, _ = oracle.lpa(V, s, d, 5, per_iter=True)
        for t in range(5):
            for g in ranks:
                g.step(1)
            full = np.concatenate([g.exchange_get() for g in ranks])
            for g in ranks:
                g.exchange_put(full)
            assert np.array_equal(ranks[0].labels(), hist[t]), f"P={P} superstep {t + 1}"
    finally:
        for g in ranks:
            g.close()


@pytest.mark.parametrize("P", [2, 4])
def test_virtual_partitions_rmat_power_of_two(gfa, oracle, P):
    """Power-of-two slices: the al[] rebuild serves the hottest vertices of every
    slice from LDS (rank-strided hot set); bit-exact per superstep (R-MAT scale 16)."""
    s, d = gfa.gen_rmat(16, 16, seed=2)
    V = 1 << 16
    s, d = s.cpu().numpy(), d.cpu().numpy()
    ranks = [gfa.Graph(s, d, V, rank=r, nranks=P) for r in range(P)]
    try:
        assert ranks[0].info()["slice"] == V // P
        _, hist, _ = oracle.lpa(V, s, d, 5, per_iter=True)
        for t in range(5):
            for g in ranks:
                g.step(1)
            full = np.concatenate([g.exchange_get() for g in ranks])
            for g in ranks:
                g.exchange_put(full)
            assert np.array_equal(ranks[-1].labels(), hist[t]), f"P={P} superstep {t + 1}"
    finally:
        for g in ranks:
            g.close()


@pytest.mark.parametrize("P", [2, 4])
def test_virtual_partitions_delta_exchange(gfa, oracle, P):
    """The changed-label delta exchange (the converged-superstep protocol of the
    in-library RCCL exchange, lpa_exchange.hip) with P virtual ranks: full
    exchange while a delta exceeds slice / 4, deltas after; bit-exact per superstep."""
    V, s, d = degree_mix(11)
    ranks = [gfa.Graph(s, d, V, rank=r, nranks=P) for r in range(P)]
    try:
        slice_ = ranks[0].info()["slice"]
        _, hist, _ = oracle.lpa(V, s, d, 8, per_iter=True)
        modes = []
        for t in range(8):
            for g in ranks:
                g.step(1)
            deltas = [g.exchange_get_delta() for g in ranks]
            for r, e in enumerate(deltas):  # entries: owned local slots, in range
                assert e.size == 0 or int((e >> np.uint64(32)).max()) < slice_
            if max(e.size for e in deltas) <= slice_ // 4:
                for g in ranks:
                    g.exchange_put_delta(deltas)
                modes.append("delta")
            else:
                full = np.concatenate([g.exchange_get() for g in ranks])
                for g in ranks:
                    g.exchange_put(full)
                modes.append("full")
            for g in ranks:
                assert np.array_equal(g.labels(), hist[t]), f"P={P} superstep {t + 1} ({modes[-1]})"
        # consecutive deltas exercise the double application (previous + new change
        # list) that replaces the copy of the other slices
        assert modes[0] == "full" and any(a == b == "delta" for a, b in zip(modes, modes[1:])), modes
    finally:
        for g in ranks:
            g.close()


def test_outlier_l1_l2_golden(gfa, golden):
    V = golden["ids"].size
    with gfa.Graph(golden["src"], golden["dst"], V) as g:
        lab = g.run(5)
        o1 = g.outlier(lab, "L1")
        assert np.array_equal(o1["size"], golden["l1_size"])
        assert np.array_equal(o1["incident"], golden["l1_inc"])
        assert np.array_equal(o1["flags"], golden["l1_flags"].astype(bool))
        s1 = golden["l1_summary"]
        assert (o1["summary"]["n_groups"], o1["summary"]["k"], o1["summary"]["threshold"],
                o1["summary"]["n_flagged"]) == tuple(int(x) for x in s1)
        o2 = g.outlier(lab, "L2", sub_iter=5)
        assert np.array_equal(o2["sub_labels"], golden["l2_sub"])
        assert np.array_equal(o2["flags"], golden["l2_flags"].astype(bool))
        s2 = golden["l2_summary"]
        assert (o2["summary"]["n_communities"], o2["summary"]["n_groups"], o2["summary"]["n_flagged"],
                o2["summary"]["n_communities_flagged"]) == tuple(int(x) for x in s2)


@pytest.mark.parametrize("seed", [1, 2])
def test_outlier_vs_oracle(gfa, oracle, seed):
    V, s, d = degree_mix(seed, hubs=(700, 3000), n_low=2000, extra=8000)
    with gfa.Graph(s, d, V) as g:
        lab = g.run(3)
        o1 = g.outlier(lab, "L1")
        size, inc, flags, summ = oracle.outlier_l1(V, s, d, lab)
        assert np.array_equal(o1["size"], size) and np.array_equal(o1["incident"], inc)
        assert np.array_equal(o1["flags"], flags)
        assert o1["summary"]["threshold"] == summ["thr"]
        o2 = g.outlier(lab, "L2", sub_iter=4)
        sub, flags2, summ2 = oracle.outlier_l2(V, s, d, lab, 4)
        assert np.array_equal(o2["sub_labels"], sub) and np.array_equal(o2["flags"], flags2)
        assert o2["summary"]["n_flagged"] == summ2["n_flagged"]


@pytest.mark.parametrize("case", ["mix_run", "mix_random_labels", "reciprocal_loops", "rmat_coarse", "rmat22_codes"])
def test_outlier_l2_subgraph_and_device(gfa, oracle, case):
    """The L2 sub-graph built straight from the distinct-edge orders (no arc sort):
    reciprocal pairs (u, v) + (v, u) (two arcs of the same column in a row), self-loops,
    duplicates, isolated vertices, arbitrary (non-LPA) community labels; L1 / L2 vs the
    oracle, and the device-array form (lpa_outlier_device) equal to the host form."""
    import torch

    rng = np.random.default_rng(11)
    if case.startswith("mix"):
        V, s, d = degree_mix(7, hubs=(900, 2500), n_low=2500, extra=9000)
    elif case == "reciprocal_loops":
        V = 3000
        a = rng.integers(0, V - 200, size=6000)
        b = rng.integers(0, V - 200, size=6000)
        loops = rng.integers(0, V - 200, size=300)
        s = np.concatenate([a, b, loops, a[:500]]).astype(np.int32)     # (a, b), (b, a), loops, dups
        d = np.concatenate([b, a, loops, b[:500]]).astype(np.int32)
    elif case == "rmat22_codes":
        # round 6: a sub-graph of >= 4 M slots, whose second LPA takes the giant-code
        # refresh and settles (the main LPA's schedule on the pooled, rebuild-only handle)
        ts, td = gfa.gen_rmat(22, 16, seed=9)
        V, s, d = 1 << 22, ts.cpu().numpy(), td.cpu().numpy()
    else:
        ts, td = gfa.gen_rmat(15, 16, seed=4)
        V, s, d = 1 << 15, ts.cpu().numpy(), td.cpu().numpy()
    with gfa.Graph(s, d, V) as g:
        if case == "mix_random_labels":
            lab = rng.integers(0, 40, size=V).astype(np.int32)        # 40 arbitrary communities
        elif case == "rmat_coarse":
            lab = (g.run(2) % 97).astype(np.int32)
        elif case == "rmat22_codes":
            lab = g.run(10)
        else:
            lab = g.run(3)
        o1 = g.outlier(lab, "L1")
        o2 = g.outlier(lab, "L2", sub_iter=4)
        dl = torch.from_numpy(lab).cuda()
        d1 = g.outlier(dl, "L1")
        d2 = g.outlier(dl, "L2", sub_iter=4)
    size, inc, flags, summ = oracle.outlier_l1(V, s, d, lab)
    assert np.array_equal(o1["size"], size) and np.array_equal(o1["incident"], inc)
    assert np.array_equal(o1["flags"], flags) and o1["summary"]["threshold"] == summ["thr"]
    sub, flags2, summ2 = oracle.outlier_l2(V, s, d, lab, 4)
    assert np.array_equal(o2["sub_labels"], sub), int((o2["sub_labels"] != sub).sum())
    assert np.array_equal(o2["flags"], flags2)
    assert o2["summary"]["n_groups"] == summ2["n_subgroups"]
    assert o2["summary"]["n_communities_flagged"] == summ2["n_communities_flagged"]
    for h, dv in ((o1, d1), (o2, d2)):
        assert dv["summary"] == h["summary"]
        assert np.array_equal(dv["size"].cpu().numpy(), h["size"])
        assert np.array_equal(dv["incident"].cpu().numpy(), h["incident"])
        assert np.array_equal(dv["flags"].cpu().numpy(), h["flags"])
    assert np.array_equal(d2["sub_labels"].cpu().numpy(), o2["sub_labels"])


def test_dropin_graphframe_r9(gfa, golden):
    """GraphFrame(v, e).labelPropagation(maxIter=5) exactly as Graphframes.py:78-81 calls it."""
    ids, names = golden["ids"], golden["names"]
    v = pd.DataFrame({"id": ids, "name": names}).sample(frac=1.0, random_state=0)
    e = pd.DataFrame({"src": ids[golden["src"]], "dst": ids[golden["dst"]]})
    out = gfa.GraphFrame(v, e).labelPropagation(maxIter=5)
    assert list(out.columns) == ["id", "name", "label"] and out["label"].dtype == np.int64
    assert out["id"].tolist() == sorted(ids.tolist())
    assert np.array_equal(out["label"].to_numpy(), golden["labels_iter"][4].astype(np.int64))
    assert out["label"].nunique() == 619   # Graphframes.py:85 community count


def test_dropin_integral_ids_and_dangling(gfa, oracle):
    V, s, d = two_cliques()
    ids = np.arange(V, dtype=np.int64) * 10 + 7
    v = pd.DataFrame({"id": ids, "attr": np.arange(V)})
    e = pd.DataFrame({"src": np.append(ids[s], 999), "dst": np.append(ids[d], 7)})  # dangling edge
    out = gfa.label_propagation(v, e, 20)
    assert out["label"].tolist() == [7] * 5 + [57] * 6   # labels are original ids
    res = gfa.outlier_scores(v, e, labels=out, mode="L1")
    assert res.communities["size"].tolist() == [5, 6]
    assert res.summary["threshold"] == 6 and res.flagged_ids.tolist() == ids[:5].tolist()


def test_c1_end_to_end_from_parquet(gfa, golden, tmp_path):
    """Config C1 through the reference's own pipeline shape (Graphframes.py:16-85 and
    the intended :121-137): outlinks parquet (4 nullable string columns, one all-null
    row) -> null filter -> SHA-1[:8] ids -> GraphFrame -> labelPropagation(maxIter=5)
    -> distinct-label count -> outlier L1 / L2.  The parquet is rebuilt from the
    committed R9 fixture (the reference data itself is not on the GPU box)."""
    import pyarrow as pa
    import pyarrow.parquet as pq

    names = golden["names"].astype(str)
    pdom, cdom = names[golden["src"]].tolist(), names[golden["dst"]].tolist()
    tbl = pa.table({"_c0": [f"http://{x}/" for x in pdom] + ['"'], "_c1": pdom + [None],
                    "_c2": cdom + [None], "_c3": [f"http://{x}/" for x in cdom] + [None]})
    pq.write_table(tbl, str(tmp_path / "part-00000-c000.snappy.parquet"), compression="snappy")
    v, e = gfa.ingest.load_outlinks_graph(str(tmp_path))
    assert len(e) == 18398 and len(v) == 4613                     # :18, :30 filter, :53
    assert v["id"].tolist() == golden["ids"].tolist()             # NodeHash ids (:57-58)
    gf = gfa.GraphFrame(v, e)                                     # :78
    try:
        out = gf.labelPropagation(maxIter=5)                      # :81
        assert out["label"].nunique() == 619                      # :85
        assert np.array_equal(out["label"].to_numpy(), golden["labels_iter"][4].astype(np.int64))
        r1 = gf.outlierScores(labels=out, mode="L1")
        assert r1.summary["n_flagged"] == 0 and r1.flagged_ids.size == 0
        assert r1.communities["size"].sum() == 4613 and len(r1.communities) == 619   # :100-120
        r2 = gf.outlierScores(labels=out, mode="L2", subIter=5)   # :121-137
        assert r2.summary["n_flagged"] == 40
        assert r2.flagged_ids.tolist() == golden["ids"][golden["l2_flags"].astype(bool)].tolist()
    finally:
        gf.close()


def test_outlier_rejects_out_of_range_labels(gfa):
    V, s, d = two_cliques()
    with gfa.Graph(s, d, V) as g:
        bad = np.zeros(V, np.int32)
        bad[3] = V + 5
        for mode in ("L1", "L2"):
            with pytest.raises(ValueError, match="outside"):
                g.outlier(bad, mode)
        # the handle is still usable afterwards
        assert g.outlier(g.run(20), "L1")["summary"]["n_communities"] == 2


@pytest.mark.parametrize("which", ["rmat", "mix", "star"])
def test_frontier_on_off_identical(gfa, oracle, which):
    """Frontier (re-tally only rows with a changed neighbour, lpa_set_frontier) vs
    every row every superstep: identical labels per superstep, also when the mode is
    toggled mid-run, against the oracle (the oscillating star keeps every row dirty;
    R-MAT converges to a few dirty rows)."""
    if which == "rmat":
        s, d = gfa.gen_rmat(16, 16, seed=5)
        V, s, d = 1 << 16, s.cpu().numpy(), d.cpu().numpy()
    elif which == "mix":
        V, s, d = degree_mix(4)
    else:
        V, s, d = star(300)
    _, hist, _ = oracle.lpa(V, s, d, 12, per_iter=True)
    with gfa.Graph(s, d, V) as g:
        for pattern in ([1] * 12, [0] * 12, [1, 1, 1, 0, 1, 1, 0, 0, 1, 1, 1, 1]):
            g.reset()
            for t, on in enumerate(pattern):
                g.set_frontier(bool(on))
                g.step(1)
                assert np.array_equal(g.labels(), hist[t]), f"{which} pattern {pattern} superstep {t + 1}"
        g.set_frontier(True)
        assert np.array_equal(g.run(12), hist[11])


@pytest.mark.parametrize("seed", [0, 1])
def test_hub_spill_adversarial_bucket(gfa, oracle, seed):
    """One hub whose 20 000 distinct superstep-1 labels share both the combine bucket
    and the sub-bucket hash (lpa_hub.hip comb_bucket / comb_sub): the bucket pass meets
    more distinct labels than its 8192-slot LDS table.  The spill guard re-runs that
    pass on label-value sub-ranges instead of dropping votes; labels
    are bit-exact against the oracle per superstep, no LPA_EOVERFLOW."""
    V, s, d = adversarial_hub(seed=seed)
    _, hist, _ = oracle.lpa(V, s, d, 3, per_iter=True)
    got = _per_step(gfa, V, s, d, 3)
    for t in range(3):
        bad = np.flatnonzero(got[t] != hist[t])
        assert bad.size == 0, f"superstep {t + 1}: {bad.size} differ, first {bad[:5]}"


@pytest.mark.parametrize("seed", [0, 1])
def test_frontier_from_superstep_2_with_block_rows(gfa, oracle, seed):
    """A graph where superstep 1 changes ~0.25 % of the arcs' labels (self-loops keep
    almost every L0 label): superstep 2 -- a label-dense superstep, whose hub rows of
    1024 < deg <= 4096 are tallied one block per row -- already runs on the frontier
    lists, and superstep 3 must re-tally every row (the block rows staged no unit
    words).  Bit-exact per superstep, and lpa_run agrees."""
    V, s, d = settled_hubs(seed)
    _, hist, _ = oracle.lpa(V, s, d, 8, per_iter=True)
    got = _per_step(gfa, V, s, d, 8)
    for t in range(8):
        bad = np.flatnonzero(got[t] != hist[t])
        assert bad.size == 0, f"superstep {t + 1}: {bad.size} differ, first {bad[:5]}"
    with gfa.Graph(s, d, V) as g:
        assert np.array_equal(g.run(8), hist[7])


def _modularity_np(V, s, d, lab):
    """Newman modularity on the symmetrised multigraph (numpy restatement)."""
    A = 2 * s.size
    intra = 2 * int((lab[s] == lab[d]).sum())
    deg = np.bincount(s, minlength=V) + np.bincount(d, minlength=V)
    D = np.bincount(lab, weights=deg, minlength=V)
    return intra / A - float(((D / A) ** 2).sum()), intra


@pytest.mark.parametrize("graph", ["r9", "rmat16", "mix"])
def test_quality_matches_numpy(gfa, golden, graph):
    """lpa_quality (community count, intra arcs, modularity) against a numpy
    restatement, on the labels the GPU computes (maxIter 5) and on L0."""
    if graph == "r9":
        V, s, d = golden["ids"].size, golden["src"], golden["dst"]
    elif graph == "rmat16":
        ts, td = gfa.gen_rmat(16, 16, seed=2)
        V, s, d = 1 << 16, ts.cpu().numpy(), td.cpu().numpy()
    else:
        V, s, d = degree_mix(4)
    with gfa.Graph(s, d, V) as g:
        for lab in (g.run(5), np.arange(V, dtype=np.int32)):
            q = g.quality(lab)
            Q, intra = _modularity_np(V, s.astype(np.int64), d.astype(np.int64), lab.astype(np.int64))
            assert q["n_communities"] == np.unique(lab).size
            assert q["intra_arcs"] == intra and q["arcs"] == 2 * s.size
            assert abs(q["modularity"] - Q) < 1e-9
        with pytest.raises(ValueError, match="outside"):
            g.quality(np.full(V, V, dtype=np.int32))
        # device tensors: int32 on this device equals the host result; an
        # int64 tensor (torch.arange's default) is refused, not read as int32 pairs
        import torch

        lab = g.run(5)
        dl = torch.from_numpy(lab).cuda()
        assert g.quality(dl) == g.quality(lab)
        with pytest.raises(ValueError, match="int32"):
            g.quality(torch.arange(V, device="cuda"))


@pytest.fixture(scope="module")
def rmat22(gfa, oracle):
    s, d = gfa.gen_rmat(22, 16, seed=11)
    sn, dn = s.cpu().numpy(), d.cpu().numpy()
    _, hist, _ = oracle.lpa(1 << 22, sn, dn, 5, per_iter=True)
    return sn, dn, hist


@pytest.mark.parametrize("env", [{"LPA_BLOCK_DEG": "0"}, {"LPA_BLOCK_DEG": "8"}, {"LPA_BLOCK_DEG": "64"},
                                 {"LPA_BLOCK_DEG": "1000"}, {"LPA_BLOCK_DEG": "64", "LPA_LOCALITY": "0"},
                                 {"LPA_BLOCK_DEG": "64", "LPA_GIANT_CODES": "0"}])
def test_class_blocked_rebuild_bit_exact(gfa, rmat22, monkeypatch, env):
    """The class-blocked labels-mode al[] rebuild (rows of degree > LPA_BLOCK_DEG in
    (class, column) order, per-XCD class pieces -- 8 classes at this size, one phase per 8;
    the multi-phase class counts run at C4 / C5 size, tests/test_gpu_configs.py --
    + the plain stream below; its arc giant bits ORed piecewise): R-MAT-22 (4 M slots, the LDS hot-set rebuild) bit-exact against
    the oracle at supersteps 1..5 -- superstep 1's column runs over the reordered rows,
    the labels-/hybrid-mode rebuild after it, superstep 2's settles from its arc bits."""
    monkeypatch.setenv("LPA_BLOCK_MIN_SLOTS", "0")   # shipped: label vectors of >= 32 M slots
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    sn, dn, hist = rmat22
    V = 1 << 22
    with gfa.Graph(sn, dn, V) as g:
        info = g.info()
        if env["LPA_BLOCK_DEG"] == "0":
            assert info["blocked_rows"] == 0
        else:
            assert info["blocked_rows"] > 0 and info["blocked_pieces"] % 8 == 0, info
        for t in range(5):
            g.step(1)
            bad = int((g.labels() != hist[t]).sum())
            assert bad == 0, f"{env} superstep {t + 1}: {bad} labels differ"
        g.reset()
        assert np.array_equal(g.run(5), hist[4]), f"{env} lpa_run(5) after reset"


@pytest.fixture(scope="module")
def codemix22(gfa, oracle):
    from graphs import code_mix
    s, d = gfa.gen_rmat(22, 16, seed=11)
    V, sn, dn = code_mix(s.cpu().numpy(), d.cpu().numpy(), 1 << 22)
    _, hist, _ = oracle.lpa(V, sn, dn, 5, per_iter=True)
    return V, sn, dn, hist


def test_giant_code_refresh_every_superstep(gfa, codemix22):
    """The giant-code refresh after superstep 1 (R-MAT: G on the hubs, not on half the
    hot slots) and superstep 2's settle from the 1-byte codes, with every exact fallback
    populated -- wave-bin rows, block-tier hub rows and > 8192-arc hub rows whose mode is
    not G (tests/graphs.py code_mix): bit-exact at supersteps 1..5, then lpa_run(5)."""
    V, sn, dn, hist = codemix22
    with gfa.Graph(sn, dn, V) as g:
        for t in range(5):
            g.step(1)
            if t == 0:
                assert g.info()["code_refresh"] == 1, "the giant-code refresh was not taken"
            bad = int((g.labels() != hist[t]).sum())
            assert bad == 0, f"superstep {t + 1}: {bad} labels differ"
        g.reset()
        assert np.array_equal(g.run(5), hist[4]), "lpa_run(5) after reset"
        g.reset()
        assert np.array_equal(g.run(5), hist[4]), "lpa_run(5), second call (replayed graphs)"


@pytest.fixture(scope="module")
def chunglu5m(gfa, oracle):
    # 40,000,002 arcs: not a multiple of the rebuild's 512-arc batches (every BASELINE
    # config's arc count is), on a label vector large enough for the LDS hot-set rebuild
    V, m = 5_000_000, 20_000_001
    s, d = gfa.gen_chunglu(V, m, 2.1, 200_000.0, seed=3)
    sn, dn = s.cpu().numpy(), d.cpu().numpy()
    _, hist, _ = oracle.lpa(V, sn, dn, 5, per_iter=True)
    return V, sn, dn, hist


@pytest.mark.parametrize("env", [{}, {"LPA_BLOCK_MIN_SLOTS": "0"}, {"LPA_BLOCK_MIN_SLOTS": "0", "LPA_BLOCK_DEG": "64"}])
def test_hot_rebuild_partial_batch(gfa, chunglu5m, monkeypatch, env):
    """The hot-set rebuild's partial last batch (and, blocked, the plain stream after the
    listed range ending mid-batch), labels and bits modes: bit-exact at supersteps 1..5."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    V, sn, dn, hist = chunglu5m
    with gfa.Graph(sn, dn, V) as g:
        assert g.info()["arcs"] % 512 != 0
        for t in range(5):
            g.step(1)
            bad = int((g.labels() != hist[t]).sum())
            assert bad == 0, f"{env} superstep {t + 1}: {bad} labels differ"


def test_giant_code_refresh_after_superstep_2(gfa, chunglu5m):
    """Chung-Lu (5 M / 20 M, max degree ~200 K): the giant-code refresh is taken after
    superstep 2 (G on the hubs, on 43 % of the hot slots) and superstep 3 settles hub and
    wave rows from the codes, lists the rest (k_code_commit) and rebuilds al[] after it;
    the refresh after superstep 1 takes it too on this graph (G on half the top hubs).
    Bit-exact at supersteps 1..5, the arc count not a multiple of 512 (the code
    rebuild's partial last batch)."""
    V, sn, dn, hist = chunglu5m
    with gfa.Graph(sn, dn, V) as g:
        taken = []
        for t in range(5):
            g.step(1)
            taken.append(g.info()["code_refresh"])
            bad = int((g.labels() != hist[t]).sum())
            assert bad == 0, f"superstep {t + 1}: {bad} labels differ"
        assert taken[1] == 1, taken   # the refresh after superstep 2
        g.reset()
        assert np.array_equal(g.run(5), hist[4]), "lpa_run(5) after reset"


def test_sbm_hot_path_every_superstep(gfa, oracle):
    """A family with no giant label (planted partition, 400 blocks) at the LDS hot-set
    rebuild's size (4 M slots): every superstep's giant pick finds no dominant label, so
    the giant decisions and settles must stand aside -- bit-exact at supersteps 1..10."""
    V, B, m = 1 << 22, 400, 40_000_000
    s, d = gfa.gen_sbm(V, B, m)
    sn, dn = s.cpu().numpy(), d.cpu().numpy()
    _, hist, _ = oracle.lpa(V, sn, dn, 10, per_iter=True)
    with gfa.Graph(s, d, V) as g:
        for t in range(10):
            g.step(1)
            bad = int((g.labels() != hist[t]).sum())
            assert bad == 0, f"SBM-4M superstep {t + 1}: {bad} labels differ"
        g.reset()
        assert np.array_equal(g.run(10), hist[9])

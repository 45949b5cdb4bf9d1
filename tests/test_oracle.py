"""CPU oracle pinning (no GPU): the C restatement vs the pure-Python one, the
upstream-suite-shaped known answers, and the facts of the reference's own
sample data (R9, /root/reference/CommunityDetection/data, restated per
Graphframes.py:16-73 into tests/golden/r9_golden.npz by make_golden.py)."""
import numpy as np
import pytest

from graphs import degree_mix, random_multigraph, star, two_cliques


def test_two_cliques_kat(oracle):
    V, s, d = two_cliques()
    lab = oracle.lpa(V, s, d, 20)
    # upstream LabelPropagationSuite: each clique one label, the two labels differ;
    # min-tie answer computed at survey time
    assert lab.tolist() == [0, 0, 0, 0, 0, 5, 5, 5, 5, 5, 5]
    assert oracle.lpa_py(V, list(zip(s, d)), 20) == lab.tolist()


def test_star_period_two(oracle):
    V, s, d = star(10)
    _, hist, _ = oracle.lpa(V, s, d, 4, per_iter=True)
    assert hist[0][0] == 1 and (hist[0][1:] == 0).all()
    assert hist[1][0] == 0 and (hist[1][1:] == 1).all()
    assert np.array_equal(hist[2], hist[0])


def test_votes_semantics(oracle):
    # self-loop (u,u) = 2 votes for L[u]; duplicates counted; isolated keep label
    V = 5
    s = np.array([1, 1, 1, 3], np.int32)
    d = np.array([1, 0, 2, 4], np.int32)
    lab = oracle.lpa(V, s, d, 1)
    assert lab[1] == 1          # 2 votes for own label beat 1 each for 0 and 2
    assert lab[0] == 1 and lab[2] == 1
    assert lab[3] == 4 and lab[4] == 3
    s = np.array([0, 0, 0], np.int32)
    d = np.array([2, 2, 1], np.int32)
    assert oracle.lpa(3, s, d, 1)[0] == 2   # duplicate edge = 2 votes


def test_max_iter_must_be_positive(oracle):
    with pytest.raises(ValueError, match="greater than 0"):
        oracle.lpa(3, np.array([0], np.int32), np.array([1], np.int32), 0)
    with pytest.raises(ValueError):
        oracle.lpa_py(3, [(0, 1)], -1)


@pytest.mark.parametrize("V,m,seed", [(7, 20, 0), (30, 100, 1), (60, 400, 2), (200, 300, 3)])
def test_c_matches_python(oracle, V, m, seed):
    V, s, d = random_multigraph(V, m, seed)
    for it in (1, 2, 5):
        assert oracle.lpa(V, s, d, it).tolist() == oracle.lpa_py(V, list(zip(s.tolist(), d.tolist())), it)


def test_outlier_l1_matches_python(oracle):
    V, s, d = random_multigraph(300, 500, 9)
    lab = oracle.lpa(V, s, d, 3)
    size, inc, flags, summ = oracle.outlier_l1(V, s, d, lab)
    psize, pinc, pflags, pthr = oracle.outlier_l1_py(V, list(zip(s.tolist(), d.tolist())), lab.tolist())
    assert summ["thr"] == pthr
    assert flags.tolist() == pflags
    assert all(size[l] == c for l, c in psize.items()) and size.sum() == V
    assert all(inc[l] == c for l, c in pinc.items())


def test_threshold_rule_lst_minus_zero(oracle):
    # n < 10 groups -> k = 0 -> lst[-0] == lst[0] = the LARGEST size (Graphframes.py:136)
    assert oracle.threshold_rule_py({1: 5, 2: 3, 3: 1}) == 5
    sizes = {i: i for i in range(1, 21)}   # n = 20 -> k = 2 -> 2nd smallest
    assert oracle.threshold_rule_py(sizes) == 2


def test_r9_fixture_facts(golden):
    # facts of the reference's own sample data
    assert int(golden["rows_total"]) == 18399          # Graphframes.py:18 print
    assert int(golden["rows_after_filter"]) == 18398   # :30 null filter drops 1 row
    V = golden["ids"].size
    assert V == 4613                                   # :54 print (distinct domains)
    s, d = golden["src"], golden["dst"]
    assert s.size == 18398
    assert np.unique(s.astype(np.int64) * V + d).size == 7742
    assert int((s == d).sum()) == 0
    deg = np.bincount(s, minlength=V) + np.bincount(d, minlength=V)
    assert deg.max() == 1223
    names = golden["names"]
    assert names[np.argmax(deg)] == "twitter.com"
    assert all(len(i) == 8 for i in golden["ids"][:50])


def test_r9_golden_reproduced_by_oracle(oracle, golden):
    V = golden["ids"].size
    final, hist, ties = oracle.lpa(V, golden["src"], golden["dst"], 10, per_iter=True)
    assert np.array_equal(hist, golden["labels_iter"])
    # survey-time scratch run: 619 communities, ties 622/310/201/184/194
    assert np.unique(hist[4]).size == 619
    assert ties[:5].tolist() == [622, 310, 201, 184, 194]
    assert ties.tolist() == golden["ties"].tolist()


def test_r9_outlier_facts(oracle, golden):
    V = golden["ids"].size
    lab = golden["labels_iter"][4]
    size, inc, flags, summ = oracle.outlier_l1(V, golden["src"], golden["dst"], lab)
    # App. B: n = 619, k = 61, 272 singletons -> thr = 1 -> nothing flagged
    assert (summ["n_groups"], summ["k"], summ["thr"], summ["n_flagged"]) == (619, 61, 1, 0)
    assert int((size == 1).sum()) == 272
    assert np.array_equal(size, golden["l1_size"]) and np.array_equal(inc, golden["l1_inc"])
    sub, flags2, s2 = oracle.outlier_l2(V, golden["src"], golden["dst"], lab, 5)
    # App. B L2 on C1: 40 vertices in 11 communities flagged
    assert (s2["n_flagged"], s2["n_communities_flagged"]) == (40, 11)
    assert np.array_equal(flags2, golden["l2_flags"].astype(bool))


def test_degree_mix_covers_bins():
    V, s, d = degree_mix(0)
    deg = np.bincount(s, minlength=V) + np.bincount(d, minlength=V)
    assert (deg > 4096).sum() >= 2 and ((deg > 512) & (deg <= 2048)).sum() >= 1
    for lo, hi in ((256, 512), (128, 256), (64, 128), (32, 64), (16, 32), (8, 16), (4, 8), (2, 4),
                   (1, 2), (0, 1)):
        assert ((deg > lo) & (deg <= hi)).sum() > 0, (lo, hi)
    assert (deg == 0).sum() > 0


def test_generators_deterministic(oracle):
    s1, d1 = oracle.gen_rmat(10, 16, seed=1)
    s2, d2 = oracle.gen_rmat(10, 16, seed=1)
    assert np.array_equal(s1, s2) and np.array_equal(d1, d2)
    assert s1.min() >= 0 and s1.max() < 1024
    s3, _ = oracle.gen_rmat(10, 16, seed=2)
    assert not np.array_equal(s1, s3)
    s, d = oracle.gen_sbm(1000, 10, 50000)
    same = (s // 100) == (d // 100)
    assert abs(same.mean() - 0.9) < 0.01


def test_chunglu_generator(oracle):
    """Config C5's generator (Chung-Lu, exponent 2.1, seed 7):
    deterministic, ids in range, the requested expected maximum degree, a heavy tail."""
    V, m = 200_000, 2_000_000
    s1, d1 = oracle.gen_chunglu(V, m, 2.1, 20_000.0, 7)
    s2, d2 = oracle.gen_chunglu(V, m, 2.1, 20_000.0, 7)
    assert np.array_equal(s1, s2) and np.array_equal(d1, d2)
    assert s1.min() >= 0 and max(s1.max(), d1.max()) < V
    s3, _ = oracle.gen_chunglu(V, m, 2.1, 20_000.0, 8)
    assert not np.array_equal(s1, s3)
    deg = np.bincount(s1, minlength=V) + np.bincount(d1, minlength=V)
    assert 0.9 * 20_000 < deg.max() < 1.1 * 20_000
    top = np.sort(deg)[::-1]
    # power-law tail: the top 1 % of vertices hold far more than 1 % of the arcs
    assert top[: V // 100].sum() > 0.2 * deg.sum()

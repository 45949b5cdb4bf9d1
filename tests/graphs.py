"""Seeded test graphs covering every degree bin and the edge cases of the path."""
import numpy as np


def two_cliques(n=5):
    """Upstream LabelPropagationSuite shape (Spark graphx + GraphFrames): clique1 =
    all (u, v) for u, v in [0, n) (self-loops included), clique2 = all (u+n, v+n)
    for u, v in [0, n], plus the bridge (0, n)."""
    e = [(u, v) for u in range(n) for v in range(n)]
    e += [(u + n, v + n) for u in range(n + 1) for v in range(n + 1)]
    e.append((0, n))
    a = np.array(e, dtype=np.int32)
    return 2 * n + 1, a[:, 0].copy(), a[:, 1].copy()


def star(k):
    """Hub 0 with leaves 1..k: period-2 oscillation under synchronous LPA."""
    s = np.zeros(k, dtype=np.int32)
    d = np.arange(1, k + 1, dtype=np.int32)
    return k + 1, s, d


def degree_mix(seed=0, hubs=(600, 2100, 4500, 9000), n_low=3000, extra=20000):
    """Random multigraph whose symmetrised degrees span every bin: a few hubs
    (single- and multi-segment), a wave band, and the g1..g16 bands; duplicates,
    self-loops and isolated vertices included."""
    rng = np.random.default_rng(seed)
    V = n_low + len(hubs) + 50
    src, dst = [], []
    for h, deg in enumerate(hubs):
        nb = rng.integers(len(hubs), V, size=deg)
        # few distinct neighbours for some hubs -> repeated labels, many for others
        if h % 2:
            nb = nb % 97 + len(hubs)
        src.append(np.full(deg, h))
        dst.append(nb)
    s = rng.integers(len(hubs), V - 50, size=extra)
    d = rng.integers(len(hubs), V - 50, size=extra)
    # skew: square-law endpoints make a wave band of medium degrees
    d = (len(hubs) + ((d - len(hubs)) ** 2) // (V - 50 - len(hubs))).astype(np.int64)
    src.append(s)
    dst.append(d)
    src.append(np.array([len(hubs) + 7, len(hubs) + 9]))   # self-loops
    dst.append(np.array([len(hubs) + 7, len(hubs) + 9]))
    s = np.concatenate(src).astype(np.int32)
    d = np.concatenate(dst).astype(np.int32)
    perm = rng.permutation(V).astype(np.int32)   # scramble ids
    return V, perm[s], perm[d]


def stale_units(leaves=10_000, leaf_loops=200):
    """A hub of > 8192 arcs (above the block tiers: tallied by 512-arc units) whose
    superstep-1 changes touch < 0.5 % of the arcs (leaves held by self-loops), so that
    superstep 2 runs on the exact frontier right after the column-run superstep 1.
    The hub row is dirty in superstep 2 only through x (a late unit); b sits in the
    hub row's first unit, keeps its label in superstep 1 and changes in superstep 2
    (to its cluster's label), so a unit word staged by an earlier run differs from the
    superstep-2 truth.  (the column-run path staged no unit words.)"""
    hub, b, c0, y = 0, 1, 2, 3
    nclu = 350
    clu = np.arange(4, 4 + nclu)
    lv = np.arange(4 + nclu, 4 + nclu + leaves)
    x = 4 + nclu + leaves
    V = x + 1
    e = []
    e.append(np.stack([np.full(leaves, hub), lv]))                      # hub - leaves
    e.append(np.stack([np.repeat(lv, leaf_loops), np.repeat(lv, leaf_loops)]))  # leaf self-loops
    e.append(np.stack([np.full(3, hub), np.full(3, b)]))                # b: 3 votes at the hub
    e.append(np.stack([np.full(300, b), np.full(300, b)]))              # b: 600 own votes
    e.append(np.stack([np.repeat(np.full(nclu, b), 2), np.repeat(clu, 2)]))  # b: 700 cluster votes
    e.append(np.stack([np.repeat(clu, 3), np.full(3 * nclu, c0)]))      # cluster -> c0 in superstep 1
    e.append(np.stack([np.full(200, x), np.full(200, y)]))              # x -> y in superstep 1
    e.append(np.stack([np.array([x]), np.array([hub])]))                # x dirties the hub row
    a = np.concatenate(e, axis=1).astype(np.int32)
    return V, a[0].copy(), a[1].copy()


def random_multigraph(V, m, seed):
    rng = np.random.default_rng(seed)
    return V, rng.integers(0, V, size=m).astype(np.int32), rng.integers(0, V, size=m).astype(np.int32)


def comb_bucket(labels, lg):
    """k_hub_combine's label-hash bucket (lpa_iter.hip comb_bucket)."""
    x = (labels.astype(np.uint64) * np.uint64(0x85EBCA77)) & np.uint64(0xFFFFFFFF)
    return (x >> np.uint64(32 - lg)).astype(np.int64) if lg else np.zeros(labels.shape, np.int64)


def giant_hub(seed=0, n_plain=200000, n_skew=20000, lg=7):
    """Hub 0 with n_plain + n_skew distinct neighbours (iteration 1: every staged
    word distinct -> 2^lg combine buckets), n_skew of which hash into ONE bucket
    (-> that bucket needs sub-bucket passes).  One skewed neighbour carries three
    parallel edges, so the hub's mode is decided inside the overloaded bucket; two
    plain neighbours carry two, testing the cross-bucket maximum."""
    rng = np.random.default_rng(seed)
    V = 4 * (n_plain + n_skew) + 1
    ids = np.arange(1, V, dtype=np.int64)
    b = comb_bucket(ids, lg)
    skew = rng.permutation(ids[b == 3])[:n_skew]
    rest = rng.permutation(ids[b != 3])[:n_plain]
    nb = np.concatenate([skew, rest, [skew[5]] * 2, [rest[7], rest[9]]])
    s = np.zeros(nb.size, np.int64)
    # a sparse random background so the leaves are not all degree 1
    bs = rng.integers(1, V, size=V // 2)
    bd = rng.integers(1, V, size=V // 2)
    return V, np.concatenate([s, bs]).astype(np.int32), np.concatenate([nb, bd]).astype(np.int32)


def comb_sub(labels, lg):
    """k_hub_bucket's sub-bucket hash (lpa_hub.hip comb_sub)."""
    x = (labels.astype(np.uint64) * np.uint64(0xC2B2AE3D)) & np.uint64(0xFFFFFFFF)
    return (x >> np.uint64(32 - lg)).astype(np.int64) if lg else np.zeros(labels.shape, np.int64)


def adversarial_hub(n_nb=20000, seed=0):
    """Hub 0 whose n_nb distinct neighbours ALL share one combine bucket (4 hash bits)
    and one sub-bucket (3 bits): in superstep 1 (labels = ids) its bucket pass meets
    n_nb > 8192 distinct labels, more than the LDS table holds (the case the spill
    guard must handle without dropping votes).  One neighbour carries a triple edge,
    so the hub's mode is decided inside that pass; a sparse background among the
    neighbours keeps later supersteps non-trivial."""
    rng = np.random.default_rng(seed)
    ids = np.arange(1, 200 * n_nb, dtype=np.int64)
    sel = ids[(comb_bucket(ids, 4) == 5) & (comb_sub(ids, 3) == 2)][:n_nb]
    assert sel.size == n_nb
    V = int(sel.max()) + 1
    nb = np.concatenate([rng.permutation(sel), [sel[17]] * 2])
    s = np.zeros(nb.size, np.int64)
    bs = rng.choice(sel, size=n_nb)
    bd = rng.choice(sel, size=n_nb)
    return V, np.concatenate([s, bs]).astype(np.int32), np.concatenate([nb, bd]).astype(np.int32)


def settled_hubs(seed=0, V=20000, n_hub=30, n_mover=40):
    """Nearly every vertex keeps its L0 label in superstep 1 (a self-loop = 2 votes
    for itself against single votes from distinct neighbours), so only the few
    `movers` (no self-loop) change and superstep 2 already runs on a frontier list
    -- with hub rows of 1024 < deg <= 4096, the rows the label-dense supersteps tally
    with one block each (k_lpa_block in list mode)."""
    rng = np.random.default_rng(seed)
    perm = rng.permutation(V)
    hubs, movers = perm[:n_hub], perm[n_hub:n_hub + n_mover]
    src, dst = [], []
    for h in hubs:
        nb = rng.choice(V, size=int(rng.integers(1100, 3000)), replace=False)
        nb = nb[nb != h]
        src.append(np.full(nb.size, h)), dst.append(nb)
    bg = rng.integers(0, V, size=(2 * V, 2))
    src.append(bg[:, 0]), dst.append(bg[:, 1])
    keep = np.setdiff1d(np.arange(V), movers)
    src.append(keep), dst.append(keep)                      # one self-loop each
    src.append(np.repeat(hubs, 2)), dst.append(np.repeat(hubs, 2))   # hubs: 3 in all
    for m in movers:                                        # 4 distinct hubs each
        hs = rng.choice(hubs, size=4, replace=False)
        src.append(np.full(4, m)), dst.append(hs)
    return V, np.concatenate(src).astype(np.int32), np.concatenate(dst).astype(np.int32)


def code_mix(src, dst, V0):
    """R-MAT edges (V0 vertices) plus structures whose superstep-2 mode is NOT the giant
    label, so that the giant-code settle of superstep 2 (lpa_iter.hip "Giant codes")
    leaves rows to its exact fallback paths: five 200-cliques (wave-bin rows, 199 arcs,
    their own block's label), a 1,100-clique (block-tier hub rows, glist) and a leader
    l < hub h pair sharing 9,000 two-arc members (rows of 9,000 arcs above the block
    tiers, ulist2: every member's superstep-1 label is l).  Returns V, src, dst."""
    es, ed = [src.astype(np.int64)], [dst.astype(np.int64)]
    nxt = V0

    def clique(n):
        nonlocal nxt
        ids = np.arange(nxt, nxt + n, dtype=np.int64)
        nxt += n
        iu, ju = np.triu_indices(n, 1)
        es.append(ids[iu])
        ed.append(ids[ju])

    for _ in range(5):
        clique(200)
    clique(1100)
    lead, hub = nxt, nxt + 1
    mem = np.arange(nxt + 2, nxt + 2 + 9000, dtype=np.int64)
    nxt += 9002
    es += [np.full(mem.size, hub), np.full(mem.size, lead)]
    ed += [mem, mem]
    return nxt, np.concatenate(es).astype(np.int32), np.concatenate(ed).astype(np.int32)

"""Generate tests/golden/r9_golden.npz from the reference's own sample data.

Run HERE only (needs /root/reference, absent on the GPU box):
    python tests/golden/make_golden.py

Input: /root/reference/CommunityDetection/data/outlinks_pq/*.snappy.parquet (R9),
restated into a graph exactly as Graphframes.py:16-73 builds it (package
``ingest`` module: null filter, distinct domains, sha1[:8] ids, undeduplicated
edges).  Expected outputs come from the CPU oracle (oracle/lpa_oracle.c),
cross-checked against the pure-Python restatement (oracle.lpa_py) before they
are written.  The fixture holds data only (ids, names, dense edges, labels).
"""
import importlib.util
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
PARQUET_DIR = "/root/reference/CommunityDetection/data/outlinks_pq"


def _load_ingest():
    pkg = [d for d in os.listdir(ROOT) if d.endswith("._amd")][0]
    spec = importlib.util.spec_from_file_location("_ingest", os.path.join(ROOT, pkg, "ingest.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    from oracle import oracle

    ingest = _load_ingest()
    df = ingest.read_outlinks(PARQUET_DIR)
    vertices, edges = ingest.build_graph(df)
    ids, src, dst = ingest.dense_edges(vertices, edges)
    assert (vertices["id"].to_numpy() == ids).all()
    V = ids.size
    names = vertices["name"].to_numpy().astype(str)

    max_iter = 10
    final10, hist, ties = oracle.lpa(V, src, dst, max_iter, per_iter=True)
    lab5 = hist[4]
    py5 = np.asarray(oracle.lpa_py(V, list(zip(src.tolist(), dst.tolist())), 5), dtype=np.int32)
    assert (py5 == lab5).all(), "C oracle disagrees with the pure-Python restatement"

    size, inc, flags, s1 = oracle.outlier_l1(V, src, dst, lab5)
    sub, flags2, s2 = oracle.outlier_l2(V, src, dst, lab5, 5)

    out = os.path.join(HERE, "r9_golden.npz")
    np.savez_compressed(
        out,
        ids=ids.astype("U8"), names=names, src=src, dst=dst,
        labels_iter=hist, ties=ties,
        l1_size=size, l1_inc=inc, l1_flags=flags.astype(np.uint8),
        l1_summary=np.array([s1["n_groups"], s1["k"], s1["thr"], s1["n_flagged"]], dtype=np.int64),
        l2_sub=sub, l2_flags=flags2.astype(np.uint8),
        l2_summary=np.array([s2["n_communities"], s2["n_subgroups"], s2["n_flagged"],
                             s2["n_communities_flagged"]], dtype=np.int64),
        rows_total=np.int64(18399), rows_after_filter=np.int64(len(df)),
    )
    print("V", V, "m", src.size, "communities@5", np.unique(lab5).size, "ties", ties.tolist())
    print("L1", s1, "L2", s2)
    print("wrote", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main()

"""Input construction for config C1 without Spark.

Restates /root/reference/CommunityDetection/Graphframes.py:16-73 with pyarrow +
hashlib instead of a SparkSession:

* ``:16``      read the outlinks parquet (4 nullable string columns ``_c0.._c3``);
* ``:26-30``   rename to Parent/ParentDomain/ChildDomain/Child and drop rows with a
               null ParentDomain or ChildDomain;
* ``:53``      vertices = distinct union of both domain columns;
* ``:57-58``   ``NodeHash(x) = sha1(utf8(x)).hexdigest()[:8]``;
* ``:67``      ``Graph_Vertices(id, name)``;
* ``:70-73``   ``Graph_Edges(src, dst)`` = hashed (ParentDomain, ChildDomain) per
               row, NOT deduplicated (a multigraph: duplicates are votes).

Spark's ``distinct()`` has no defined row order; the rows returned here are in
ascending ``id`` order, which is the order ``label_propagation`` returns anyway.
"""
from __future__ import annotations

import hashlib

import numpy as np
import pandas as pd

COLUMNS = {"_c0": "Parent", "_c1": "ParentDomain", "_c2": "ChildDomain", "_c3": "Child"}


def node_hash(x: str) -> str:
    """Graphframes.py:57-58."""
    return hashlib.sha1(x.encode("UTF-8")).hexdigest()[:8]


def read_outlinks(path: str) -> pd.DataFrame:
    """Graphframes.py:16 + :26-30 (rename, null filter).  ``path`` is one parquet
    file or a directory of ``*.snappy.parquet`` parts."""
    import glob
    import os

    import pyarrow.parquet as pq

    files = sorted(glob.glob(os.path.join(path, "*.snappy.parquet"))) if os.path.isdir(path) else [path]
    if not files:
        raise FileNotFoundError(f"no parquet parts under {path}")
    frames = [pq.read_table(f).to_pandas() for f in files]
    df = pd.concat(frames, ignore_index=True).rename(columns=COLUMNS)
    return df[df["ParentDomain"].notna() & df["ChildDomain"].notna()].reset_index(drop=True)


def build_graph(df: pd.DataFrame):
    """Graphframes.py:53-73.  Returns (vertices[id, name], edges[src, dst])."""
    names = pd.unique(pd.concat([df["ParentDomain"], df["ChildDomain"]], ignore_index=True))
    hashed = {n: node_hash(n) for n in names}
    vertices = pd.DataFrame({"id": [hashed[n] for n in names], "name": names})
    vertices = vertices.sort_values("id", kind="stable").reset_index(drop=True)
    edges = pd.DataFrame({"src": df["ParentDomain"].map(hashed).to_numpy(),
                          "dst": df["ChildDomain"].map(hashed).to_numpy()})
    return vertices, edges


def load_outlinks_graph(path: str):
    """Convenience: parquet -> (vertices, edges) exactly as Graphframes.py:16-73 builds them."""
    return build_graph(read_outlinks(path))


def dense_edges(vertices: pd.DataFrame, edges: pd.DataFrame):
    """Dense int32 edge arrays in ascending-unique-id order."""
    ids = np.unique(vertices["id"].to_numpy())
    s = np.searchsorted(ids, edges["src"].to_numpy())
    d = np.searchsorted(ids, edges["dst"].to_numpy())
    return ids, s.astype(np.int32), d.astype(np.int32)

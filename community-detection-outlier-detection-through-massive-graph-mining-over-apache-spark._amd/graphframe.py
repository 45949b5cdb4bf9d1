"""Drop-in for the reference's community-detection call surface.

The reference drives GraphFrames 0.6.0 from PySpark:

    Graphs = GraphFrame(Graph_Vertices, Graph_Edges)          # Graphframes.py:78
    Community_Graphs = Graphs.labelPropagation(maxIter=5)     # Graphframes.py:81

and then runs the outlier stage of Graphframes.py:92-137 over the result.
Here the same calls take pandas DataFrames (pyspark is not part of this
stack) and return a pandas DataFrame with every vertex column plus
``label`` (int64), computed by liblpa_hip.so on the GPU.

Id handling follows GraphFrames' ``indexedVertices`` / ``indexedEdges``
(SURVEY.md §8(a) a2, §8(b)):

* edges whose ``src`` or ``dst`` is not a vertex id are dropped (inner join);
* integral ids: ``label`` is the original id of the label vertex, so results are
  bit-comparable with GraphFrames on tie-free graphs;
* other ids (the reference's 8-hex-char SHA-1 strings): ``label`` is the dense
  index of the label vertex in ascending unique-id order (GraphFrames' own
  value, ``monotonically_increasing_id``, is partition-dependent and not
  reproducible; compare partitions, not values).

Ties are broken by the smallest label.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import pandas as pd

from .graph import Graph

ID, SRC, DST, LABEL = "id", "src", "dst", "label"


def _check_max_iter(maxIter):
    if not isinstance(maxIter, (int, np.integer)) or isinstance(maxIter, bool):
        raise TypeError(f"maxIter must be an int, got {type(maxIter).__name__}")
    if maxIter <= 0:
        # GraphX LabelPropagation.run: require(maxSteps > 0, ...)
        raise ValueError(f"requirement failed: Maximum of steps must be greater than 0, but got {maxIter}")


def _check_schema(v: pd.DataFrame, e: pd.DataFrame):
    # messages as raised by graphframes.GraphFrame.__init__ (0.6.0)
    if ID not in v.columns:
        raise ValueError("Vertex ID column {} missing from vertex DataFrame, which has columns: {}"
                         .format(ID, ",".join(map(str, v.columns))))
    if SRC not in e.columns:
        raise ValueError("Source vertex ID column {} missing from edge DataFrame, which has columns: {}"
                         .format(SRC, ",".join(map(str, e.columns))))
    if DST not in e.columns:
        raise ValueError("Destination vertex ID column {} missing from edge DataFrame, which has columns: {}"
                         .format(DST, ",".join(map(str, e.columns))))


@dataclass
class IndexedGraph:
    """Dense view of a (vertices, edges) pair: ids sorted ascending, int32 edges."""
    ids: np.ndarray          # unique vertex ids, ascending
    src: np.ndarray          # int32 dense
    dst: np.ndarray          # int32 dense
    integral: bool           # integral ids -> labels are original ids
    dropped_edges: int = 0

    @property
    def num_vertices(self) -> int:
        return int(self.ids.size)


def index_graph(v: pd.DataFrame, e: pd.DataFrame) -> IndexedGraph:
    ids_col = v[ID].to_numpy()
    integral = pd.api.types.is_integer_dtype(v[ID].dtype)
    ids = np.unique(ids_col)
    n = ids.size
    s_raw = e[SRC].to_numpy()
    d_raw = e[DST].to_numpy()
    if n == 0:
        return IndexedGraph(ids, np.empty(0, np.int32), np.empty(0, np.int32), integral, len(e))
    if integral:
        s_raw = s_raw.astype(ids.dtype, copy=False) if pd.api.types.is_integer_dtype(e[SRC].dtype) else s_raw
        d_raw = d_raw.astype(ids.dtype, copy=False) if pd.api.types.is_integer_dtype(e[DST].dtype) else d_raw
    s = np.searchsorted(ids, s_raw)
    d = np.searchsorted(ids, d_raw)
    s_ok = (s < n)
    d_ok = (d < n)
    s_ok[s_ok] = ids[s[s_ok]] == s_raw[s_ok]
    d_ok[d_ok] = ids[d[d_ok]] == d_raw[d_ok]
    keep = s_ok & d_ok
    return IndexedGraph(ids, s[keep].astype(np.int32), d[keep].astype(np.int32), integral,
                        int((~keep).sum()))


def _label_values(ig: IndexedGraph, dense_labels: np.ndarray) -> np.ndarray:
    if ig.integral:
        return ig.ids[dense_labels].astype(np.int64)
    return dense_labels.astype(np.int64)


def _attach(v: pd.DataFrame, ig: IndexedGraph, per_vertex: dict) -> pd.DataFrame:
    """Vertex rows (sorted by id, all columns kept) + per-vertex columns."""
    out = v.sort_values(ID, kind="stable").reset_index(drop=True)
    pos = np.searchsorted(ig.ids, out[ID].to_numpy())
    for name, values in per_vertex.items():
        out[name] = values[pos]
    return out


class GraphFrame:
    """``graphframes.GraphFrame`` call surface over pandas DataFrames.

    ``GraphFrame(v, e).labelPropagation(maxIter)`` mirrors Graphframes.py:78-81.
    """

    def __init__(self, v: pd.DataFrame, e: pd.DataFrame, device: int = 0):
        _check_schema(v, e)
        self._v = v
        self._e = e
        self._device = device
        self._ig = None
        self._graph = None

    @property
    def vertices(self) -> pd.DataFrame:
        return self._v

    @property
    def edges(self) -> pd.DataFrame:
        return self._e

    def _indexed(self) -> IndexedGraph:
        if self._ig is None:
            self._ig = index_graph(self._v, self._e)
        return self._ig

    def _gpu_graph(self) -> Graph:
        if self._graph is None:
            ig = self._indexed()
            self._graph = Graph(ig.src, ig.dst, ig.num_vertices, device=self._device)
        return self._graph

    def labelPropagation(self, maxIter: int) -> pd.DataFrame:
        """Static LPA for exactly ``maxIter`` synchronous supersteps (GraphX
        LabelPropagation.run via Pregel).  Returns vertices + ``label`` (int64)."""
        _check_max_iter(maxIter)
        ig = self._indexed()
        dense = self._gpu_graph().run(int(maxIter))
        return _attach(self._v, ig, {LABEL: _label_values(ig, dense)})

    def dense_labels(self, maxIter: int) -> np.ndarray:
        _check_max_iter(maxIter)
        return self._gpu_graph().run(int(maxIter))

    def degrees(self) -> pd.DataFrame:
        """Symmetrised degree per vertex (each directed edge counts at both ends)."""
        ig = self._indexed()
        return _attach(self._v, ig, {"degree": self._gpu_graph().degrees().astype(np.int64)})

    def outlierScores(self, labels: pd.DataFrame | None = None, mode: str = "L1", maxIter: int = 5,
                      subIter: int = 5) -> "OutlierResult":
        return outlier_scores(self._v, self._e, labels=labels, mode=mode, maxIter=maxIter,
                              subIter=subIter, _gf=self)

    def close(self):
        if self._graph is not None:
            self._graph.close()
            self._graph = None


def label_propagation(vertices: pd.DataFrame, edges: pd.DataFrame, maxIter: int,
                      device: int = 0) -> pd.DataFrame:
    """Function form of ``GraphFrame(vertices, edges).labelPropagation(maxIter)``."""
    gf = GraphFrame(vertices, edges, device=device)
    try:
        return gf.labelPropagation(maxIter)
    finally:
        gf.close()


@dataclass
class OutlierResult:
    """Outlier stage output.

    communities: one row per community ``label`` with ``size`` (members,
        Graphframes.py:100-104 / the print at :120) and ``incident_edges``
        (distinct directed edges touching it, len(Edges_List) at :115-118).
    vertices: vertex rows + ``label`` (+ ``sub_label`` in L2) + ``outlier`` flag.
    flagged_ids: ids of flagged vertices, ascending.
    summary: counts and the L1 threshold.
    """
    communities: pd.DataFrame
    vertices: pd.DataFrame
    flagged_ids: np.ndarray
    summary: dict = field(default_factory=dict)


def outlier_scores(vertices: pd.DataFrame, edges: pd.DataFrame, labels: pd.DataFrame | None = None,
                   mode: str = "L1", maxIter: int = 5, subIter: int = 5, device: int = 0,
                   _gf: GraphFrame | None = None) -> OutlierResult:
    """Community-size / incident-edge histograms and outlier flags on the GPU.

    ``labels``: a DataFrame with ``id`` and ``label`` as returned by
    ``labelPropagation`` (computed here with ``maxIter`` when omitted).
    mode "L1": threshold rule over top-level community sizes; "L2": second LPA
    (``subIter`` supersteps) on each community's induced, deduplicated edge set
    and the threshold rule per community (the commented Steps 5-6,
    Graphframes.py:121-137).
    """
    if mode not in ("L1", "L2"):
        raise ValueError(f"mode must be 'L1' or 'L2', got {mode!r}")
    gf = _gf if _gf is not None else GraphFrame(vertices, edges, device=device)
    try:
        ig = gf._indexed()
        g = gf._gpu_graph()
        if labels is None:
            _check_max_iter(maxIter)
            dense = g.run(int(maxIter))
        else:
            if ID not in labels.columns or LABEL not in labels.columns:
                raise ValueError("labels must have columns 'id' and 'label'")
            lab = labels.drop_duplicates(ID).set_index(ID)[LABEL]
            lab_vals = lab.reindex(ig.ids).to_numpy()
            if pd.isna(lab_vals).any():
                raise ValueError("labels must cover every vertex id")
            lab_vals = lab_vals.astype(np.int64)
            if ig.integral:
                dense = np.searchsorted(ig.ids, lab_vals)
                if (dense >= ig.num_vertices).any() or (ig.ids[np.minimum(dense, ig.num_vertices - 1)] != lab_vals).any():
                    raise ValueError("labels must be vertex ids")
            else:
                dense = lab_vals
            dense = dense.astype(np.int32)
        res = g.outlier(dense, mode=mode, sub_iter=subIter)
        size, inc, flags = res["size"], res["incident"], res["flags"]
        present = np.flatnonzero(size > 0)
        communities = pd.DataFrame({LABEL: _label_values(ig, present.astype(np.int64)),
                                    "size": size[present], "incident_edges": inc[present]})
        per_vertex = {LABEL: _label_values(ig, dense.astype(np.int64)), "outlier": flags}
        if res["sub_labels"] is not None:
            per_vertex["sub_label"] = _label_values(ig, res["sub_labels"].astype(np.int64))
        vdf = _attach(gf.vertices, ig, per_vertex)
        flagged = ig.ids[np.flatnonzero(flags)]
        return OutlierResult(communities, vdf, flagged, res["summary"])
    finally:
        if _gf is None:
            gf.close()

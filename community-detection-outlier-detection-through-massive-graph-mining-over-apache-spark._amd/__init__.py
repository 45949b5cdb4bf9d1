"""MI355X-native label propagation + outlier scoring (drop-in for the
GraphFrames ``labelPropagation`` path of
/root/reference/CommunityDetection/Graphframes.py).

Importable as ``graphframes_amd`` (see the shim at the repository root).  The
compute runs in liblpa_hip.so (hand-written HIP for gfx950, C ABI in
include/lpa.h); importing this package does not load it -- the first call does,
and fails loudly if it has not been built.
"""
from .graph import Graph, Loopback, comm_unique_id, gen_chunglu, gen_rmat, gen_sbm, run_ranks
from .graphframe import (GraphFrame, IndexedGraph, OutlierResult, index_graph, label_propagation,
                         outlier_scores)
from . import ingest

__all__ = ["Graph", "Loopback", "run_ranks", "GraphFrame", "IndexedGraph", "OutlierResult", "comm_unique_id", "gen_chunglu", "gen_rmat",
           "gen_sbm", "index_graph", "ingest", "label_propagation", "outlier_scores"]

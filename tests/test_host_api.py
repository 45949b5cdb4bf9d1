"""Host-side logic and the C-ABI boundary, no GPU needed: library loads and
exports every symbol include/lpa.h declares; argument checks that fire before
any device work; GraphFrames-compatible schema errors; id indexing (inner-join
semantics); ingest restatement of Graphframes.py:16-73."""
import os
import re

import numpy as np
import pandas as pd
import pytest

import graphframes_amd as gfa
from graphframes_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "lpa.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(lpa_\w+)\(", txt, re.M)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    syms = _header_symbols()
    assert len(syms) >= 17
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) == set(_lib.SIGNATURES), "ctypes signatures out of sync with include/lpa.h"


def _bundle_targets(data):
    """Target ids of the library's offload bundles: plain bundles carry them in the clear;
    compressed ones (csrc/Makefile builds with --offload-compress: a "CCOB" header, version,
    method, then the bundle's total size) are listed by clang-offload-bundler."""
    import shutil
    import struct
    import subprocess
    import tempfile

    if b"__CLANG_OFFLOAD_BUNDLE__" in data:
        return data.decode("latin-1")
    i = data.find(b"CCOB")
    assert i >= 0, "no offload bundle in the library"
    total = struct.unpack_from("<Q", data, i + 8)[0]
    tool = shutil.which("clang-offload-bundler") or "/opt/rocm/lib/llvm/bin/clang-offload-bundler"
    with tempfile.NamedTemporaryFile(suffix=".ccob") as f:
        f.write(data[i:i + total])
        f.flush()
        out = subprocess.run([tool, "--list", "--type=o", f"--input={f.name}"], capture_output=True, text=True,
                             check=True)
    return out.stdout


def test_library_is_hip_gfx950():
    data = open(_lib.LIB_PATH, "rb").read()
    # the kernels' host-side registration names, and a gfx950 device code object
    assert b"k_lpa_wave" in data and b"k_lpa_group" in data
    assert "gfx950" in _bundle_targets(data)


def test_no_device_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(_lib.LpaError, match="device"):
        gfa.Graph(np.array([0], np.int32), np.array([1], np.int32), 2)


def test_last_error_and_null_args():
    lib = _lib.load()
    assert lib.lpa_reset(None) == _lib.LPA_EINVAL
    assert "null handle" in _lib.last_error()
    assert lib.lpa_step(None, 1, None) == _lib.LPA_EINVAL
    assert lib.lpa_graph_get_info(None, None) == _lib.LPA_EINVAL
    assert lib.lpa_graph_get_info_sized(None, None, 8) == _lib.LPA_EINVAL
    # the ctypes struct matches this header version's layout
    hdr = open(os.path.join(ROOT, "include", "lpa.h")).read()
    assert lib.lpa_abi_version() == int(re.search(r"#define LPA_ABI_VERSION (\d+)", hdr).group(1))
    lib.lpa_graph_destroy(None)   # no-op


def test_schema_errors_match_graphframes():
    v = pd.DataFrame({"vid": [1]})
    e = pd.DataFrame({"src": [1], "dst": [1]})
    with pytest.raises(ValueError, match="Vertex ID column id missing from vertex DataFrame, which has columns: vid"):
        gfa.GraphFrame(v, e)
    with pytest.raises(ValueError, match="Source vertex ID column src missing"):
        gfa.GraphFrame(pd.DataFrame({"id": [1]}), pd.DataFrame({"a": [1], "dst": [1]}))
    with pytest.raises(ValueError, match="Destination vertex ID column dst missing"):
        gfa.GraphFrame(pd.DataFrame({"id": [1]}), pd.DataFrame({"src": [1], "b": [1]}))


def test_max_iter_checked_before_device():
    gf = gfa.GraphFrame(pd.DataFrame({"id": [1, 2]}), pd.DataFrame({"src": [1], "dst": [2]}))
    with pytest.raises(ValueError, match="requirement failed: Maximum of steps must be greater than 0, but got 0"):
        gf.labelPropagation(maxIter=0)
    with pytest.raises(ValueError, match="but got -3"):
        gfa.label_propagation(gf.vertices, gf.edges, -3)
    with pytest.raises(TypeError):
        gf.labelPropagation(maxIter=2.5)


def test_index_graph_inner_join_and_order():
    v = pd.DataFrame({"id": ["b", "a", "c", "a"], "name": ["B", "A", "C", "A2"]})
    e = pd.DataFrame({"src": ["a", "b", "zz", "c"], "dst": ["b", "c", "a", "q"]})
    ig = gfa.index_graph(v, e)
    assert ig.ids.tolist() == ["a", "b", "c"] and not ig.integral
    assert ig.src.tolist() == [0, 1] and ig.dst.tolist() == [1, 2]
    assert ig.dropped_edges == 2
    vi = pd.DataFrame({"id": np.array([30, 10, 20], dtype=np.int64)})
    ei = pd.DataFrame({"src": np.array([10, 30], dtype=np.int64), "dst": np.array([20, 10], dtype=np.int64)})
    ig = gfa.index_graph(vi, ei)
    assert ig.integral and ig.ids.tolist() == [10, 20, 30]
    assert ig.src.tolist() == [0, 2] and ig.dst.tolist() == [1, 0]


def test_ingest_restatement(golden):
    # Graphframes.py:53-73 on a tiny frame, then the committed R9 fixture
    df = pd.DataFrame({"Parent": ["p1", "p2", "p3"], "ParentDomain": ["a.com", "b.com", "a.com"],
                       "ChildDomain": ["b.com", "c.com", "b.com"], "Child": ["c1", "c2", "c3"]})
    v, e = gfa.ingest.build_graph(df)
    assert sorted(v["name"]) == ["a.com", "b.com", "c.com"]
    assert v["id"].tolist() == sorted(v["id"].tolist())
    assert len(e) == 3   # not deduplicated (duplicates are votes)
    assert gfa.ingest.node_hash("twitter.com") == __import__("hashlib").sha1(b"twitter.com").hexdigest()[:8]
    ids = golden["ids"]
    names = golden["names"]
    assert all(gfa.ingest.node_hash(n) == i for n, i in zip(names[:200], ids[:200]))


@pytest.mark.skipif(not os.path.isdir("/root/reference/CommunityDetection/data/outlinks_pq"),
                    reason="reference data only present in the build container")
def test_ingest_from_reference_parquet(golden):
    v, e = gfa.ingest.load_outlinks_graph("/root/reference/CommunityDetection/data/outlinks_pq")
    ids, s, d = gfa.ingest.dense_edges(v, e)
    assert np.array_equal(ids, golden["ids"]) and np.array_equal(s, golden["src"])
    assert np.array_equal(d, golden["dst"])


def test_loopback_group_host_side():
    """The loopback group is host state only: it is created and aborted without a GPU,
    and a handle on it checks the device like any other."""
    lb = gfa.Loopback(3)
    assert lb.nranks == 3
    lib = _lib.load()
    assert lib.lpa_loopback_create(0, None) == _lib.LPA_EINVAL
    import torch

    if not torch.cuda.is_available():
        with pytest.raises(_lib.LpaError, match="device"):
            gfa.Graph(np.array([0], np.int32), np.array([1], np.int32), 2, rank=1, loopback=lb)
    lb.abort()
    lb.close()
    lb.close()   # idempotent


def test_run_ranks_reraises_and_aborts():
    class _G:
        def __init__(self, lb):
            self._loopback = lb

    class _LB:
        aborted = 0

        def abort(self):
            _LB.aborted += 1

    lb = _LB()
    with pytest.raises(RuntimeError, match="rank 1"):
        gfa.run_ranks([_G(lb), _G(lb)], lambda r, g: (_ for _ in ()).throw(RuntimeError("rank 1")) if r else r)
    assert _LB.aborted == 1
    assert gfa.run_ranks([_G(lb), _G(lb)], lambda r, g: r * 10) == [0, 10]

"""ctypes binding of liblpa_hip.so (C ABI in include/lpa.h).

The library is the product: there is no CPU fallback.  If the shared object
is missing, loading fails loudly with instructions to build it.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# LPA_LIB_PATH: load a diagnostic build instead (profiling experiments only)
LIB_PATH = os.environ.get("LPA_LIB_PATH") or os.path.join(_HERE, "liblpa_hip.so")

LPA_OK = 0
LPA_EINVAL = -22
LPA_ENOMEM = -12
LPA_ENODEV = -19
LPA_EHIP = -1000
LPA_ERCCL = -2000
LPA_EOVERFLOW = -75
LPA_INPUT_DEVICE = 0x1
LPA_NBINS = 13
LPA_NKERNELS = 17
LPA_STATS_MAX_ITERS = 64
BIN_NAMES = ("seg", "w16", "w8", "w4", "w2", "g64", "g32", "g16", "g8", "g4", "g2", "g1", "isolated")
# timed kernels: the bin kernels plus the hub combine ("hub") and the al[] refresh
KERNEL_NAMES = ("k_lpa_units", "hub", "k_lpa_wave<16>", "k_lpa_wave<8>", "k_lpa_wave<4>", "k_lpa_wave<2>",
                "k_lpa_rows<64>", "k_lpa_rows<32>", "k_lpa_rows<16>", "k_lpa_rows<8>",
                "k_lpa_group<4>", "k_lpa_group<2>", "k_lpa_group<1>", "refresh", "k_al_rebuild_hot",
                "k_frontier_lists", "k_lpa_block")
KERNEL_BIN = {"k_lpa_units": "seg", "k_lpa_wave<16>": "w16", "k_lpa_wave<8>": "w8", "k_lpa_wave<4>": "w4", "k_lpa_wave<2>": "w2",
              "k_lpa_rows<64>": "g64", "k_lpa_rows<32>": "g32", "k_lpa_rows<16>": "g16",
              "k_lpa_rows<8>": "g8", "k_lpa_group<4>": "g4", "k_lpa_group<2>": "g2",
              "k_lpa_group<1>": "g1"}


class LpaStats(ctypes.Structure):
    _fields_ = [
        ("iters", ctypes.c_int32),
        ("n_iter_ms", ctypes.c_int32),
        ("iter_ms", ctypes.c_float * LPA_STATS_MAX_ITERS),
        ("kernel_ms", ctypes.c_float * LPA_NKERNELS),
        ("exchange_ms", ctypes.c_float),
        ("total_ms", ctypes.c_double),
    ]

    def to_dict(self):
        return dict(iters=self.iters, iter_ms=list(self.iter_ms[: self.n_iter_ms]),
                    kernel_ms={KERNEL_NAMES[k]: self.kernel_ms[k] for k in range(LPA_NKERNELS)},
                    exchange_ms=self.exchange_ms, total_ms=self.total_ms)


class LpaGraphInfo(ctypes.Structure):
    _fields_ = [
        ("V", ctypes.c_int64), ("m", ctypes.c_int64), ("arcs", ctypes.c_int64),
        ("slice", ctypes.c_int64), ("own_begin", ctypes.c_int64),
        ("rank", ctypes.c_int32), ("nranks", ctypes.c_int32), ("device", ctypes.c_int32),
        ("max_degree", ctypes.c_int32),
        ("bin_vertices", ctypes.c_int64 * LPA_NBINS), ("bin_arcs", ctypes.c_int64 * LPA_NBINS),
        ("hub_vertices", ctypes.c_int64), ("segments", ctypes.c_int64),
        ("device_bytes", ctypes.c_int64),
        ("exchanges_full", ctypes.c_int64), ("exchanges_delta", ctypes.c_int64),
        ("exchanges_giant", ctypes.c_int64),
        ("blocked_rows", ctypes.c_int64),
        ("blocked_pieces", ctypes.c_int64),
        ("code_refresh", ctypes.c_int64),
        ("graph_replays", ctypes.c_int64),
        ("exchanges_posted", ctypes.c_int64),
        ("exchanges_post_missed", ctypes.c_int64),
        ("gather_mode", ctypes.c_int64),
        ("host_allgathers", ctypes.c_int64),
    ]

    def to_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_ if k not in ("bin_vertices", "bin_arcs")}
        d["bin_vertices"] = {BIN_NAMES[b]: self.bin_vertices[b] for b in range(LPA_NBINS)}
        d["bin_arcs"] = {BIN_NAMES[b]: self.bin_arcs[b] for b in range(LPA_NBINS)}
        return d


class LpaQualitySummary(ctypes.Structure):
    _fields_ = [("n_communities", ctypes.c_int64), ("intra_arcs", ctypes.c_int64), ("arcs", ctypes.c_int64),
                ("degree_term", ctypes.c_double), ("modularity", ctypes.c_double)]

    def to_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class LpaOutlierSummary(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int64) for k in (
        "n_groups", "k", "threshold", "n_flagged", "n_communities", "n_communities_flagged",
        "distinct_edges")]

    def to_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


# every symbol include/lpa.h declares, with its ctypes signature
_vp = ctypes.c_void_p
_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)
_u8p = ctypes.POINTER(ctypes.c_uint8)
# lpa_allgather_fn: (send, recv, bytes_per_rank, ctx) -> 0 on success
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p)
SIGNATURES = {
    "lpa_graph_create": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                        ctypes.c_uint32, ctypes.POINTER(_vp)]),
    "lpa_comm_unique_id": (ctypes.c_int, [ctypes.c_char_p]),
    "lpa_graph_create_dist": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int32,
                                             ctypes.c_int32, ctypes.c_uint32, ctypes.c_int32,
                                             ctypes.c_int32, ctypes.c_char_p, ctypes.POINTER(_vp)]),
    "lpa_graph_create_hostcoll": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                                 ctypes.c_uint32, ctypes.c_int32, ctypes.c_int32, ALLGATHER_FN,
                                                 _vp, ctypes.POINTER(_vp)]),
    "lpa_set_stream": (ctypes.c_int, [_vp, _vp]),
    "lpa_set_serial": (ctypes.c_int, [_vp, ctypes.c_int32]),
    "lpa_set_frontier": (ctypes.c_int, [_vp, ctypes.c_int32]),
    "lpa_set_posted": (ctypes.c_int, [_vp, ctypes.c_int64]),
    "lpa_reset": (ctypes.c_int, [_vp]),
    "lpa_step": (ctypes.c_int, [_vp, ctypes.c_int32, ctypes.POINTER(LpaStats)]),
    "lpa_get_labels": (ctypes.c_int, [_vp, _vp, ctypes.c_int32]),
    "lpa_run": (ctypes.c_int, [_vp, ctypes.c_int32, _vp, ctypes.c_int32, ctypes.POINTER(LpaStats)]),
    "lpa_outlier": (ctypes.c_int, [_vp, _vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                   _i64p, _i64p, _i32p, _u8p, ctypes.POINTER(LpaOutlierSummary)]),
    "lpa_outlier_device": (ctypes.c_int, [_vp, _vp, ctypes.c_int32, ctypes.c_int32, _vp, _vp, _vp, _vp,
                                          ctypes.POINTER(LpaOutlierSummary)]),
    "lpa_degrees": (ctypes.c_int, [_vp, _i32p]),
    "lpa_quality": (ctypes.c_int, [_vp, _vp, ctypes.c_int32, _vp]),
    "lpa_loopback_create": (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(_vp)]),
    "lpa_loopback_abort": (None, [_vp]),
    "lpa_loopback_destroy": (None, [_vp]),
    "lpa_graph_create_loopback": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                                 ctypes.c_uint32, ctypes.c_int32, _vp, ctypes.POINTER(_vp)]),
    "lpa_exchange_get": (ctypes.c_int, [_vp, _i32p]),
    "lpa_exchange_put": (ctypes.c_int, [_vp, _i32p]),
    "lpa_exchange_get_delta": (ctypes.c_int, [_vp, _vp, _i64p]),
    "lpa_exchange_put_delta": (ctypes.c_int, [_vp, _vp, _i64p, ctypes.c_int64]),
    "lpa_abi_version": (ctypes.c_int, []),
    "lpa_graph_get_info": (ctypes.c_int, [_vp, ctypes.POINTER(LpaGraphInfo)]),
    "lpa_graph_get_info_sized": (ctypes.c_int, [_vp, ctypes.POINTER(LpaGraphInfo), ctypes.c_int64]),
    "lpa_graph_destroy": (None, [_vp]),
    "lpa_last_error": (ctypes.c_char_p, []),
    "lpa_gen_rmat": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int32,
                                    _vp, _vp, ctypes.c_int32, _vp]),
    "lpa_gen_sbm": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32,
                                   ctypes.c_uint64, _vp, _vp, ctypes.c_int32, _vp]),
    "lpa_gen_chunglu": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_double,
                                       ctypes.c_uint64, _vp, _vp, ctypes.c_int32, _vp]),
}

_lib = None


class LpaError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{msg} (lpa error {code})")
        self.code = code


def load():
    """Load liblpa_hip.so (fails loudly when it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: the HIP library has not been built. "
            "Run `python -c 'import __graft_entry__ as g; g.build()'` (or `make -C <pkg>/csrc`).")
    try:
        # One HIP runtime per process: torch-ROCm ships its own libamdhip64 /
        # librccl / libhsa-runtime64 (same sonames as /opt/rocm's).  Loading torch
        # first makes liblpa_hip.so bind to those already-loaded copies; loading
        # ours first would leave torch to open a second runtime that sees no GPU.
        import torch  # noqa: F401
    except ImportError:
        pass
    # LPA_LIB_PATH: a diagnostic build of the same library (csrc/Makefile `trace`)
    lib = ctypes.CDLL(os.environ.get("LPA_LIB_PATH") or LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def last_error() -> str:
    msg = load().lpa_last_error()
    return msg.decode("utf-8", "replace") if msg else ""


def check(rc: int):
    """Map a C-ABI return code onto a Python exception (ValueError for bad arguments,
    as GraphFrames raises for a bad schema / IllegalArgumentException for maxIter)."""
    if rc == LPA_OK:
        return
    msg = last_error()
    if rc == LPA_EINVAL:
        raise ValueError(msg)
    if rc == LPA_ENOMEM:
        raise MemoryError(msg)
    raise LpaError(rc, msg)

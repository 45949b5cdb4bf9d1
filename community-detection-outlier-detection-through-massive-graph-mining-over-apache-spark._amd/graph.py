"""Low-level handle over liblpa_hip.so: one built graph on one GPU (or one rank's slice).

Inputs are dense int32 edge arrays: host numpy arrays, or device tensors (any
object with ``data_ptr()`` and ``is_cuda``, e.g. torch-ROCm tensors), which are
handed to the C ABI as plain device pointers (torch is only the allocator).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib

OUTLIER_MODES = {"L1": 1, "L2": 2, 1: 1, 2: 2}


def _is_device_tensor(x) -> bool:
    return hasattr(x, "data_ptr") and getattr(x, "is_cuda", False)


def _edge_ptrs(src, dst):
    """Returns (src_ptr, dst_ptr, m, flags, keepalive)."""
    if _is_device_tensor(src) != _is_device_tensor(dst):
        raise ValueError("src and dst must both be host arrays or both device tensors")
    if _is_device_tensor(src):
        import torch

        if src.dtype != torch.int32 or dst.dtype != torch.int32:
            raise ValueError("device edge tensors must be int32")
        if src.numel() != dst.numel():
            raise ValueError("src/dst length mismatch")
        src = src.contiguous()
        dst = dst.contiguous()
        torch.cuda.current_stream(src.device).synchronize()
        return src.data_ptr(), dst.data_ptr(), int(src.numel()), _lib.LPA_INPUT_DEVICE, (src, dst)
    s = np.ascontiguousarray(src, dtype=np.int32)
    d = np.ascontiguousarray(dst, dtype=np.int32)
    if s.shape != d.shape or s.ndim != 1:
        raise ValueError("src/dst must be 1-D arrays of equal length")
    return s.ctypes.data, d.ctypes.data, int(s.size), 0, (s, d)


class Graph:
    """A symmetrised, degree-sorted CSR resident in HBM plus its label vectors.

    ``Graph(src, dst, V)`` builds on ``device``; ``Graph(..., rank=r, nranks=P,
    comm_id=id)`` builds rank r's slice for a P-GPU run (one process per GPU,
    RCCL allgather per superstep); ``Graph(..., rank=r, loopback=group)`` builds
    rank r of an in-process ``Loopback`` group (P handles on one device, one host
    thread each, the same exchange code with D2D copies for the allgather);
    ``comm_id=None`` with ``nranks > 1`` selects the caller-driven exchange
    (``exchange_get`` / ``exchange_put``); ``allgather=fn`` the host-staged collective
    (``lpa_graph_create_hostcoll``): the library's own exchange schedule with every
    allgather done by ``fn(send: np.ndarray[uint8]) -> bytes-like of nranks * send.size``
    (e.g. torch.distributed gloo between processes).
    """

    def __init__(self, src, dst, num_vertices: int, device: int = 0, rank: int = 0,
                 nranks: int = 1, comm_id: bytes | None = None, loopback: "Loopback | None" = None,
                 allgather=None):
        lib = _lib.load()
        self._lib = lib
        self._h = ctypes.c_void_p()
        self._allgather_cb = None
        self._allgather_err = None
        sp, dp, m, flags, keep = _edge_ptrs(src, dst)
        V = int(num_vertices)
        if V < 0 or V > np.iinfo(np.int32).max:
            raise ValueError(f"num_vertices out of range: {V}")
        if allgather is not None:
            P = int(nranks)

            def _cb(send, recv, nbytes, _ctx):
                try:
                    n = int(nbytes)
                    src_b = np.ctypeslib.as_array((ctypes.c_uint8 * max(n, 1)).from_address(send))[:n]
                    out = np.frombuffer(memoryview(allgather(src_b.copy())), dtype=np.uint8)
                    if out.size != P * n:
                        raise ValueError(f"allgather returned {out.size} bytes, expected {P * n}")
                    if n > 0:
                        ctypes.memmove(recv, out.ctypes.data, P * n)
                    return 0
                except BaseException as e:  # noqa: BLE001 -- reported after the failed call
                    self._allgather_err = e
                    return -1

            self._allgather_cb = _lib.ALLGATHER_FN(_cb)   # kept alive with the handle
            rc = lib.lpa_graph_create_hostcoll(sp, dp, m, V, device, flags, rank, P, self._allgather_cb, None,
                                               ctypes.byref(self._h))
        elif loopback is not None:
            nranks = loopback.nranks
            rc = lib.lpa_graph_create_loopback(sp, dp, m, V, device, flags, rank, loopback._handle(),
                                               ctypes.byref(self._h))
        elif nranks == 1 and comm_id is None:
            rc = lib.lpa_graph_create(sp, dp, m, V, device, flags, ctypes.byref(self._h))
        else:
            cid = None if comm_id is None else bytes(comm_id)
            if cid is not None and len(cid) != 128:
                raise ValueError("comm_id must be 128 bytes")
            rc = lib.lpa_graph_create_dist(sp, dp, m, V, device, flags, rank, nranks, cid,
                                           ctypes.byref(self._h))
        del keep
        _lib.check(rc)
        self.num_vertices = V
        self.num_edges = m
        self.device = device
        self.rank = rank
        self.nranks = nranks
        self._loopback = loopback   # the group must outlive the handle

    # -- lifetime ---------------------------------------------------------
    def close(self):
        if self._h:
            self._lib.lpa_graph_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _handle(self):
        if not self._h:
            raise ValueError("graph handle is closed")
        return self._h

    def _check(self, rc: int):
        """check() that re-raises a host allgather function's own exception as the cause."""
        err, self._allgather_err = self._allgather_err, None
        if rc != _lib.LPA_OK and err is not None:
            raise _lib.LpaError(rc, _lib.last_error()) from err
        _lib.check(rc)

    # -- LPA ----------------------------------------------------------------
    def info(self) -> dict:
        info = _lib.LpaGraphInfo()
        _lib.check(self._lib.lpa_graph_get_info_sized(self._handle(), ctypes.byref(info), ctypes.sizeof(info)))
        return info.to_dict()

    def reset(self):
        _lib.check(self._lib.lpa_reset(self._handle()))

    def step(self, n: int = 1, stats: bool = False):
        st = _lib.LpaStats() if stats else None
        self._check(self._lib.lpa_step(self._handle(), int(n), ctypes.byref(st) if stats else None))
        return st.to_dict() if stats else None

    def labels(self, out=None) -> np.ndarray:
        """Current labels by dense vertex id (host int32), or into a device tensor `out`."""
        if out is not None and _is_device_tensor(out):
            _lib.check(self._lib.lpa_get_labels(self._handle(), out.data_ptr(), 1))
            return out
        lab = np.empty(self.num_vertices, dtype=np.int32)
        _lib.check(self._lib.lpa_get_labels(self._handle(), lab.ctypes.data, 0))
        return lab

    def run(self, max_iter: int, stats: bool = False, out=None):
        """labelPropagation(maxIter): reset, exactly max_iter supersteps, labels
        (host int32 array, or written into the device tensor ``out``)."""
        st = _lib.LpaStats() if stats else None
        if out is not None and _is_device_tensor(out):
            if out.numel() != self.num_vertices:
                raise ValueError(f"out must hold {self.num_vertices} labels")
            lab, ptr, on_dev = out, out.data_ptr(), 1
        else:
            lab = np.empty(self.num_vertices, dtype=np.int32)
            ptr, on_dev = lab.ctypes.data, 0
        self._check(self._lib.lpa_run(self._handle(), int(max_iter), ptr, on_dev,
                                      ctypes.byref(st) if stats else None))
        return (lab, st.to_dict()) if stats else lab

    def degrees(self) -> np.ndarray:
        deg = np.empty(self.num_vertices, dtype=np.int32)
        _lib.check(self._lib.lpa_degrees(self._handle(), deg.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
        return deg

    def set_frontier(self, on: bool = True):
        """Re-tally only rows with a changed neighbour (exact; default on) or every row."""
        _lib.check(self._lib.lpa_set_frontier(self._handle(), int(bool(on))))

    def set_posted(self, cap: int = -1):
        """P > 1: posted delta exchange capacity (-1 adaptive, 0 off, > 0 fixed; labels identical)."""
        _lib.check(self._lib.lpa_set_posted(self._handle(), int(cap)))

    def set_serial(self, serial: bool = True):
        """Profiling: queue every tally kernel on one stream (standalone kernel times)."""
        _lib.check(self._lib.lpa_set_serial(self._handle(), int(bool(serial))))

    # -- caller-driven exchange (virtual ranks) -------------------------------
    def exchange_get(self) -> np.ndarray:
        sl = np.empty(self.info()["slice"], dtype=np.int32)
        _lib.check(self._lib.lpa_exchange_get(self._handle(), sl.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
        return sl

    def exchange_put(self, full: np.ndarray):
        full = np.ascontiguousarray(full, dtype=np.int32)
        _lib.check(self._lib.lpa_exchange_put(self._handle(), full.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))

    def exchange_get_delta(self) -> np.ndarray:
        """This rank's changed owned labels as (local slot << 32 | label) entries."""
        buf = np.empty(max(self.info()["slice"], 1), dtype=np.uint64)
        n = ctypes.c_int64(0)
        _lib.check(self._lib.lpa_exchange_get_delta(self._handle(), buf.ctypes.data_as(ctypes.c_void_p),
                                                    ctypes.byref(n)))
        return buf[: n.value].copy()

    def exchange_put_delta(self, per_rank):
        """Apply every rank's delta entries (list in rank order)."""
        cap = max((e.size for e in per_rank), default=0)
        P = len(per_rank)
        table = np.zeros((P, max(cap, 1)), dtype=np.uint64)
        for r, e in enumerate(per_rank):
            table[r, : e.size] = e
        counts = np.array([e.size for e in per_rank], dtype=np.int64)
        _lib.check(self._lib.lpa_exchange_put_delta(self._handle(), table.ctypes.data_as(ctypes.c_void_p),
                                                    counts.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                                    cap))

    # -- outlier stage --------------------------------------------------------
    def outlier(self, labels, mode="L1", sub_iter: int = 5):
        """Appendix B outlier stage.  Returns dict(size, incident, sub_labels, flags, summary):
        host numpy arrays for host labels; for a device label tensor (int32, this
        handle's device) every output is a device tensor of this device and nothing is
        staged through the host (lpa_outlier_device)."""
        if mode not in OUTLIER_MODES:
            raise ValueError(f"mode must be 'L1' or 'L2', got {mode!r}")
        md = OUTLIER_MODES[mode]
        V = self.num_vertices
        if _is_device_tensor(labels):
            return self._outlier_device(labels, md, sub_iter)
        lab = np.ascontiguousarray(labels, dtype=np.int32)
        if lab.shape != (V,):
            raise ValueError(f"labels must have shape ({V},)")
        size = np.empty(V, dtype=np.int64)
        inc = np.empty(V, dtype=np.int64)
        sub = np.empty(V, dtype=np.int32) if md == 2 else None
        flags = np.empty(V, dtype=np.uint8)
        summ = _lib.LpaOutlierSummary()
        i64p = ctypes.POINTER(ctypes.c_int64)
        _lib.check(self._lib.lpa_outlier(
            self._handle(), lab.ctypes.data, 0, md, int(sub_iter),
            size.ctypes.data_as(i64p), inc.ctypes.data_as(i64p),
            sub.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)) if sub is not None else None,
            flags.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), ctypes.byref(summ)))
        return dict(size=size, incident=inc, sub_labels=sub, flags=flags.astype(bool),
                    summary=summ.to_dict())


    def _outlier_device(self, labels, md: int, sub_iter: int):
        import torch

        V = self.num_vertices
        if labels.dtype != torch.int32:
            raise ValueError(f"device labels must be int32, got {labels.dtype}")
        if labels.device.index != self.device:
            raise ValueError(f"device labels must be on cuda:{self.device}, got {labels.device}")
        if labels.numel() != V:
            raise ValueError(f"labels must hold {V} entries")
        lab = labels.contiguous()
        dev = lab.device
        size = torch.empty(V, dtype=torch.int64, device=dev)
        inc = torch.empty(V, dtype=torch.int64, device=dev)
        sub = torch.empty(V, dtype=torch.int32, device=dev) if md == 2 else None
        flags = torch.empty(V, dtype=torch.uint8, device=dev)
        torch.cuda.current_stream(dev).synchronize()   # the library works on its own stream
        summ = _lib.LpaOutlierSummary()
        _lib.check(self._lib.lpa_outlier_device(
            self._handle(), lab.data_ptr(), md, int(sub_iter), size.data_ptr(), inc.data_ptr(),
            sub.data_ptr() if sub is not None else None, flags.data_ptr(), ctypes.byref(summ)))
        return dict(size=size, incident=inc, sub_labels=sub, flags=flags.bool(), summary=summ.to_dict())

    def quality(self, labels) -> dict:
        """Community count and modularity of a labelling (host array or device tensor of
        dense-id labels) on this graph's symmetrised multigraph (lpa_quality)."""
        q = _lib.LpaQualitySummary()
        if _is_device_tensor(labels):
            import torch

            # the library reads V int32 values on its own stream (as _edge_ptrs guards the
            # edge tensors): wrong dtype / device would be read silently, an unfinished
            # producer on torch's stream too early
            if labels.dtype != torch.int32:
                raise ValueError(f"device labels must be int32, got {labels.dtype}")
            if labels.device.index != self.device:
                raise ValueError(f"device labels must be on cuda:{self.device}, got {labels.device}")
            if labels.numel() != self.num_vertices:
                raise ValueError(f"labels must hold {self.num_vertices} entries")
            lab, on_dev = labels.contiguous(), 1
            torch.cuda.current_stream(lab.device).synchronize()
            ptr = lab.data_ptr()
        else:
            lab = np.ascontiguousarray(labels, dtype=np.int32)
            if lab.shape != (self.num_vertices,):
                raise ValueError(f"labels must have shape ({self.num_vertices},)")
            ptr, on_dev = lab.ctypes.data, 0
        _lib.check(self._lib.lpa_quality(self._handle(), ptr, on_dev, ctypes.byref(q)))
        return q.to_dict()


class Loopback:
    """In-process collective group of ``nranks`` handles on one device (the
    multi-GPU exchange rehearsed on one GPU).  Drive each rank's Graph from its own
    thread; ctypes releases the GIL during the library calls."""

    def __init__(self, nranks: int):
        self._lib = _lib.load()
        self._h = ctypes.c_void_p()
        _lib.check(self._lib.lpa_loopback_create(int(nranks), ctypes.byref(self._h)))
        self.nranks = int(nranks)

    def _handle(self):
        if not self._h:
            raise ValueError("loopback group is closed")
        return self._h

    def abort(self):
        """Release every thread blocked in a collective of this group (they fail)."""
        if self._h:
            self._lib.lpa_loopback_abort(self._h)

    def close(self):
        if self._h:
            self._lib.lpa_loopback_destroy(self._h)
            self._h = ctypes.c_void_p()


def run_ranks(graphs, fn):
    """Call ``fn(rank, graph)`` for every rank of a loopback group on its own thread;
    returns the results in rank order, re-raising the first failure in time (after
    aborting the group so no thread stays blocked in a collective)."""
    import threading

    res = [None] * len(graphs)
    errs = []   # in the order the ranks failed: the first is the cause, the rest
    lock = threading.Lock()   # are peers released by the abort

    def work(r):
        try:
            res[r] = fn(r, graphs[r])
        except BaseException as e:  # noqa: BLE001 -- re-raised below
            with lock:
                errs.append(e)
            lb = graphs[r]._loopback
            if lb is not None:
                lb.abort()

    th = [threading.Thread(target=work, args=(r,)) for r in range(len(graphs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]
    return res


def comm_unique_id() -> bytes:
    """RCCL unique id for a distributed build (create on one rank, broadcast)."""
    buf = ctypes.create_string_buffer(128)
    _lib.check(_lib.load().lpa_comm_unique_id(buf))
    return buf.raw


def gen_rmat(scale: int, edgefactor: int = 16, seed: int = 1, scramble: bool = True, device: int = 0):
    """R-MAT edge list generated in HBM (torch int32 tensors on `device`)."""
    import torch

    m = edgefactor << scale
    dev = torch.device("cuda", device)
    src = torch.empty(m, dtype=torch.int32, device=dev)
    dst = torch.empty(m, dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)
    _lib.check(_lib.load().lpa_gen_rmat(scale, m, seed, int(scramble), src.data_ptr(), dst.data_ptr(),
                                        device, None))
    return src, dst


def gen_sbm(num_vertices: int, blocks: int, m: int, seed: int = 20261015,
            p_in_q32: int = 3865470566, device: int = 0):
    """Planted-partition SBM edge list generated in HBM (p_in = p_in_q32 / 2^32)."""
    import torch

    dev = torch.device("cuda", device)
    src = torch.empty(m, dtype=torch.int32, device=dev)
    dst = torch.empty(m, dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)
    _lib.check(_lib.load().lpa_gen_sbm(num_vertices, blocks, m, p_in_q32, seed, src.data_ptr(),
                                       dst.data_ptr(), device, None))
    return src, dst


def gen_chunglu(num_vertices: int, m: int, gamma: float = 2.1, max_deg: float = 0.0, seed: int = 7,
                device: int = 0):
    """Chung-Lu power-law edge list generated in HBM (config C5: heavy hubs)."""
    import torch

    dev = torch.device("cuda", device)
    src = torch.empty(m, dtype=torch.int32, device=dev)
    dst = torch.empty(m, dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)
    _lib.check(_lib.load().lpa_gen_chunglu(num_vertices, m, gamma, max_deg, seed, src.data_ptr(),
                                           dst.data_ptr(), device, None))
    return src, dst

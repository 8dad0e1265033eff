"""Host-side API over libdervet_hip: batch solve of window LPs.

``BatchSolver.solve(lps)`` is the batched replacement of the per-window
``storagevet Scenario.solve_optimization(functions, constraints)`` call made at
``dervet/MicrogridScenario.py:319``: it takes every window's canonical LP (CSR K with equality rows first,
then >= rows; c, c0, q, l, u) and returns per-window primal/dual solutions, objective and status.
``BatchSolver.solve_packed`` runs a batch that is already resident in HBM (torch tensors), which is what
``bench.py`` times.
"""
import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _lib


@dataclass
class WindowLP:
    """One window's LP:  min c'x + c0  s.t.  K[:m_eq] x = q[:m_eq],  K[m_eq:] x >= q[m_eq:],  l <= x <= u."""
    indptr: np.ndarray
    indices: np.ndarray
    data: np.ndarray
    c: np.ndarray
    q: np.ndarray
    l: np.ndarray
    u: np.ndarray
    m_eq: int
    c0: float = 0.0
    structure: int = 0
    meta: dict = field(default_factory=dict)

    @property
    def n(self):
        return len(self.c)

    @property
    def m(self):
        return len(self.q)

    @classmethod
    def from_csr(cls, K, q, c, l, u, m_eq, c0=0.0, **kw):
        K = K.tocsr()
        K.sort_indices()
        return cls(np.ascontiguousarray(K.indptr, np.int32), np.ascontiguousarray(K.indices, np.int32),
                   np.ascontiguousarray(K.data, np.float64), np.ascontiguousarray(c, np.float64),
                   np.ascontiguousarray(q, np.float64), np.ascontiguousarray(l, np.float64),
                   np.ascontiguousarray(u, np.float64), int(m_eq), float(c0), **kw)


@dataclass
class WindowResult:
    x: np.ndarray
    y: np.ndarray
    obj: float
    status: int
    iters: int
    primal_res_rel: float
    dual_res_rel: float
    gap_rel: float

    @property
    def status_name(self):
        return _lib.STATUS_NAMES.get(self.status, "solver_error")


class SolverError(RuntimeError):
    pass


def _init_torch_first():
    """Let PyTorch (device memory, streams, torch.distributed in this package) create its HIP context before the
    library's first HIP call: on the GPU box, torch.cuda.is_available() reported no device when libdervet_hip
    had initialised HIP first in the process."""
    try:
        import torch
    except ImportError:
        return
    if torch.cuda.is_available():
        torch.cuda.init()


class BatchSolver:
    """A libdervet_hip handle: one GPU (``device``) or several (``devices``: a host-buffer batch is split over them
    and solved concurrently; devices may repeat).  Options are dvh_options fields (eps, max_iters, ...)."""

    def __init__(self, device=0, devices=None, **options):
        _init_torch_first()
        self._lib = _lib.load()
        self._opts = _lib.default_options(**options)
        h = ctypes.c_void_p()
        if devices is None:
            rc = self._lib.dvh_create(1 << int(device), ctypes.byref(self._opts), ctypes.byref(h))
        else:
            arr = (ctypes.c_int32 * len(devices))(*[int(d) for d in devices])
            rc = self._lib.dvh_create_devices(arr, len(devices), ctypes.byref(self._opts), ctypes.byref(h))
        if rc != 0:
            raise SolverError(f"dvh_create failed ({rc}): no usable GPU device {devices or device} or invalid options")
        self._h = h

    @property
    def device_count(self):
        return int(self._lib.dvh_device_count(self._h))

    def close(self):
        if getattr(self, "_h", None):
            self._lib.dvh_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc, what):
        if rc != 0:
            msg = self._lib.dvh_last_error(self._h)
            raise SolverError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")

    def options(self):
        """The handle's current dvh_options (a copy)."""
        o = type(self._opts)()
        ctypes.pointer(o)[0] = self._opts
        return o

    def set_options(self, **options):
        for k, v in options.items():
            setattr(self._opts, k, v)
        self._check(self._lib.dvh_set_options(self._h, ctypes.byref(self._opts)), "dvh_set_options")

    def timing(self):
        t = (ctypes.c_double * 3)()
        self._check(self._lib.dvh_last_timing(self._h, t), "dvh_last_timing")
        return {"total_ms": t[0], "setup_ms": t[1], "pdhg_ms": t[2]}

    def kernel_stats(self):
        v = (ctypes.c_int32 * 4)()
        self._check(self._lib.dvh_last_stats(self._h, v), "dvh_last_stats")
        c = (ctypes.c_int32 * 5)()
        self._check(self._lib.dvh_last_path_counts5(self._h, c), "dvh_last_path_counts5")
        a = ctypes.c_int32()
        self._check(self._lib.dvh_last_chain_aborts(self._h, ctypes.byref(a)), "dvh_last_chain_aborts")
        return {"band_windows": c[3], "ell_windows": v[0], "generic_windows": v[1], "variant": v[2],
                "generic_only": bool(v[3]), "large_windows": c[2], "chain_windows": c[4],
                "chain_aborts": int(a.value)}

    def last_warning(self):
        """Diagnostics of the last solve's fallbacks (a medium-tier team launch that aborted), or ''."""
        return (self._lib.dvh_last_warning(self._h) or b"").decode()

    def host_syncs(self):
        """Host waits on the stream during the last solve (dvh_last_host_syncs)."""
        v = ctypes.c_int32()
        self._check(self._lib.dvh_last_host_syncs(self._h, ctypes.byref(v)), "dvh_last_host_syncs")
        return int(v.value)

    _PATHS = {"default": 0, "generic": 1, "ell": 2, "band1": 3, "band3": 4}

    def set_kernel_path(self, path):
        """Kernel cascade: "default" (battery-banded -> ELL -> generic CSR), "ell" (ELL -> generic), "generic", or
        "band1" / "band3" (the default cascade with the battery band kernel's form forced: one step per lane, 768
        threads / three steps per lane, 256 threads, two windows per CU; the default picks one-step for batches of
        at most one battery window per CU).  A bool selects "generic" (True) / "default" (False)."""
        mode = (1 if path else 0) if isinstance(path, bool) else self._PATHS[path]
        self._check(self._lib.dvh_set_kernel_path(self._h, mode), "dvh_set_kernel_path")

    def set_launch_order(self, order):
        """The next solve launches its battery-band pass over the windows in this order (a permutation of the batch's
        window indices; scheduling only, the results do not depend on it).  None / empty clears."""
        o = np.ascontiguousarray(np.zeros(0, np.int32) if order is None else order, np.int32)
        self._check(self._lib.dvh_set_launch_order(self._h, o.ctypes.data_as(ctypes.c_void_p), len(o)),
                    "dvh_set_launch_order")

    def solve(self, lps, start=None):
        """Solve a list of WindowLP on the GPU; returns a list of WindowResult (same order).

        start: optional list of (x, y) starting points (unscaled; None entries start cold), used when the
        solver's ``warm_start`` option is set (battery-banded windows)."""
        count = len(lps)
        if count == 0:
            return []
        keep = []
        arr = (_lib.LP * count)()
        res = (_lib.Result * count)()
        outs = []

        def ptr(a, t, ct):
            a = np.ascontiguousarray(a, dtype=t)
            keep.append(a)
            return a.ctypes.data_as(ct)

        for k, lp in enumerate(lps):
            m = lp.m
            if len(lp.indptr) != m + 1:
                raise ValueError(f"window {k}: indptr has {len(lp.indptr)} entries, expected m+1={m + 1}")
            L = arr[k]
            L.n, L.m_eq, L.m_ineq, L.nnz = lp.n, lp.m_eq, m - lp.m_eq, len(lp.indices)
            L.indptr = ptr(lp.indptr, np.int32, _lib.c_int32_p)
            L.indices = ptr(lp.indices, np.int32, _lib.c_int32_p)
            L.data = ptr(lp.data, np.float64, _lib.c_double_p)
            L.c = ptr(lp.c, np.float64, _lib.c_double_p)
            L.q = ptr(lp.q, np.float64, _lib.c_double_p)
            L.l = ptr(lp.l, np.float64, _lib.c_double_p)
            L.u = ptr(lp.u, np.float64, _lib.c_double_p)
            L.c0 = lp.c0
            L.structure = lp.structure
            x = np.zeros(lp.n)
            y = np.zeros(m)
            if start is not None and start[k] is not None:
                x[:] = start[k][0]
                y[:] = start[k][1]
            outs.append((x, y))
            res[k].x = x.ctypes.data_as(_lib.c_double_p)
            res[k].y = y.ctypes.data_as(_lib.c_double_p) if m else None
        self._check(self._lib.dvh_solve_batch(self._h, arr, count, res), "dvh_solve_batch")
        return [WindowResult(outs[k][0], outs[k][1], res[k].obj, res[k].status, res[k].iters, res[k].primal_res_rel,
                             res[k].dual_res_rel, res[k].gap_rel) for k in range(count)]

    # ---- the result all-gather across ranks, through the library's own RCCL communicator (dvh_comm_*)
    def comm_unique_id(self):
        """128 bytes from ncclGetUniqueId (rank 0 draws it; the launcher hands it to every rank)."""
        buf = ctypes.create_string_buffer(_lib.COMM_ID_BYTES)
        self._check(self._lib.dvh_comm_unique_id(self._h, buf), "dvh_comm_unique_id")
        return buf.raw

    def comm_init(self, rank, world, uid):
        if len(uid) != _lib.COMM_ID_BYTES:
            raise ValueError(f"a communicator id has {_lib.COMM_ID_BYTES} bytes, got {len(uid)}")
        self._check(self._lib.dvh_comm_init(self._h, int(rank), int(world), bytes(uid)), "dvh_comm_init")

    def comm_info(self):
        v = (ctypes.c_int32 * 2)()
        self._check(self._lib.dvh_comm_info(self._h, v), "dvh_comm_info")
        return int(v[0]), int(v[1])

    def gather_results(self, rows, out, stream=None):
        """out (device, world x rows' bytes) = every rank's ``rows`` (a contiguous device tensor) in rank order, enqueued
        on ``stream`` (a torch stream or a hipStream_t; None = the solver's own stream)."""
        if not rows.is_contiguous() or not out.is_contiguous():
            raise ValueError("gather_results needs contiguous tensors")
        nb = rows.numel() * rows.element_size()
        world = self.comm_info()[1]
        if world and out.numel() * out.element_size() != nb * world:
            raise ValueError("out must hold world x the rows' bytes")
        s = getattr(stream, "cuda_stream", stream)
        self._check(self._lib.dvh_gather_results(self._h, ctypes.c_void_p(rows.data_ptr()), nb,
                                                 ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(s or 0)),
                    "dvh_gather_results")

    def solve_packed(self, pb, stream=None, sync=True):
        """Solve a device-resident packed batch (``dervet_hip.packed.PackedBatch`` of torch tensors)."""
        p = pb.as_ctypes()
        s = ctypes.c_void_p(stream) if stream else None
        self._check(self._lib.dvh_solve_packed_device(self._h, ctypes.byref(p), s), "dvh_solve_packed_device")
        if sync and stream:
            self._check(self._lib.dvh_synchronize(self._h), "dvh_synchronize")


def version():
    return _lib.load().dvh_version().decode()

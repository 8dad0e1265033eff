"""Packed batch layout (dvh_packed in include/dervet_hip.h): all windows' CSR, vectors and outputs as
flat arrays, with an int64 descriptor per window {n, m, m_eq, nnz, off_row, off_nz, off_n, off_m}.

This is the HBM layout the kernels read.  Arrays may be numpy (host) or torch
tensors (device); ``as_ctypes`` requires device tensors.
"""
from dataclasses import dataclass

import numpy as np

from . import _lib

IN_FIELDS = ("desc", "indptr", "indices", "data", "c", "c0", "q", "l", "u")
OUT_FIELDS = ("x", "y", "stats", "istats")


@dataclass
class PackedBatch:
    desc: object      # int64 [count, 8]
    indptr: object    # int32 [sum(m+1)]
    indices: object   # int32 [sum nnz]
    data: object      # f64   [sum nnz]
    c: object         # f64   [sum n]
    c0: object        # f64   [count]
    q: object         # f64   [sum m]
    l: object         # f64   [sum n]
    u: object         # f64   [sum n]
    x: object = None  # f64   [sum n]   (outputs)
    y: object = None  # f64   [sum m]
    stats: object = None   # f64 [count, 4] obj, primal_res_rel, dual_res_rel, gap_rel
    istats: object = None  # int32 [count, 2] status, iters

    @property
    def count(self):
        return int(self.desc.shape[0])

    def sizes(self):
        return dict(total_n=int(self.c.shape[0]), total_m=int(self.q.shape[0]), total_nnz=int(self.data.shape[0]),
                    total_rows=int(self.indptr.shape[0]))

    def alloc_outputs(self):
        tn, tm = int(self.c.shape[0]), int(self.q.shape[0])
        if isinstance(self.c, np.ndarray):
            self.x, self.y = np.zeros(tn), np.zeros(max(tm, 1))
            self.stats, self.istats = np.zeros((self.count, 4)), np.zeros((self.count, 2), np.int32)
        else:
            import torch
            dev = self.c.device
            self.x = torch.zeros(tn, dtype=torch.float64, device=dev)
            self.y = torch.zeros(max(tm, 1), dtype=torch.float64, device=dev)
            self.stats = torch.zeros((self.count, 4), dtype=torch.float64, device=dev)
            self.istats = torch.zeros((self.count, 2), dtype=torch.int32, device=dev)
        return self

    def to_torch(self, device):
        import torch
        kw = {}
        for f in IN_FIELDS + OUT_FIELDS:
            v = getattr(self, f)
            kw[f] = None if v is None else torch.as_tensor(np.ascontiguousarray(v)).to(device)
        return PackedBatch(**kw)

    def to_numpy(self):
        kw = {}
        for f in IN_FIELDS + OUT_FIELDS:
            v = getattr(self, f)
            kw[f] = None if v is None else (v if isinstance(v, np.ndarray) else v.detach().cpu().numpy())
        return PackedBatch(**kw)

    def as_ctypes(self):
        import torch
        p = _lib.Packed()
        p.count = self.count
        for k, v in self.sizes().items():
            setattr(p, k, v)
        for f in IN_FIELDS + OUT_FIELDS:
            t = getattr(self, f)
            if t is None:
                raise ValueError(f"packed batch field {f} not set (call alloc_outputs)")
            if not isinstance(t, torch.Tensor) or not t.is_cuda or not t.is_contiguous():
                raise ValueError(f"packed batch field {f} must be a contiguous device tensor")
            setattr(p, f, t.data_ptr())
        return p

    # ---- per-window views (host; slices of a device batch are copied to the host)
    def window(self, k):
        h = lambda v: v.detach().cpu().numpy() if hasattr(v, "detach") else v  # noqa: E731
        d = h(self.desc[k])
        n, m, meq, nnz, orow, onz, on, om = (int(v) for v in d)
        return dict(n=n, m=m, m_eq=meq, nnz=nnz, indptr=h(self.indptr[orow:orow + m + 1]),
                    indices=h(self.indices[onz:onz + nnz]), data=h(self.data[onz:onz + nnz]), c=h(self.c[on:on + n]),
                    l=h(self.l[on:on + n]), u=h(self.u[on:on + n]), q=h(self.q[om:om + m]), c0=float(self.c0[k]),
                    x=None if self.x is None else h(self.x[on:on + n]),
                    y=None if self.y is None else h(self.y[om:om + m]))

    def window_lp(self, k):
        """Window k as a solver.WindowLP (host copies)."""
        from .solver import WindowLP
        w = self.window(k)
        ip = np.asarray(w["indptr"], np.int32)
        return WindowLP(ip - ip[0], np.array(w["indices"], np.int32), np.array(w["data"]), np.array(w["c"]),
                        np.array(w["q"]), np.array(w["l"]), np.array(w["u"]), w["m_eq"], w["c0"])


def pack(lps):
    """Concatenate a list of solver.WindowLP into a numpy PackedBatch."""
    count = len(lps)
    desc = np.zeros((count, 8), np.int64)
    tr = tz = tn = tm = 0
    for k, lp in enumerate(lps):
        desc[k] = (lp.n, lp.m, lp.m_eq, len(lp.indices), tr, tz, tn, tm)
        tr += lp.m + 1
        tz += len(lp.indices)
        tn += lp.n
        tm += lp.m
    cat = lambda f, t: np.concatenate([np.asarray(getattr(lp, f), t) for lp in lps]) if count else np.zeros(0, t)
    return PackedBatch(desc=desc, indptr=cat("indptr", np.int32), indices=cat("indices", np.int32),
                       data=cat("data", np.float64), c=cat("c", np.float64),
                       c0=np.array([lp.c0 for lp in lps], np.float64), q=cat("q", np.float64),
                       l=cat("l", np.float64), u=cat("u", np.float64))

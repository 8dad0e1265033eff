"""ORACLE / CPU BASELINE (test infrastructure only): ctypes driver of oracle/libdvh_cpu.so, the C++ restatement of
the batched PDHG behind the same C ABI (oracle/cpu_pdhg.cpp; built by ``build()`` below / __graft_entry__.build).

``CpuPdhgSolver.solve(lps)`` has the signature of ``dervet_hip.BatchSolver.solve`` (list of WindowLP in, list of
WindowResult out), so tests can run the drop-in / ABI stack without a GPU and bench.py can time the same algorithm
on host cores.  The product never loads this library.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libdvh_cpu.so")
SRC = os.path.join(HERE, "cpu_pdhg.cpp")


VALIDATE = os.path.join(HERE, "..", "der-vet_amd", "csrc", "dvh_validate.cpp")
DEPS = [SRC, VALIDATE, os.path.join(HERE, "..", "der-vet_amd", "csrc", "dvh_validate.h"),
        os.path.join(HERE, "..", "include", "dervet_hip.h")]


def build(force=False, verbose=False):
    if not force and os.path.exists(LIB) and all(os.path.getmtime(LIB) >= os.path.getmtime(d) for d in DEPS):
        return LIB
    cmd = ["g++", "-O3", "-march=x86-64-v2", "-std=c++17", "-fopenmp", "-fPIC", "-shared", "-o", LIB + ".tmp", SRC,
           VALIDATE]
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("g++ failed building oracle/libdvh_cpu.so")
    os.replace(LIB + ".tmp", LIB)
    return LIB


class CpuPdhgSolver:
    """The C++ CPU restatement through the dervet_hip ctypes structs (threads: OpenMP threads, 0 = default)."""

    def __init__(self, threads=0, **options):
        sys.path.insert(0, os.path.join(HERE, "..", "der-vet_amd"))
        from dervet_hip import _lib
        self._L = _lib
        if threads:
            os.environ["DVH_CPU_THREADS"] = str(int(threads))
        self._lib = _lib.load(build())
        self._opts = _lib.Options()
        self._lib.dvh_default_options(ctypes.byref(self._opts))
        for k, v in options.items():
            setattr(self._opts, k, v)
        h = ctypes.c_void_p()
        if self._lib.dvh_create(1, ctypes.byref(self._opts), ctypes.byref(h)) != 0:
            raise RuntimeError("dvh_create failed (CPU restatement)")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._lib.dvh_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_options(self, **options):
        for k, v in options.items():
            setattr(self._opts, k, v)
        self._lib.dvh_set_options(self._h, ctypes.byref(self._opts))

    def timing(self):
        t = (ctypes.c_double * 3)()
        self._lib.dvh_last_timing(self._h, t)
        return {"total_ms": t[0], "setup_ms": t[1], "pdhg_ms": t[2]}

    def solve(self, lps, start=None):
        from dervet_hip.solver import WindowResult
        L = self._L
        count = len(lps)
        arr = (L.LP * count)()
        res = (L.Result * count)()
        keep, outs = [], []

        def ptr(a, t, ct):
            a = np.ascontiguousarray(a, dtype=t)
            keep.append(a)
            return a.ctypes.data_as(ct)

        for k, lp in enumerate(lps):
            m = lp.m
            a = arr[k]
            a.n, a.m_eq, a.m_ineq, a.nnz = lp.n, lp.m_eq, m - lp.m_eq, len(lp.indices)
            a.indptr, a.indices = ptr(lp.indptr, np.int32, L.c_int32_p), ptr(lp.indices, np.int32, L.c_int32_p)
            a.data, a.c = ptr(lp.data, np.float64, L.c_double_p), ptr(lp.c, np.float64, L.c_double_p)
            a.q, a.l = ptr(lp.q, np.float64, L.c_double_p), ptr(lp.l, np.float64, L.c_double_p)
            a.u, a.c0 = ptr(lp.u, np.float64, L.c_double_p), lp.c0
            x, y = np.zeros(lp.n), np.zeros(m)
            if start is not None and start[k] is not None:
                x[:], y[:] = start[k]
            outs.append((x, y))
            res[k].x = x.ctypes.data_as(L.c_double_p)
            res[k].y = y.ctypes.data_as(L.c_double_p) if m else None
        if self._lib.dvh_solve_batch(self._h, arr, count, res) != 0:
            raise RuntimeError("dvh_solve_batch failed (CPU restatement)")
        return [WindowResult(outs[k][0], outs[k][1], res[k].obj, res[k].status, res[k].iters, res[k].primal_res_rel,
                             res[k].dual_res_rel, res[k].gap_rel) for k in range(count)]

"""ORACLE (test / CPU-baseline infrastructure only): HiGHS over a process pool.

``bench.py``'s ``cpu_baseline`` leg times the restated window LP (``oracle.window_lp``) solved by HiGHS
(scipy 1.15 ``linprog(method="highs")``), one LP per process, on the host cores of the GPU box.  The
reference's own loop (CVXPY 1.0.31 -> ECOS / GLPK, dervet/MicrogridScenario.py:310-320) cannot run on
either box (storagevet, cvxpy, ecos and cvxopt are absent), so this is a "port"
baseline of the same LP, and it doubles as the parity check of the GPU results on the sample.
"""
import os
import time
from multiprocessing import get_context

import numpy as np

from . import window_lp


def cpu_model():
    """CPU model name of this host (/proc/cpuinfo), for the bench line's cpu_baseline."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _solve_one(lp):
    t = time.perf_counter()
    r = window_lp.solve_highs(lp)
    return (r.get("obj", np.nan), r["status"], time.perf_counter() - t)


def highs_batch(lps, procs=None):
    """Solve the LP dicts with HiGHS on `procs` processes. Returns (objs, statuses, wall_s, procs)."""
    procs = int(procs or min(16, os.cpu_count() or 1))
    t = time.perf_counter()
    if procs <= 1:
        res = [_solve_one(lp) for lp in lps]
    else:
        pool = get_context("fork").Pool(procs)
        try:
            res = pool.map(_solve_one, lps, chunksize=max(1, len(lps) // (4 * procs)))
            pool.close()  # workers exit on their own (no SIGTERM: a profiler's signal handler in them can hang)
        except BaseException:
            pool.terminate()
            raise
        finally:
            pool.join()
    wall = time.perf_counter() - t
    return (np.array([r[0] for r in res]), np.array([r[1] for r in res]), wall, procs)

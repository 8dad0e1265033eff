"""Iteration-count study of PDHG variants on a config-4 sample, with the host restatement (dev helper, CPU).

Usage: python scripts/iter_study.py <scenarios> <variant> [<variant> ...]
  a variant is name:key=val,key=val (keys of oracle.pdlp_ref.DEFAULTS), e.g.  base:  art36:b_art=0.36
"""
import os
import sys
import time
from multiprocessing import Pool

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "der-vet_amd"))
from dervet_hip.lp import builder, scenarios  # noqa: E402
from oracle import pdlp_ref  # noqa: E402

_LPS = []


def _init(S):
    global _LPS
    for g in scenarios.config4(range(S)):
        for lp in builder.group_window_lps(g):
            K = sp.csr_matrix((lp.data, lp.indices, lp.indptr), shape=(lp.m, lp.n))
            _LPS.append(dict(K=K, q=lp.q, c=lp.c, c0=lp.c0, l=lp.l, u=lp.u, m_eq=lp.m_eq))


def _run(arg):
    k, opts = arg
    r = pdlp_ref.solve(_LPS[k], opts)
    return r["status"], r["iters"], r["obj"]


def parse(v):
    name, _, kv = v.partition(":")
    opts = {}
    for item in filter(None, kv.split(",")):
        key, val = item.split("=")
        opts[key] = float(val) if "." in val or "e" in val else int(val)
    return name, opts


def main():
    S = int(sys.argv[1])
    variants = [parse(v) for v in sys.argv[2:]]
    nwin = 12 * S
    with Pool(8, initializer=_init, initargs=(S,)) as pool:
        base_obj = None
        for name, opts in variants:
            t = time.time()
            res = pool.map(_run, [(k, opts) for k in range(nwin)], chunksize=1)
            st = np.array([r[0] for r in res])
            it = np.array([r[1] for r in res], float)
            obj = np.array([r[2] for r in res])
            if base_obj is None:
                base_obj = obj
            dev = np.max(np.abs(obj - base_obj) / np.maximum(np.abs(base_obj), 1e-9))
            print(f"{name:14s} opt {np.mean(st == 0):.3f} iters mean {it.mean():7.1f} p50 {np.median(it):6.0f} "
                  f"p90 {np.percentile(it, 90):6.0f} max {it.max():6.0f}  obj dev {dev:.1e}  {time.time() - t:.0f}s",
                  flush=True)


if __name__ == "__main__":
    main()

"""HiGHS objectives of BASELINE config 3's annual 5-minute windows (dervet_hip.lp.scenarios.config3), committed as
tests/golden/config3_highs.json: the GPU test (tests/test_gpu_config3.py) compares against them instead of
re-running HiGHS on the box (the DCM variant takes minutes there).  The windows are built by the product builder
from the committed reference_inputs fixture (tests/test_builder.py pins that builder to the oracle restatement);
this script solves them with the oracle (restated LP + HiGHS, oracle/window_lp.py).

Usage: python tests/golden/make_config3_golden.py [variant ...]   (default: da dcm)
"""
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "der-vet_amd")]

from dervet_hip.lp import scenarios  # noqa: E402
from oracle import window_lp  # noqa: E402


def lp_of(g):
    K = sp.csr_matrix((g.data[0], g.indices, g.indptr), shape=(g.m, g.n))
    return dict(K=K, q=g.q[0], c=g.c[0], c0=float(g.c0[0]), l=g.l[0], u=g.u[0], m_eq=g.m_eq)


def main(variants):
    path = os.path.join(HERE, "config3_highs.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    for v in variants:
        g = scenarios.config3(v)[0]
        t = time.time()
        h = window_lp.solve_highs(lp_of(g))
        wall = time.time() - t
        if h["status"] != 0:
            raise SystemExit(f"{v}: HiGHS status {h['status']} {h['message']}")
        terms = {k: float(coef @ h["x"] + const) for k, (coef, const) in g.terms.items()}
        out[v] = {"obj": h["obj"], "n": g.n, "m": g.m, "nnz": int(len(g.data[0])), "terms": terms,
                  "highs_s": round(wall, 1), "scipy": __import__("scipy").__version__,
                  "ene_first": float(h["x"][2 * g.T]), "ene_min": float(np.min(h["x"][2 * g.T:3 * g.T]))}
        print(v, out[v], flush=True)
        with open(path, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:] or ["da", "dcm"])

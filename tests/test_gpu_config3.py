"""GPU: BASELINE config 3 -- the 5-minute annual window (T = 105,120 steps, Model_Parameters_Template_DER.csv:4 dt,
:8 n = year) -- on the medium tier's long team (csrc/dvh_chain.hip: 137 segments of <= 768 steps, one workgroup
each, spanning the chip; grid-wide setup, leader check reduction).

Both variants of dervet_hip.lp.scenarios.config3 -- DA time shift alone (n = 315,360), and DA + retailETS + 12
monthly demand charges on the site load less the template's fixed PV (n = 315,372, m = 210,241) -- are checked
against the HiGHS objectives committed by tests/golden/make_config3_golden.py (objective within 1e-5, primal
residual <= 1e-6 recomputed here), against the grid-wide large-LP path (the same algorithm: objectives within 2e-6),
and for bitwise reproducibility.
"""
import json
import os

import numpy as np
import pytest
import scipy.sparse as sp

from dervet_hip.lp import builder, scenarios
from oracle import window_lp

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "config3_highs.json")))


def _lp(g):
    K = sp.csr_matrix((g.data[0], g.indices, g.indptr), shape=(g.m, g.n))
    return dict(K=K, q=g.q[0], c=g.c[0], c0=float(g.c0[0]), l=g.l[0], u=g.u[0], m_eq=g.m_eq)


@pytest.fixture(scope="module", params=["da", "dcm"])
def case(request):
    g = scenarios.config3(request.param)[0]
    assert (g.n, g.m, len(g.data[0])) == (GOLD[request.param]["n"], GOLD[request.param]["m"], GOLD[request.param]["nnz"])
    return request.param, g


def test_config3_long_team_matches_highs(gpu_solver, case):
    name, g = case
    lps = builder.group_window_lps(g)
    r = gpu_solver.solve(lps)[0]
    ks = gpu_solver.kernel_stats()
    assert ks["chain_windows"] == 1 and ks["large_windows"] == 0, ks
    h = GOLD[name]["obj"]
    assert r.status == 0, r.status_name
    rel = abs(r.obj - h) / abs(h)
    pres = window_lp.primal_residual_rel(_lp(g), r.x)[0]
    assert rel <= 1e-5 and pres <= 1e-6, (rel, pres)
    t = gpu_solver.timing()
    print(f"config3 {name}: {r.iters} iterations, obj rel err {rel:.2e}, primal res {pres:.2e}, "
          f"solve {t['total_ms']:.1f} ms (setup {t['setup_ms']:.1f}, PDHG {t['pdhg_ms']:.1f})")


def test_config3_long_team_agrees_with_grid_wide_path_and_reproduces(gpu_solver, case):
    name, g = case
    lps = builder.group_window_lps(g)
    a = gpu_solver.solve(lps)[0]
    b = gpu_solver.solve(lps)[0]
    assert np.array_equal(a.x, b.x) and a.iters == b.iters
    gpu_solver.set_kernel_path("ell")  # band kernels (and the medium tier) off: the grid-wide large-LP path
    try:
        c = gpu_solver.solve(lps)[0]
        assert gpu_solver.kernel_stats()["large_windows"] == 1
    finally:
        gpu_solver.set_kernel_path("default")
    assert c.status == 0 and abs(a.obj - c.obj) <= 2e-6 * abs(c.obj), (a.obj, c.obj)

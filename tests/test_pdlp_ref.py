"""The host restatement of the GPU algorithm (oracle/pdlp_ref.py) solves golden and synthetic windows to
the north-star bars (objective within 1e-5 of HiGHS, primal residual <= 1e-6).  The GPU kernels are then
checked against this restatement iterate-for-iterate in tests/test_gpu_parity.py."""
import numpy as np
import pytest
import scipy.sparse as sp

from dervet_hip.lp import scenarios
from oracle import cases, pdlp_ref, window_lp


@pytest.mark.parametrize("name,idx", [("es", 0), ("es", 6), ("es+pv+dg", 3)])
def test_reference_pdhg_on_golden_windows(name, idx):
    wins, arr, meta, _ = cases.case_windows(name)
    lp = window_lp.build(wins[idx])
    h = window_lp.solve_highs(lp)
    r = pdlp_ref.solve(lp)
    assert r["status"] == pdlp_ref.OPTIMAL
    assert abs(r["obj"] - h["obj"]) <= 1e-5 * abs(h["obj"])
    assert abs(r["obj"] - arr["golden_objective"][idx].sum()) <= 1e-5 * abs(h["obj"])
    pres, _ = window_lp.primal_residual_rel(lp, r["x"])
    assert pres <= 1e-6
    assert r["iters"] % 16 == 0 and r["iters"] < 20000


def test_reference_pdhg_on_sweep_windows():
    g = scenarios.config4([11])
    for gg in (g[0], g[6]):
        K = sp.csr_matrix((gg.data[0], gg.indices, gg.indptr), shape=(gg.m, gg.n))
        lp = dict(K=K, q=gg.q[0], c=gg.c[0], c0=gg.c0[0], l=gg.l[0], u=gg.u[0], m_eq=gg.m_eq)
        h = window_lp.solve_highs(lp)
        r = pdlp_ref.solve(lp)
        assert r["status"] == 0 and abs(r["obj"] - h["obj"]) <= 1e-5 * abs(h["obj"])


def test_iteration_limit_reports_last_checked_candidate():
    wins, _, _, _ = cases.case_windows("es")
    lp = window_lp.build(wins[0])
    r = pdlp_ref.solve(lp, {"max_iters": 256})
    assert r["status"] == pdlp_ref.ITER_LIMIT and r["iters"] == 256
    assert np.isfinite(r["obj"]) and r["kkt"]["pres_rel"] > 1e-6

"""GPU parity of the medium tier (dvh_chain.hip): battery windows longer than one workgroup solved as a batch, a
team of one 768-thread workgroup per segment of <= 768 steps.  Windows from the config-4 generator with the
reference's window options (Model_Parameters_Template_DER.csv `n` = "year": T = 8,760; `dt` = 0.25: monthly
T = 2,688..2,976), checked against HiGHS on the same LP (objective within 1e-5, primal residual <= 1e-6), against
the grid-wide large-LP path (the same algorithm), and for bitwise reproducibility."""
import dataclasses

import numpy as np
import pytest
import scipy.sparse as sp

from dervet_hip import BatchSolver
from dervet_hip.lp import builder, scenarios
from oracle import window_lp

pytestmark = pytest.mark.gpu


def _lps(groups):
    return [lp for g in groups for lp in builder.group_window_lps(g)]


def _highs_check(lp, r):
    o = dict(K=sp.csr_matrix((lp.data, lp.indices, lp.indptr), shape=(lp.m, lp.n)), q=lp.q, c=lp.c, c0=lp.c0, l=lp.l,
             u=lp.u, m_eq=lp.m_eq)
    h = window_lp.solve_highs(o)
    assert h["status"] == 0 and r.status == 0, r.status_name
    assert abs(r.obj - h["obj"]) <= 1e-5 * abs(h["obj"]), (r.obj, h["obj"])
    assert window_lp.primal_residual_rel(o, r.x)[0] <= 1e-6


def test_annual_hourly_windows_on_the_medium_tier(gpu_solver):
    lps = _lps(scenarios.config4([0, 1, 2], n="year"))
    assert all(lp.n == 26292 for lp in lps)
    res = gpu_solver.solve(lps)
    ks = gpu_solver.kernel_stats()
    assert ks["chain_windows"] == 3 and ks["large_windows"] == 0, ks
    for lp, r in zip(lps, res):
        _highs_check(lp, r)


def test_quarter_hour_monthly_windows_share_the_demand_column(gpu_solver):
    """dt = 0.25: one demand column spans the window's four segments (its update is redundant in each)."""
    lps = _lps(scenarios.config4([5], dt=0.25))
    res = gpu_solver.solve(lps)
    ks = gpu_solver.kernel_stats()
    assert ks["chain_windows"] == 12, ks
    assert all(r.status == 0 for r in res)
    for k in (0, 7):
        _highs_check(lps[k], res[k])


def test_medium_tier_agrees_with_the_grid_wide_path():
    lps = _lps(scenarios.config4([3], n="year")) + _lps(scenarios.config4([4], dt=0.25))[:2]
    with BatchSolver(0) as s:
        chain = s.solve(lps)
        assert s.kernel_stats()["chain_windows"] == 3
        s.set_kernel_path("ell")  # the medium tier runs only on the default path
        big = s.solve(lps)
        assert s.kernel_stats()["large_windows"] == 3
    for a, b in zip(chain, big):
        assert a.status == b.status == 0
        assert abs(a.obj - b.obj) <= 2e-6 * abs(b.obj), (a.obj, b.obj)


def test_mixed_batch_routes_each_window_and_is_reproducible(gpu_solver):
    """Monthly windows (band kernel) and annual windows (medium tier) interleaved in one batch; two solves give
    bitwise-equal results."""
    monthly = _lps(scenarios.config4([6]))
    annual = _lps(scenarios.config4([6, 7], n="year"))
    lps = monthly[:3] + annual[:1] + monthly[3:5] + annual[1:]
    a = gpu_solver.solve(lps)
    ks = gpu_solver.kernel_stats()
    assert ks["band_windows"] == 5 and ks["chain_windows"] == 2, ks
    b = gpu_solver.solve(lps)
    for ra, rb in zip(a, b):
        assert ra.status == 0
        assert np.array_equal(ra.x, rb.x) and np.array_equal(ra.y, rb.y) and ra.iters == rb.iters
    for lp, r in zip(lps[3:4], a[3:4]):
        _highs_check(lp, r)


def test_crossed_bounds_medium_window_is_reported_infeasible(gpu_solver):
    lps = _lps(scenarios.config4([8, 9], n="year"))
    T = lps[1].m_eq - 1
    bad_l = lps[1].l.copy()
    bad_l[2 * T + 100] = lps[1].u[2 * T + 100] + 1.0
    bad = [lps[0], dataclasses.replace(lps[1], l=bad_l)]
    res = gpu_solver.solve(bad)
    assert res[1].status_name == "infeasible" and res[1].iters == 0
    assert res[0].status == 0
    assert gpu_solver.kernel_stats()["chain_windows"] == 1


def test_team_launch_abort_hands_windows_to_the_grid_wide_path(monkeypatch):
    """A team whose exchange outlasts the spin limit (forced here: the test limit aborts at the first wait) aborts: the
    windows it had not finished are solved on the grid-wide path, every window still comes back OPTIMAL and within
    1e-5 of HiGHS, the solve returns OK, the abort count is reported (dvh_last_chain_aborts) and the diagnostics go to
    dvh_last_warning, not dvh_last_error; the next solve resets both."""
    lps = _lps(scenarios.config4([11], dt=0.25))[:2]
    monkeypatch.setenv("DVH_CHAIN_SPIN_TICKS", "-1")  # abort at the first exchange that has to wait
    with BatchSolver(0) as s:
        res = s.solve(lps)
        ks = s.kernel_stats()
        assert ks["chain_aborts"] >= 1, ks
        assert ks["chain_windows"] + ks["large_windows"] == 2, ks
        assert "timed out" in s.last_warning()
        for lp, r in zip(lps, res):
            _highs_check(lp, r)
        s.solve(lps[:0] + [lp for lp in _lps(scenarios.config4([11]))[:1]])  # a band-only solve resets them
        assert s.kernel_stats()["chain_aborts"] == 0 and s.last_warning() == ""

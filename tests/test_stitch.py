"""Coarse-to-fine start for a long window (dervet_hip/stitch.py).

CPU: the start stitched from the sub-windows' optimal solutions (HiGHS) is feasible for the long window and
its objective is an upper bound close to the long window's optimum (DA-only and retail + DCM variants, hourly
annual window from monthly / weekly sub-windows).
GPU: the config-3 annual 5-minute window started from its 365 daily windows reaches the same objective as the
cold solve and HiGHS in fewer iterations.
"""
import numpy as np
import pytest

from dervet_hip.lp import scenarios
from dervet_hip.stitch import stitched_start
from oracle import window_lp


def _lp(g):
    import scipy.sparse as sp
    return dict(K=sp.csr_matrix((g.data[0], g.indices, g.indptr), shape=(g.m, g.n)), q=g.q[0], c=g.c[0],
                c0=g.c0[0], l=g.l[0], u=g.u[0], m_eq=g.m_eq)


def _groups(n, with_retail, T=8760):
    ri = scenarios.reference_inputs()
    da = ri["hourly_da_price"][None, :T]
    load = ri["hourly_site_load"][None, :T] if with_retail else np.zeros((1, T))
    return scenarios.windows_by_period(2017, 1.0, load, None, scenarios.template_battery(), da_price=da,
                                       tariff_def=scenarios.tariff() if with_retail else None, n=n)


@pytest.mark.parametrize("with_retail,sub", [(False, "month"), (True, "month"), (True, 168)])
def test_stitched_start_is_feasible_and_near_optimal(with_retail, sub):
    long = _groups("year", with_retail)[0]
    subs = _groups(sub, with_retail)
    sol = [window_lp.solve_highs(_lp(g)) for g in subs]
    assert all(s["status"] == 0 for s in sol)
    # HiGHS returns no duals here: the primal part is what is checked
    x0, y0 = stitched_start(long, subs, [s["x"] for s in sol], [np.zeros(g.m) for g in subs])
    lp = _lp(long)
    pres, linf = window_lp.primal_residual_rel(lp, x0)
    assert pres <= 1e-9 and linf <= 1e-5, (pres, linf)
    assert np.all(x0 >= lp["l"] - 1e-9) and np.all(x0 <= lp["u"] + 1e-9)
    h = window_lp.solve_highs(lp)
    obj0 = lp["c"] @ x0 + lp["c0"]
    assert obj0 >= h["obj"] - 1e-6 * abs(h["obj"])
    assert obj0 - h["obj"] <= 0.1 * abs(h["obj"])  # the dropped sub-window targets cost little
    assert y0.shape == (long.m,)


def test_stitched_duals_map_rows():
    long = _groups("year", False, T=96)[0]
    subs = _groups(24, False, T=96)
    ys = [np.arange(g.m, dtype=float) + 100 * s for s, g in enumerate(subs)]
    xs = [np.zeros(g.n) for g in subs]
    _, y0 = stitched_start(long, subs, xs, ys)
    assert y0[0] == 0.0 and y0[1] == 1.0 and y0[24] == 24.0      # day 0: init, recurrences, end row
    assert y0[25] == 101.0 and y0[48] == 124.0 and y0[96] == 324.0  # day 1 rows, last day's end row
    with pytest.raises(ValueError):
        stitched_start(long, subs[:-1], xs[:-1], ys[:-1])


@pytest.mark.gpu
def test_config3_stitched_from_daily_windows_on_gpu(gpu_solver):
    from dervet_hip.lp import builder
    from dervet_hip.stitch import solve_stitched
    ri = scenarios.reference_inputs()
    T = len(ri["fivemin_da_price"])
    mk = lambda n: scenarios.windows_by_period(2019, 1.0 / 12, np.zeros((1, T)), None,  # noqa: E731
                                               scenarios.template_battery(),
                                               da_price=ri["fivemin_da_price"][None, :], n=n)
    long = mk("year")[0]
    subs = mk(288)
    s = gpu_solver
    cold = s.solve(builder.group_window_lps(long))[0]
    res, sres, tm = solve_stitched(s, long, subs)
    assert s.options().warm_start == 0
    assert all(r.status == 0 for r in sres) and res.status == 0 and cold.status == 0
    assert res.iters < cold.iters
    assert abs(res.obj - cold.obj) <= 1e-5 * abs(cold.obj)
    h = window_lp.solve_highs(_lp(long))
    assert abs(res.obj - h["obj"]) <= 1e-5 * abs(h["obj"])
    assert window_lp.primal_residual_rel(_lp(long), res.x)[0] <= 1e-6
    print(f"config 3: cold {cold.iters} iterations, stitched {res.iters} (+365 daily windows in "
          f"{tm['subs_ms']:.1f} ms), long-window solve {tm['long_ms']:.1f} ms")


def test_monthly_sub_windows_carry_their_demand_charge_duals_over():
    """dcm_duals=True: the long window's DCM epigraph row of step t takes the dual of the monthly sub-window's row of the
    same step (the sub-windows are the long window's own demand-charge periods); without it those rows start at 0."""
    long = _groups("year", True)[0]
    subs = _groups("month", True)
    sub_y = [np.arange(g.m, dtype=np.float64) + 1e6 * (s + 1) for s, g in enumerate(subs)]
    sub_x = [np.zeros(g.n) for g in subs]
    _, y0 = stitched_start(long, subs, sub_x, sub_y, dcm_duals=True)
    _, y_off = stitched_start(long, subs, sub_x, sub_y)
    from dervet_hip.stitch import _dcm_rows
    rows = _dcm_rows(long)
    assert len(rows) == long.m - long.m_eq  # every >= row of the retail + DCM window is a DCM row
    a, want = 0, {}
    for s, g in enumerate(subs):
        for t, k, r in _dcm_rows(g):
            want[(a + t, k)] = sub_y[s][r]
        a += g.T
    for t, k, r in rows:
        assert y0[r] == want[(t, k)] and y_off[r] == 0.0
    np.testing.assert_array_equal(y0[:long.m_eq], y_off[:long.m_eq])


def test_dcm_duals_only_where_both_windows_count_the_same_charges():
    """the (step, rank) key identifies a charge only where both windows cover the step with the same number
    of charges.  A monthly sub-window without its demand charge (no DCM rows) leaves its month's long-window rows at 0;
    the other months still carry their duals over."""
    long = _groups("year", True)[0]
    subs = _groups("month", True)
    subs[0] = _groups("month", False)[0]  # January without the demand charge
    sub_y = [np.arange(g.m, dtype=np.float64) + 1e6 * (s + 1) for s, g in enumerate(subs)]
    sub_x = [np.zeros(g.n) for g in subs]
    _, y0 = stitched_start(long, subs, sub_x, sub_y, dcm_duals=True)
    from dervet_hip.stitch import _dcm_rows
    jan = subs[0].T
    rows = _dcm_rows(long)
    assert any(t < jan for t, _, _ in rows) and any(t >= jan for t, _, _ in rows)
    for t, k, r in rows:
        assert (y0[r] == 0.0) == (t < jan)

"""GPU: the band kernels scale the windows they take themselves (csrc/dvh_band.hip, round 3) instead of reading
setup_kernel's outputs; the ELL path (dvh_set_kernel_path("ell")) still scales through setup_kernel.  Both are
setup_kernel's preconditioner (Ruiz inf-norm passes + one Pock-Chambolle pass), so the two paths solve the same
windows to the same optimum -- also on a badly scaled copy (costs x 1e4, the SOE rows in Wh) -- and agree with HiGHS.
A band window with crossed bounds is reported PRIMAL_INFEASIBLE with no iterations, as setup_kernel reports it."""
import dataclasses

import numpy as np
import pytest
import scipy.sparse as sp

from dervet_hip.lp import builder, scenarios
from oracle import window_lp

pytestmark = pytest.mark.gpu


def _badly_scaled(lp):
    T = lp.m_eq - 1
    data, q = lp.data.copy(), lp.q.copy()
    rows = np.repeat(np.arange(lp.m), np.diff(lp.indptr))
    soe = (rows >= 1) & (rows <= T)  # the SOE recurrence rows, in Wh
    data[soe] *= 1e3
    q[1:T + 1] *= 1e3
    return dataclasses.replace(lp, data=data, q=q, c=lp.c * 1e4, c0=lp.c0 * 1e4)


def _highs(lp):
    o = dict(K=sp.csr_matrix((lp.data, lp.indices, lp.indptr), shape=(lp.m, lp.n)), q=lp.q, c=lp.c, c0=lp.c0,
             l=lp.l, u=lp.u, m_eq=lp.m_eq)
    return o, window_lp.solve_highs(o)


def test_band_kernel_scaling_matches_the_setup_kernel_path_and_highs(gpu_solver):
    base = [lp for g in scenarios.config4(range(3)) for lp in builder.group_window_lps(g)]
    lps = base + [_badly_scaled(lp) for lp in base[::3]]
    band = gpu_solver.solve(lps)
    assert gpu_solver.kernel_stats()["band_windows"] == len(lps)
    try:
        gpu_solver.set_kernel_path("ell")
        ell = gpu_solver.solve(lps)
        assert gpu_solver.kernel_stats()["band_windows"] == 0
    finally:
        gpu_solver.set_kernel_path("default")
    for i, (lp, a, b) in enumerate(zip(lps, band, ell)):
        assert a.status == 0 and b.status == 0, (i, a.status_name, b.status_name)
        assert abs(a.obj - b.obj) <= 2e-6 * abs(b.obj), (i, a.obj, b.obj)
    for i in (0, 5, 11, len(base), len(lps) - 1):
        o, h = _highs(lps[i])
        assert h["status"] == 0
        assert abs(band[i].obj - h["obj"]) <= 1e-5 * abs(h["obj"]), (i, band[i].obj, h["obj"])
        assert window_lp.primal_residual_rel(o, band[i].x)[0] <= 1e-6


def test_band_kernel_reports_crossed_bounds_without_iterating(gpu_solver):
    lps = [lp for g in scenarios.config4(range(2)) for lp in builder.group_window_lps(g)]
    k = 5
    T = lps[k].m_eq - 1
    l = lps[k].l.copy()
    l[2 * T + 7] = lps[k].u[2 * T + 7] + 1.0  # ene_7 above the energy rating
    lps[k] = dataclasses.replace(lps[k], l=l)
    res = gpu_solver.solve(lps)
    assert res[k].status_name == "infeasible" and res[k].iters == 0, (res[k].status_name, res[k].iters)
    assert all(r.status == 0 for i, r in enumerate(res) if i != k)
    # reported by the band pass itself: no window was handed on to setup_kernel / the ELL or generic kernels
    ks = gpu_solver.kernel_stats()
    assert ks["band_windows"] == len(lps) and ks["ell_windows"] == 0 and ks["generic_windows"] == 0, ks


def test_factors_outside_single_precision_range_leave_the_band_kernel(gpu_solver):
    """A row scaled by 1e-70 (right-hand side with it: the same LP) needs a row factor near 1e70, which the band
    kernel's single-precision check copies cannot hold: the band kernel hands the window on (the ELL / generic path
    keeps its factors in double) and it is still solved to the unscaled window's HiGHS objective."""
    lps = [lp for g in scenarios.config4([2]) for lp in builder.group_window_lps(g)][:3]
    lp = lps[1]
    i = lp.m_eq  # the first DCM (>=) row
    data, q = lp.data.copy(), lp.q.copy()
    data[lp.indptr[i]:lp.indptr[i + 1]] *= 1e-70
    q[i] *= 1e-70
    lps[1] = dataclasses.replace(lp, data=data, q=q)
    res = gpu_solver.solve(lps)
    ks = gpu_solver.kernel_stats()
    assert ks["band_windows"] == 2 and ks["ell_windows"] + ks["generic_windows"] == 1, ks
    o, h = _highs(lp)
    assert res[1].status == 0 and abs(res[1].obj - h["obj"]) <= 1e-5 * abs(h["obj"]), (res[1].obj, h["obj"])


def test_box_form_matches_the_plain_form(gpu_solver, monkeypatch):
    """The battery forms iterate on [0, 1]-normalised column boxes (csrc/dvh_band.hip BOX: the projection is the FMA's
    clamp).  The change of variables is exact, so the box form reaches the plain form's optimum on the same windows --
    the bench shape and the badly scaled copies -- in about as many iterations."""
    base = [lp for g in scenarios.config4(range(3)) for lp in builder.group_window_lps(g)]
    lps = base + [_badly_scaled(lp) for lp in base[::3]]
    box = gpu_solver.solve(lps)
    assert gpu_solver.kernel_stats()["band_windows"] == len(lps)
    monkeypatch.setenv("DVH_BAND_BOX", "0")
    plain = gpu_solver.solve(lps)
    monkeypatch.delenv("DVH_BAND_BOX")
    it_box = it_plain = 0
    for i, (lp, a, b) in enumerate(zip(lps, box, plain)):
        assert a.status == 0 and b.status == 0, (i, a.status_name, b.status_name)
        assert abs(a.obj - b.obj) <= 2e-6 * abs(b.obj), (i, a.obj, b.obj)
        assert np.all(a.x >= lp.l - 1e-9 * (1 + np.abs(lp.l))) and np.all(a.x <= lp.u + 1e-9 * (1 + np.abs(lp.u)))
        it_box += a.iters
        it_plain += b.iters
    assert it_box <= 1.1 * it_plain, (it_box, it_plain)
    for i in (0, 5, len(base)):
        o, h = _highs(lps[i])
        assert abs(box[i].obj - h["obj"]) <= 1e-5 * abs(h["obj"]), (i, box[i].obj, h["obj"])
        assert window_lp.primal_residual_rel(o, box[i].x)[0] <= 1e-6


def test_unbounded_column_goes_to_the_plain_form(gpu_solver):
    """A window whose charge column has no upper bound has no box: the box form returns it (status -3) and the plain
    band form solves it in the same cascade pass (still counted as a band window) to HiGHS's optimum; a fixed column
    (lo == hi) stays in the box form with width 0."""
    lps = [lp for g in scenarios.config4([1]) for lp in builder.group_window_lps(g)][:4]
    u = lps[1].u.copy()
    u[3] = np.inf  # ch_3 unbounded
    lps[1] = dataclasses.replace(lps[1], u=u)
    T2 = lps[2].m_eq - 1
    l2, u2 = lps[2].l.copy(), lps[2].u.copy()
    l2[2 * T2 + 5] = u2[2 * T2 + 5] = 0.5 * (l2[2 * T2 + 5] + u2[2 * T2 + 5])  # ene_5 fixed mid-box
    lps[2] = dataclasses.replace(lps[2], l=l2, u=u2)
    res = gpu_solver.solve(lps)
    ks = gpu_solver.kernel_stats()
    assert ks["band_windows"] == len(lps) and ks["ell_windows"] == 0 and ks["generic_windows"] == 0, ks
    for i in (1, 2):
        o, h = _highs(lps[i])
        assert h["status"] == 0 and res[i].status == 0, (i, res[i].status_name)
        assert abs(res[i].obj - h["obj"]) <= 1e-5 * abs(h["obj"]), (i, res[i].obj, h["obj"])
    assert abs(res[2].x[2 * T2 + 5] - l2[2 * T2 + 5]) <= 1e-9 * abs(l2[2 * T2 + 5]), res[2].x[2 * T2 + 5]


def test_unbounded_column_with_out_of_range_factors_reaches_the_double_path(gpu_solver):
    """a window with no box (unbounded ch column: the box form returns it, status -3) whose
    factors also leave float's range (a DCM row scaled by 1e-70) is refused by the plain form's factor check (-2)
    AFTER the first -2 list was formed; the cascade lists the -2s again once the plain form has run, so the window
    still reaches the ELL / generic path and is solved to HiGHS's optimum, not returned with its internal status."""
    lps = [lp for g in scenarios.config4([2]) for lp in builder.group_window_lps(g)][:3]
    lp = lps[1]
    i = lp.m_eq
    data, q, u = lp.data.copy(), lp.q.copy(), lp.u.copy()
    data[lp.indptr[i]:lp.indptr[i + 1]] *= 1e-70
    q[i] *= 1e-70
    u[3] = np.inf
    lps[1] = dataclasses.replace(lp, data=data, q=q, u=u)
    res = gpu_solver.solve(lps)
    ks = gpu_solver.kernel_stats()
    assert ks["band_windows"] == 2 and ks["ell_windows"] + ks["generic_windows"] == 1, ks
    o, h = _highs(lps[1])
    assert h["status"] == 0 and res[1].status == 0, res[1].status_name
    assert abs(res[1].obj - h["obj"]) <= 1e-5 * abs(h["obj"]), (res[1].obj, h["obj"])


@pytest.mark.parametrize("box", ["1", "2"])
def test_ice_window_without_a_box_goes_to_the_plain_ice_form(gpu_solver, monkeypatch, box):
    """The ICE form's box (opt-in, DVH_BAND_BOX=2) covers elec / on too: an ICE window whose elec_t has no upper bound
    is returned by the box form and solved by the plain ICE form in the same pass, to HiGHS's optimum (and by the
    plain ICE form directly by default)."""
    monkeypatch.setenv("DVH_BAND_BOX", box)
    lps = [lp for g in scenarios.config5([4], years=1) for lp in builder.group_window_lps(g)][:3]
    lp = lps[1]
    T = lp.m_eq - 1
    J = lp.n - 5 * T
    u = lp.u.copy()
    u[3 * T + J + 10] = np.inf  # elec_10
    lps[1] = dataclasses.replace(lp, u=u)
    res = gpu_solver.solve(lps)
    ks = gpu_solver.kernel_stats()
    assert ks["band_windows"] == len(lps) and ks["ell_windows"] == 0 and ks["generic_windows"] == 0, ks
    for i in (0, 1):
        o, h = _highs(lps[i])
        assert h["status"] == 0 and res[i].status == 0, (i, res[i].status_name)
        assert abs(res[i].obj - h["obj"]) <= 1e-5 * abs(h["obj"]), (i, res[i].obj, h["obj"])


def test_launch_order_changes_scheduling_only(gpu_solver):
    """dvh_set_launch_order: the band pass launches its windows in the given order (the seeded sweep's warm phase
    runs longest-expected-first); every window's result is bit-identical to the packing-order solve, the order is
    consumed by one solve, and a non-permutation is refused."""
    from dervet_hip.solver import SolverError
    lps = [lp for g in scenarios.config4(range(2)) for lp in builder.group_window_lps(g)]
    a = gpu_solver.solve(lps)
    gpu_solver.set_launch_order(np.arange(len(lps))[::-1])
    b = gpu_solver.solve(lps)
    for ra, rb in zip(a, b):
        assert ra.status == rb.status == 0 and ra.iters == rb.iters and ra.obj == rb.obj
        assert np.array_equal(ra.x, rb.x) and np.array_equal(ra.y, rb.y)
    for bad in ([0, 0, 1], [1, 2, 3], [-1]):
        with pytest.raises(SolverError, match="permutation"):
            gpu_solver.set_launch_order(np.array(bad))
    gpu_solver.set_launch_order(np.arange(len(lps) + 1))  # a different count: ignored by the next solve
    c = gpu_solver.solve(lps)
    assert all(ra.obj == rc.obj for ra, rc in zip(a, c))


@pytest.mark.parametrize("form", ["battery", "ice"])
def test_persistent_form_matches_one_workgroup_per_window(gpu_solver, monkeypatch, form):
    """The persistent band forms (csrc/dvh_band_persist.hip: the grid is the resident slots, each workgroup takes the
    next window from a counter; built without machine LICM) change scheduling only: with more windows than slots, so
    that workgroups run several windows one after another, every window's result is bit-identical to the
    one-workgroup-per-window launch (DVH_BAND_QUEUE=0)."""
    if form == "battery":
        lps = [lp for g in scenarios.config4(range(48)) for lp in builder.group_window_lps(g)]  # 576 > 512 slots
    else:
        lps = [lp for g in scenarios.config5(range(24), years=1) for lp in builder.group_window_lps(g)]  # 288 > 256
    a = gpu_solver.solve(lps)
    assert gpu_solver.kernel_stats()["band_windows"] == len(lps)
    monkeypatch.setenv("DVH_BAND_QUEUE", "0")
    b = gpu_solver.solve(lps)
    monkeypatch.delenv("DVH_BAND_QUEUE")
    assert gpu_solver.kernel_stats()["band_windows"] == len(lps)
    for i, (ra, rb) in enumerate(zip(a, b)):
        assert ra.status == rb.status == 0 and ra.iters == rb.iters and ra.obj == rb.obj, (i, ra.iters, rb.iters)
        assert np.array_equal(ra.x, rb.x) and np.array_equal(ra.y, rb.y), i

"""GPU parity on market-service windows: daily DA + frequency-regulation windows of
the reference's Usecase 3 golden cases (es, es+pv, es+pv+dg; binary = 1 there, solved here as the opt-in LP
relaxation), built by the product builder and solved on cuda:0 through the C ABI.

Bars: objective within 1e-5 relative of HiGHS on the same relaxed LP (oracle/window_lp.py), primal residual
<= 1e-6 recomputed from the returned x, and the relaxed optimum never above the golden MILP objective of the day
(the relaxation is a lower bound: tests/test_market_oracle.py pins the restated MILP to every golden day).
"""
import numpy as np
import pytest
import torch

from dervet_hip import BatchSolver
from dervet_hip.lp import builder, scenarios
from oracle import cases, window_lp

pytestmark = pytest.mark.gpu

OBJ_TOL = 1e-5
PRES_TOL = 1e-6


def _signals(name):
    arr, meta = cases.load_market()
    return {k.split("__", 1)[1]: v for k, v in arr.items() if k.startswith(name + "__")}, meta[name]


@pytest.mark.parametrize("name", ["es", "es+pv", "es+pv+dg"])
def test_market_days_match_highs_and_bound_golden(gpu_solver, name):
    sig, meta = _signals(name)
    days = list(range(0, 365, 5))
    g = scenarios.market_days(sig, meta["params"], days=days)
    lps = builder.group_window_lps(g)
    res = gpu_solver.solve(lps)
    # 73 days (at most two per CU): the latency regime of the cascade, also taken by the four-wave small ELL variant
    # (tests/test_gpu_cascade.py pins the routing; test_small_window_kernel_agrees_with_generic compares it with the
    # generic kernel on these windows)
    assert gpu_solver.kernel_stats()["ell_windows"] == len(lps)
    wins, keys = cases.market_windows(name)
    worst = 0.0
    for k, (d, r) in enumerate(zip(days, res)):
        o = window_lp.build(wins[d])
        h = window_lp.solve_highs(o)
        assert h["status"] == 0 and r.status == 0, (name, d, r.status_name, r.iters)
        pres, _ = window_lp.primal_residual_rel(o, r.x)
        assert pres <= PRES_TOL, (name, d, pres)
        rel = abs(r.obj - h["obj"]) / max(abs(h["obj"]), 1.0)
        worst = max(worst, rel)
        assert rel <= OBJ_TOL, (name, d, r.obj, h["obj"])
        gold = wins[d]["golden_objective"].sum()
        assert r.obj <= gold + OBJ_TOL * max(abs(gold), 1.0), (name, d, r.obj, gold)
        # the per-key values of the GPU dispatch (the objective_values row the drop-in writes) sum to the objective
        terms = sum(coef[k] @ r.x + const[k] for coef, const in g.terms.values())
        assert abs(terms - r.obj) <= 1e-9 * max(abs(r.obj), 1.0)
    print(f"{name}: {len(days)} days, worst objective rel err {worst:.2e}")


def test_market_options_keep_the_golden_bars_and_cut_the_slowest_day():
    """scenarios.MARKET_OPTIONS (primal-weight smoothing theta = 0.5) on all 1,095 golden days through the default
    cascade (the small ELL kernels): every day optimal within 1e-5 of the theta = 1 solve (which the test above pins
    to HiGHS on its days), and the slowest day needs fewer iterations -- what a latency-bound batch of days waits for."""
    lps = []
    for name in ("es", "es+pv", "es+pv+dg"):
        sig, meta = _signals(name)
        lps += builder.group_window_lps(scenarios.market_days(sig, meta["params"]))
    with BatchSolver(0) as s:
        base = s.solve(lps)
        s.set_options(**scenarios.MARKET_OPTIONS)
        mk = s.solve(lps)
    assert all(r.status == 0 for r in base) and all(r.status == 0 for r in mk)
    for a, b in zip(base, mk):
        assert abs(a.obj - b.obj) <= OBJ_TOL * max(abs(a.obj), 1.0), (a.obj, b.obj)
    it0, it1 = max(r.iters for r in base), max(r.iters for r in mk)
    assert it1 < 0.85 * it0, (it0, it1)


def test_market_days_without_relaxation_row(gpu_solver):
    """relax=False: the same daily windows without the relaxation row (the binary = 0 form of the market LP)."""
    sig, meta = _signals("es")
    days = [3, 150, 300]
    g = scenarios.market_days(sig, meta["params"], relax=False, days=days)
    res = gpu_solver.solve(builder.group_window_lps(g))
    wins, _ = cases.market_windows("es", relax=False)
    for d, r in zip(days, res):
        h = window_lp.solve_highs(window_lp.build(wins[d]))
        assert r.status == 0 and abs(r.obj - h["obj"]) <= OBJ_TOL * max(abs(h["obj"]), 1.0), (d, r.obj, h["obj"])


def test_small_window_kernel_agrees_with_generic():
    """Small-window ELL kernel vs the generic CSR kernel on the same market days: same algorithm,
    objectives within 1e-7, iteration counts within two check periods."""
    sig, meta = _signals("es+pv+dg")
    g = scenarios.market_days(sig, meta["params"], days=list(range(0, 365, 30)))
    lps = builder.group_window_lps(g)
    out = {}
    with BatchSolver(0) as s:
        for path, key in (("ell", "ell_windows"), ("generic", "generic_windows")):
            s.set_kernel_path(path)
            out[path] = s.solve(lps)
            assert s.kernel_stats()[key] == len(lps), (path, s.kernel_stats())
    for ra, rc in zip(out["ell"], out["generic"]):
        assert ra.status == rc.status == 0
        assert abs(ra.obj - rc.obj) <= 1e-7 * max(abs(rc.obj), 1.0)
        assert abs(ra.iters - rc.iters) <= 64


def test_reserve_windows_match_highs(gpu_solver):
    """Market days with spinning / non-spinning reserves (parity unpinned: tests/test_market_reserves.py) on the
    GPU: objective within 1e-5 of HiGHS on the same LP, primal residual <= 1e-6, per-key terms sum to it."""
    from test_market_reserves import reserve_series, sp_csr
    sig, meta = _signals("es+pv+dg")
    pdis = float(meta["params"]["Battery"]["dis_max_rated"])
    days = list(range(0, 365, 15))
    g = scenarios.market_days(sig, meta["params"], days=days, reserves=reserve_series(sig, pdis))
    res = gpu_solver.solve(builder.group_window_lps(g))
    # latency regime: K^T rows of 5-6 entries, the two-columns-per-lane small variant
    assert gpu_solver.kernel_stats()["ell_windows"] == len(days), gpu_solver.kernel_stats()
    for k, (d, r) in enumerate(zip(days, res)):
        o = dict(K=sp_csr(g, k), q=g.q[k], c=g.c[k], c0=float(g.c0[k]), l=g.l[k], u=g.u[k], m_eq=g.m_eq)
        h = window_lp.solve_highs(o)
        assert h["status"] == 0 and r.status == 0, (d, r.status_name, r.iters)
        pres, _ = window_lp.primal_residual_rel(o, r.x)
        assert pres <= PRES_TOL, (d, pres)
        assert abs(r.obj - h["obj"]) <= OBJ_TOL * max(abs(h["obj"]), 1.0), (d, r.obj, h["obj"])
        terms = sum(coef[k] @ r.x + const[k] for coef, const in g.terms.values())
        assert abs(terms - r.obj) <= 1e-9 * max(abs(r.obj), 1.0)


@pytest.mark.parametrize("combined", [False, True])
def test_load_following_windows_match_highs(gpu_solver, combined):
    """Market days with FR + load following + SR / NSR (parity unpinned: tests/test_market_reserves.py) on the
    GPU: objective within 1e-5 of HiGHS on the same LP and primal residual <= 1e-6."""
    from test_market_reserves import _lf, reserve_series, sp_csr
    sig, meta = _signals("es")
    pdis = float(meta["params"]["Battery"]["dis_max_rated"])
    days = list(range(3, 365, 20))
    g = scenarios.market_days(sig, meta["params"], days=days, reserves=reserve_series(sig, pdis),
                              lf=_lf(sig, pdis, combined=combined))
    res = gpu_solver.solve(builder.group_window_lps(g))
    st = gpu_solver.kernel_stats()
    # few windows: without CombinedMarket (K^T width <= 4) the 512-thread ELL kernel takes the days (2.5x faster than
    # the generic one here); CombinedMarket LF (width 5) the two-columns-per-lane small variant
    assert st["ell_windows"] == len(days) and (st["variant"] == 5680422) == combined, st
    # many windows: the two-columns-per-lane small variant takes both (9.98 / 15.4 ms for 1,095 days against 11.3 /
    # 40.5 ms, profiles/r05x_market_candidates2.log); replicate the days past two windows per CU
    lps = builder.group_window_lps(g)
    with BatchSolver(0) as se:
        rr = se.solve(lps * (1 + 2 * torch.cuda.get_device_properties(0).multi_processor_count // len(lps)))
        assert se.kernel_stats()["variant"] == 5680422 and se.kernel_stats()["ell_windows"] == len(rr), se.kernel_stats()
        for k, r in enumerate(rr):
            assert r.status == 0 and abs(r.obj - res[k % len(res)].obj) <= 1e-5 * max(abs(r.obj), 1.0), (k, r.obj)
    # the oracle's direct form (options written into the SOE rows, no aggregate columns; tests/test_market_reserves)
    from test_market_reserves import _oracle_window
    wins, _ = cases.market_windows("es")
    res_series = reserve_series(sig, pdis)
    lf = _lf(sig, pdis, combined=combined)
    T = g.T
    for k, (d, r) in enumerate(zip(days, res)):
        o = dict(K=sp_csr(g, k), q=g.q[k], c=g.c[k], c0=float(g.c0[k]), l=g.l[k], u=g.u[k], m_eq=g.m_eq)
        h = window_lp.solve_highs(o)
        assert h["status"] == 0 and r.status == 0, (d, r.status_name, r.iters)
        pres, _ = window_lp.primal_residual_rel(o, r.x)
        assert pres <= PRES_TOL, (d, pres)
        assert abs(r.obj - h["obj"]) <= OBJ_TOL * max(abs(h["obj"]), 1.0), (d, r.obj, h["obj"])
        w = _oracle_window(wins[d], res_series, T)
        sl = slice(d * T, d * T + T)
        w["lf"] = {key: (v[sl] if np.ndim(v) else v) for key, v in lf.items()}
        od = window_lp.build(w)
        x0 = r.x[:od["K"].shape[1]]
        # the uch / udis definition rows' residual adds to the SOE rows' in the direct form: bar x3
        assert window_lp.primal_residual_rel(od, x0)[0] <= 3 * PRES_TOL, d
        assert abs(od["c"] @ x0 + od["c0"] - r.obj) <= 1e-9 * max(abs(r.obj), 1.0)

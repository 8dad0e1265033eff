"""The C++ CPU restatement of the batched PDHG behind the same C ABI (oracle/cpu_pdhg.cpp; SURVEY.md section 4 item 4
"a fake-GPU path: the same ABI served by a C++ CPU PDHG"): it reproduces the numpy restatement's iterations
(oracle/pdlp_ref.py, the algorithm the HIP kernels run) and the HiGHS optimum, and runs the drop-in loop on CPU."""
import numpy as np
import pytest
import scipy.sparse as sp

from dervet_hip.lp import builder, scenarios
from oracle import cases, pdlp_ref, window_lp
from oracle.cpu_pdhg import CpuPdhgSolver


def _lp_dict(lp):
    K = sp.csr_matrix((lp.data, lp.indices, lp.indptr), shape=(lp.m, lp.n))
    return dict(K=K, q=lp.q, c=lp.c, c0=lp.c0, l=lp.l, u=lp.u, m_eq=lp.m_eq)


def test_cpu_restatement_matches_numpy_restatement_and_highs():
    lps = [lp for g in scenarios.config4([0, 1]) for lp in builder.group_window_lps(g)][::5]
    s = CpuPdhgSolver(threads=4)
    res = s.solve(lps)
    for lp, r in zip(lps, res):
        d = _lp_dict(lp)
        ref = pdlp_ref.solve(d)
        h = window_lp.solve_highs(d)
        assert r.status == 0 and ref["status"] == 0
        assert abs(r.iters - ref["iters"]) <= 2 * 32 * 4, (r.iters, ref["iters"])  # within two KKT periods
        assert abs(r.obj - h["obj"]) <= 1e-5 * abs(h["obj"])
        assert window_lp.primal_residual_rel(d, r.x)[0] <= 1e-6


def test_cpu_restatement_golden_windows_and_warm_start():
    wins, arr, meta, _ = cases.case_windows("es")
    bat = cases.battery_from_params(meta["params"])
    groups = scenarios.windows_by_period(2017, 1.0, arr["site_load"][None], None, bat, tariff_def=meta["tariff"],
                                         ene_min=arr["agg_emin"][None], ene_max=arr["agg_emax"][None])
    lps = [lp for g in groups for lp in builder.group_window_lps(g)][:3]
    s = CpuPdhgSolver(threads=3)
    cold = s.solve(lps)
    for i, r in enumerate(cold):
        gold = float(arr["golden_objective"][i].sum())
        assert r.status == 0 and abs(r.obj - gold) <= 1e-5 * abs(gold)
    s.set_options(warm_start=1)
    warm = s.solve(lps, start=[(r.x, r.y) for r in cold])
    assert all(w.status == 0 for w in warm) and sum(w.iters for w in warm) < sum(r.iters for r in cold)


def test_dropin_loop_runs_on_the_cpu_restatement():
    """The drop-in loop with its real exporter (ECOS form -> presolve -> band layout) and the C-ABI solver path,
    without a GPU: the saved objectives equal HiGHS on the original windows."""
    from test_dropin import FakeExporter, FakeScenario, _highs
    from dervet_hip import dropin
    sc = FakeScenario(n_windows=4)
    dropin.batched_optimize_problem_loop(sc, solver=CpuPdhgSolver(threads=4), exporter=FakeExporter([]))
    assert [w for w, *_ in sc.saved] == [0, 1, 2, 3]
    for w, prob, err, _ in sc.saved:
        h = _highs(sc.lps[w])
        assert err is None and prob.status == "optimal" and prob.value == pytest.approx(h.obj, rel=1e-5)


def test_crossed_bounds_report_primal_infeasible_without_iterating():
    """A window whose ene lower bound exceeds its upper bound (a reliability requirement above the energy rating)
    is infeasible as given: PRIMAL_INFEASIBLE at 0 iterations, and the windows around it are unaffected (the GPU
    setup kernel applies the same rule, tests/test_gpu_outage.py)."""
    import dataclasses
    lps = [lp for g in scenarios.config4([0]) for lp in builder.group_window_lps(g)][:3]
    bad_l = lps[1].l.copy()
    T = lps[1].m_eq - 1
    bad_l[2 * T + 5] = lps[1].u[2 * T + 5] + 1.0
    lps[1] = dataclasses.replace(lps[1], l=bad_l)
    res = CpuPdhgSolver(threads=2).solve(lps)
    assert res[1].status_name == "infeasible" and res[1].iters == 0
    assert res[0].status == 0 and res[2].status == 0

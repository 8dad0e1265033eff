"""GPU half of the drop-in export round trip: CVXPY-shaped ECOS data of the golden windows
-> dervet_hip.export (presolve + band canonicalisation) -> the HIP solver through the C ABI -> the ECOS solution
dict -> CVXPY's ECOS inversion (restated in tests/ecos_forms.py) -> the golden per-window objectives."""
import numpy as np
import pytest
import scipy.sparse as sp

import ecos_forms
from dervet_hip import BatchSolver, dropin, export
from oracle import cases, window_lp

pytestmark = pytest.mark.gpu


def _windows(name):
    wins, arr, _, _ = cases.case_windows(name)
    out = []
    for i, w in enumerate(wins):
        olp = window_lp.build(w)
        b = w["bat"]
        data, col = ecos_forms.ecos_form(olp, w["dt"], b["rte"], b["sdr"] / 100.0, b["soc_target"] * b["E"], seed=7 + i,
                                         pins="rows" if i % 2 else "bounds")
        out.append((data, col, export.ecos_to_window(data), float(arr["golden_objective"][i].sum())))
    return out


@pytest.mark.parametrize("name", ["es", "es+pv+dg"])
def test_exported_golden_windows_run_on_the_band_kernel(name):
    ws = _windows(name)
    with BatchSolver(0) as s:
        res = s.solve([ew.lp for _, _, ew, _ in ws])
        ks = s.kernel_stats()
    assert ks["band_windows"] == len(ws), ks
    for (data, col, ew, gold), r in zip(ws, res):
        assert r.status == 0
        sol = ew.ecos_solution(r)
        inv = ecos_forms.invert(sol, data["offset"])
        assert inv["status"] == "optimal"
        assert abs(inv["value"] - gold) <= 1e-5 * abs(gold)
        # primal feasibility of the ECOS form within the solver's relative tolerance, ECOS dual signs
        A, G, b, h = data["A"], data["G"], data["b"], data["h"]
        x, y, z = sol["x"], sol["y"], sol["z"]
        pres = np.sqrt(np.sum((A @ x - b) ** 2) + np.sum(np.maximum(G @ x - h, 0) ** 2)) / (
            1 + np.linalg.norm(np.concatenate([b, h])))
        assert pres <= 1e-6
        assert z.min() >= 0.0
        stat = np.linalg.norm(data["c"] + A.T @ y + G.T @ z) / (1 + np.linalg.norm(data["c"]))
        assert stat <= 1e-5
        assert abs(sol["info"]["dcost"] + data["offset"] - gold) <= 1e-5 * abs(gold)


def test_dropin_loop_with_exported_windows_on_the_gpu():
    """batched_optimize_problem_loop over exported golden windows, saved through the ECOS inversion."""
    import types

    import pandas as pd
    ws = _windows("es")

    class Exporter:
        def export(self, functions, constraints):
            data, col, ew, _ = functions["w"]
            return dropin.CvxpyWindow(ew, ecos_forms.FakeProblem(data, col))

    saved = []
    sc = types.SimpleNamespace(
        optimization_levels=pd.DataFrame({"predictive": np.arange(len(ws))}),
        poi=types.SimpleNamespace(der_list=[], active_ders=[], is_sizing_optimization=False),
        service_agg=types.SimpleNamespace(identify_system_requirements=lambda *a: {},
                                          post_facto_reliability_only=lambda: False,
                                          post_facto_reliability_only_and_user_defined_constraints=lambda: False,
                                          value_streams={}),
        opt_years=[2017], frequency="1h", opt_engine=True,
        set_up_optimization=lambda w, annuity_scalar=1, ignore_der_costs=False: ({"w": ws[w]}, ["c"], w),
        save_optimization_results=lambda w, si, prob, obj, err: saved.append((w, prob.status, prob.value, err)))
    with BatchSolver(0) as s:
        dropin.batched_optimize_problem_loop(sc, solver=s, exporter=Exporter())
        assert s.kernel_stats()["band_windows"] == len(ws)
    assert [w for w, *_ in saved] == list(range(len(ws)))
    for (w, status, value, err), (_, _, _, gold) in zip(saved, ws):
        assert status == "optimal" and err is None and abs(value - gold) <= 1e-5 * abs(gold)


@pytest.mark.parametrize("name", ["es", "es+pv", "es+pv+dg"])
def test_relaxed_milp_market_days_through_the_exporter(name):
    """The opt-in LP relaxation of binary = 1 windows end to end: Usecase 3 golden days in the
    ECOS_BB form CVXPY hands the reference's MILP (boolean on_c / on_d, ``bool_vars_idx``) -> export with relax=True
    -> the HIP solver -> ECOS inversion.  Bars: within 1e-5 of HiGHS on the relaxed restatement, primal residual
    <= 1e-6 on the ECOS form, and <= the golden MILP objective of the day."""
    wins, _ = cases.market_windows(name, relax=False)
    days = list(range(3, 365, 9))
    exp = []
    for d in days:
        data, col = ecos_forms.ecos_bb_market_form(wins[d], seed=d)
        exp.append((data, export.ecos_to_window(data, relax=True)))
    with BatchSolver(0) as s:
        res = s.solve([ew.lp for _, ew in exp])
    worst = 0.0
    for d, (data, ew), r in zip(days, exp, res):
        assert r.status == 0, (name, d, r.status_name, r.iters)
        ref = window_lp.solve_highs(window_lp.build(dict(wins[d], binary_relax=True)))
        sol = ew.ecos_solution(r)
        inv = ecos_forms.invert(sol, data["offset"])
        assert inv["status"] == "optimal"
        rel = abs(inv["value"] - ref["obj"]) / max(abs(ref["obj"]), 1.0)
        worst = max(worst, rel)
        assert rel <= 1e-5, (name, d, inv["value"], ref["obj"])
        gold = float(wins[d]["golden_objective"].sum())
        assert inv["value"] <= gold + 1e-5 * max(abs(gold), 1.0), (name, d, inv["value"], gold)
        A, G, b, h, x = data["A"], data["G"], data["b"], data["h"], sol["x"]
        pres = np.sqrt(np.sum((A @ x - b) ** 2) + np.sum(np.maximum(G @ x - h, 0) ** 2)) / (
            1 + np.linalg.norm(np.concatenate([b, h])))
        assert pres <= 1e-6, (name, d, pres)
    print(f"{name}: {len(days)} relaxed days, worst objective rel err {worst:.2e}")


def test_two_cases_batched_through_dervet_solve_on_the_gpu():
    """DERVET.solve patched by install(batch_cases=True) -- two cases (the es and es+pv+dg golden
    years) set up by their preambles, all 24 exported windows in ONE solve on the band kernel, saved per case in the
    reference order through the ECOS inversion, add_instance in key order.  Each case's DER set changes in its last
    window (a DER not operational that year): the save sees the window's own set."""
    import types

    import pandas as pd

    class Exporter:
        def export(self, functions, constraints):
            data, col, ew, _ = functions["w"]
            return dropin.CvxpyWindow(ew, ecos_forms.FakeProblem(data, col))

    class DER:
        def __init__(self, name, last):
            self.name, self.last, self.variables_dict = name, last, None

        def operational(self, w):
            return w <= self.last

    class Case:
        def __init__(self, value):
            self.name = value
            self.ws = _windows(value)
            n = len(self.ws)
            self.ders = [DER("es", n), DER("pv", n - 2)]
            self.optimization_levels = pd.DataFrame({"predictive": np.arange(n)})
            self.poi = types.SimpleNamespace(der_list=self.ders, active_ders=list(self.ders),
                                             is_sizing_optimization=False)
            self.service_agg = types.SimpleNamespace(
                identify_system_requirements=lambda *a: {}, post_facto_reliability_only=lambda: False,
                post_facto_reliability_only_and_user_defined_constraints=lambda: False, value_streams={})
            self.opt_years, self.frequency, self.opt_engine, self.saved = [2017], "1h", True, []

        set_up_poi_and_service_aggregator = initialize_cba = fill_and_drop_extra_data = sizing_module = \
            lambda self: None

        def set_up_optimization(self, w, annuity_scalar=1, ignore_der_costs=False):
            self.poi.active_ders = [d for d in self.ders if d.operational(w)]
            for d in self.poi.active_ders:
                d.variables_dict = {"window": w}
            return {"w": self.ws[w]}, ["c"], w

        def save_optimization_results(self, w, si, prob, obj, err):
            self.saved.append((w, prob.status, prob.value, err,
                               [(d.name, d.variables_dict["window"]) for d in self.poi.active_ders]))

    added = []
    calls = []

    class Registry:
        @staticmethod
        def add_instance(key, run):
            added.append((key, run))

        @staticmethod
        def sensitivity_summary():
            added.append(("summary", None))

    class Solver(BatchSolver):
        def solve(self, lps):
            calls.append(len(lps))
            out = super().solve(lps)
            calls.append(self.kernel_stats()["band_windows"])
            return out

    class Driver:
        def __init__(self, cases_):
            self.cases = cases_

    mod = types.SimpleNamespace(MicrogridScenario=Case, MicrogridResult=Registry, DERVET=Driver)
    Driver.solve = lambda self: None
    dropin.install(mod, batch_cases=True, solver_factory=lambda: Solver(0), exporter_factory=Exporter)
    mod.DERVET({"a": "es", "b": "es+pv+dg"}).solve()
    assert calls == [24, 24]
    assert [k for k, _ in added] == ["a", "b", "summary"]
    for key, run in added[:2]:
        n = len(run.ws)
        assert [s[0] for s in run.saved] == list(range(n))
        for (w, status, value, err, seen), (_, _, _, gold) in zip(run.saved, run.ws):
            assert status == "optimal" and err is None and abs(value - gold) <= 1e-5 * abs(gold)
            assert seen == [(d.name, w) for d in run.ders if d.operational(w)]

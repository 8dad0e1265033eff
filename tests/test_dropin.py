"""Drop-in window loop (dervet_hip.dropin) exercised with fakes of the reference objects it touches.

storagevet / cvxpy are absent, so the scenario, POI, service aggregator, DERs and
the exporter are fakes with the reference's method names; the solver is a CPU stand-in that answers with
HiGHS (it replaces only the GPU call, to check the loop's ordering, write-back and fallback logic).
"""
import types

import numpy as np
import pandas as pd
import pytest

from dervet_hip import WindowResult, dropin
from dervet_hip.lp import builder, scenarios
from oracle import window_lp


class FakeDER:
    def __init__(self, name, degrade=False):
        self.name = name
        self.incl_cycle_degrade = degrade
        self.variables_dict = None


class FakeSA:
    def __init__(self):
        self.value_streams = {"Reliability": types.SimpleNamespace(use_soc_init=False, use_user_const=False)}

    def identify_system_requirements(self, der_list, opt_years, frequency):
        return {"req": len(der_list)}

    def post_facto_reliability_only(self):
        return False

    def post_facto_reliability_only_and_user_defined_constraints(self):
        return False


class FakeScenario:
    """Windows are config-4 window LPs; set_up_optimization re-creates the DER variables per window."""

    def __init__(self, n_windows=6, empty=(), milp=(), degrade=False):
        groups = scenarios.config4([0])
        self.lps = [lp for g in groups for lp in builder.group_window_lps(g)][:n_windows]
        self.optimization_levels = pd.DataFrame({"predictive": np.arange(n_windows)})
        self.ders = [FakeDER("es", degrade)]
        self.poi = types.SimpleNamespace(der_list=self.ders, active_ders=self.ders, is_sizing_optimization=False)
        self.service_agg = FakeSA()
        self.opt_years = [2017]
        self.frequency = "1h"
        self.opt_engine = True
        self.empty, self.milp = set(empty), set(milp)
        self.saved, self.reference_solves, self.log = [], [], []

    def set_up_optimization(self, opt_period, annuity_scalar=1, ignore_der_costs=False):
        self.log.append(("setup", int(opt_period)))
        for der in self.ders:
            der.variables_dict = {"window": int(opt_period)}
        if opt_period in self.empty:
            return {}, [], opt_period
        return {"lp": self.lps[opt_period]}, ["c"], opt_period

    def solve_optimization(self, functions, constraints):
        self.reference_solves.append(functions["lp"])
        lp = functions["lp"]
        h = _highs(lp)
        return types.SimpleNamespace(status="optimal", value=h.obj, x=h.x), functions, None

    def save_optimization_results(self, opt_window_num, sub_index, prob, obj_expression, cvx_error_msg):
        self.log.append(("save", int(opt_window_num)))
        self.saved.append((int(opt_window_num), prob, cvx_error_msg, dict(self.ders[0].variables_dict)))


def _highs(lp):
    import scipy.sparse as sp
    K = sp.csr_matrix((lp.data, lp.indices, lp.indptr), shape=(lp.m, lp.n))
    h = window_lp.solve_highs(dict(K=K, q=lp.q, c=lp.c, c0=lp.c0, l=lp.l, u=lp.u, m_eq=lp.m_eq))
    return WindowResult(h["x"], h["y"], h["obj"], 0, 0, 0.0, 0.0, 0.0)


class FakeExporter:
    def __init__(self, milp):
        self.milp = milp

    def export(self, functions, constraints):
        lp = functions["lp"]
        if any(lp is m for m in self.milp):
            return None
        win = types.SimpleNamespace(lp=lp)
        win.unpack = lambda r: types.SimpleNamespace(status=r.status_name, value=r.obj, x=r.x)
        return win


class CpuStandInSolver:
    def __init__(self):
        self.calls = []

    def solve(self, lps):
        self.calls.append(len(lps))
        return [_highs(lp) for lp in lps]


def test_batched_loop_orders_saves_and_repoints_variables():
    sc = FakeScenario(n_windows=6, empty={2})
    solver = CpuStandInSolver()
    plan = dropin.batched_optimize_problem_loop(sc, solver=solver, exporter=FakeExporter([]))
    assert solver.calls == [5]  # one batched call for the 5 non-empty LP windows
    assert [s[0] for s in sc.saved] == [0, 1, 3, 4, 5]
    # every setup happens before any save (batched), saves follow the reference window order
    kinds = [k for k, _ in sc.log]
    assert kinds.index("save") > max(i for i, k in enumerate(kinds) if k == "setup")
    # each save sees its own window's variables_dict (re-pointed before save_optimization_results)
    assert all(s[3]["window"] == s[0] for s in sc.saved)
    assert all(s[2] is None for s in sc.saved)
    assert len(plan) == 5


def test_milp_windows_fall_back_in_place():
    sc = FakeScenario(n_windows=4)
    milp = [sc.lps[1]]
    solver = CpuStandInSolver()
    dropin.batched_optimize_problem_loop(sc, solver=solver, exporter=FakeExporter(milp))
    assert solver.calls == [3]
    assert len(sc.reference_solves) == 1 and sc.reference_solves[0] is sc.lps[1]
    assert [s[0] for s in sc.saved] == [0, 1, 2, 3]


def test_coupled_windows_run_the_reference_loop():
    sc = FakeScenario(n_windows=3, degrade=True)
    solver = CpuStandInSolver()
    dropin.batched_optimize_problem_loop(sc, solver=solver, exporter=FakeExporter([]))
    assert solver.calls == [] and len(sc.reference_solves) == 3
    assert [k for k, _ in sc.log] == ["setup", "save"] * 3


def test_nonoptimal_status_becomes_error_message():
    sc = FakeScenario(n_windows=2)

    class Bad(CpuStandInSolver):
        def solve(self, lps):
            out = super().solve(lps)
            out[1].status = 3  # ITER_LIMIT
            return out

    dropin.batched_optimize_problem_loop(sc, solver=Bad(), exporter=FakeExporter([]))
    assert sc.saved[0][2] is None and "optimal_inaccurate" in sc.saved[1][2]


def test_opt_engine_off_returns_before_any_window():
    sc = FakeScenario(n_windows=2)
    sc.opt_engine = False
    assert dropin.batched_optimize_problem_loop(sc, solver=CpuStandInSolver(), exporter=FakeExporter([])) is None
    assert sc.log == [] and sc.system_requirements == {"req": 1}


def test_install_patches_the_hard_coded_scenario_class():
    mod = types.SimpleNamespace(MicrogridScenario=FakeScenario)
    cls = dropin.install(mod)
    assert mod.MicrogridScenario is cls and issubclass(cls, FakeScenario)
    assert dropin.install(mod) is cls


def test_cvxpy_exporter_requires_cvxpy():
    try:
        import cvxpy  # noqa: F401
    except ImportError:
        with pytest.raises(ImportError):
            dropin.CvxpyExporter()

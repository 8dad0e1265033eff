"""Drop-in window loop (dervet_hip.dropin) exercised with fakes of the reference objects it touches.

storagevet / cvxpy are absent, so the scenario, POI, service aggregator and DERs are fakes
with the reference's method names.  The export is the real one: each window is written in the form CVXPY 1.0.31
hands ECOS (tests/ecos_forms.py) and goes through dervet_hip.export; results come back through a restatement of
CVXPY's ECOS inversion (ecos_forms.FakeProblem).  The solver is a CPU stand-in that answers with HiGHS on the
exported LP (it replaces only the GPU call, to check the loop's ordering, write-back and fallback logic; the GPU
run of the same loop is tests/test_gpu_export.py).
"""
import types

import numpy as np
import pandas as pd
import pytest
import scipy.sparse as sp

import ecos_forms
from dervet_hip import WindowResult, dropin, export
from dervet_hip.lp import builder, scenarios
from oracle import cases, window_lp


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


_LPS = {}


def _config4_lps(scen):
    if scen not in _LPS:
        _LPS[scen] = [lp for g in scenarios.config4([scen]) for lp in builder.group_window_lps(g)]
    return _LPS[scen]


class FakeScenario:
    """Windows are config-4 window LPs; set_up_optimization re-creates the DER variables per window."""

    def __init__(self, n_windows=6, empty=(), milp=(), degrade=False, scen=0, journal=None):
        self.lps = _config4_lps(scen)[:n_windows]
        self.optimization_levels = pd.DataFrame({"predictive": np.arange(n_windows)})
        self.ders = [FakeDER("es", degrade)]
        self.poi = types.SimpleNamespace(der_list=self.ders, active_ders=self.ders, is_sizing_optimization=False)
        self.service_agg = FakeSA()
        self.opt_years = [2017]
        self.frequency = "1h"
        self.opt_engine = True
        self.empty, self.milp = set(empty), set(milp)
        self.saved, self.reference_solves, self.log = [], [], []
        self.journal = journal if journal is not None else []
        self.scen = scen

    def set_up_optimization(self, opt_period, annuity_scalar=1, ignore_der_costs=False):
        self.log.append(("setup", int(opt_period)))
        self.journal.append((self.scen, "setup", int(opt_period)))
        for der in self.ders:
            der.variables_dict = {"window": int(opt_period)}
        if opt_period in self.empty:
            return {}, [], opt_period
        return {"lp": self.lps[opt_period]}, ["c"], opt_period

    def solve_optimization(self, functions, constraints):
        self.reference_solves.append(functions["lp"])
        h = _highs(functions["lp"])
        return types.SimpleNamespace(status="optimal", value=h.obj, x=h.x), functions, None

    def save_optimization_results(self, opt_window_num, sub_index, prob, obj_expression, cvx_error_msg):
        self.log.append(("save", int(opt_window_num)))
        self.journal.append((self.scen, "save", int(opt_window_num)))
        self.saved.append((int(opt_window_num), prob, cvx_error_msg, dict(self.ders[0].variables_dict)))


def _highs(lp):
    K = sp.csr_matrix((lp.data, lp.indices, lp.indptr), shape=(lp.m, lp.n))
    h = window_lp.solve_highs(dict(K=K, q=lp.q, c=lp.c, c0=lp.c0, l=lp.l, u=lp.u, m_eq=lp.m_eq))
    return WindowResult(h["x"], h["y"], h["obj"], 0, 0, 0.0, 0.0, 0.0)


class FakeExporter:
    """Writes the window in CVXPY's ECOS form and exports it with dervet_hip.export (MILP windows: None)."""

    def __init__(self, milp):
        self.milp = milp

    def export(self, functions, constraints):
        lp = functions["lp"]
        if any(lp is m for m in self.milp):
            return None
        olp, dt, eta, sdr, target = ecos_forms.oracle_lp_of(lp)
        data, col = ecos_forms.ecos_form(olp, dt, eta, sdr, target, seed=len(lp.c))
        return dropin.CvxpyWindow(export.ecos_to_window(data), ecos_forms.FakeProblem(data, col))


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
    # the values arrive through the ECOS inversion: status and objective as the reference's solve leaves them
    for w, prob, err, _ in sc.saved:
        assert prob.status == "optimal"
        assert prob.value == pytest.approx(_highs(sc.lps[w]).obj, rel=1e-9)
        # the primal x in ECOS order is the window's solution (builder layout through the export's column map)
        lp = sc.lps[w]
        assert lp.c @ prob.x[prob.col] + lp.c0 == pytest.approx(prob.value, rel=1e-12)


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


def test_statuses_reach_save_as_the_reference_solve_leaves_them():
    """a non-optimal window must not abort the loop.  Iteration limit -> optimal_inaccurate with the
    solution; infeasible -> status 'infeasible' (no error, as CVXPY reports it); numerical failure -> CVXPY would
    raise SolverError: the problem stays unsolved and the message is the window's cvx_error_msg."""
    sc = FakeScenario(n_windows=4)

    class Mixed(CpuStandInSolver):
        def solve(self, lps):
            out = super().solve(lps)
            out[1].status = 3   # ITER_LIMIT
            out[2].status = 1   # PRIMAL_INFEASIBLE
            out[3].status = 4   # NUMERICAL
            return out

    dropin.batched_optimize_problem_loop(sc, solver=Mixed(), exporter=FakeExporter([]), retry_failed=False)
    st = {w: (prob.status, err) for w, prob, err, _ in sc.saved}
    assert st[0] == ("optimal", None)
    assert st[1] == ("optimal_inaccurate", None)
    assert st[2] == ("infeasible", None)
    assert st[3][0] is None and "solver error" in st[3][1]
    assert [w for w, *_ in sc.saved] == [0, 1, 2, 3]
    assert sc.dervet_hip_report.as_dict()["gpu"] == 4 and sc.reference_solves == []


def test_failed_windows_are_re_solved_by_the_reference_in_place():
    """SURVEY.md section 5 failure row: a window without a certified GPU optimum (iteration
    limit, infeasible verdict, numerical failure) is re-solved by the reference solve_optimization in its place in
    the order, and saved with what that solve returns (MicrogridScenario.py:319-320)."""
    sc = FakeScenario(n_windows=5)

    class Mixed(CpuStandInSolver):
        def solve(self, lps):
            out = super().solve(lps)
            out[1].status = 3   # ITER_LIMIT
            out[2].status = 1   # PRIMAL_INFEASIBLE
            out[4].status = 4   # NUMERICAL
            return out

    dropin.batched_optimize_problem_loop(sc, solver=Mixed(), exporter=FakeExporter([]))
    assert [w for w, *_ in sc.saved] == [0, 1, 2, 3, 4]
    assert [id(lp) for lp in sc.reference_solves] == [id(sc.lps[w]) for w in (1, 2, 4)]
    for w, prob, err, vd in sc.saved:
        assert prob.status == "optimal" and err is None and vd["window"] == w
        assert prob.value == pytest.approx(_highs(sc.lps[w]).obj, rel=1e-9)
    rep = sc.dervet_hip_report.as_dict()
    assert rep["gpu"] == 2 and rep["retried"] == 3 and rep["reference"] == 0
    assert rep["retried_status"] == {"optimal_inaccurate": 1, "infeasible": 1, "solver_error": 1}


def test_forced_iteration_limit_is_re_solved_by_the_reference():
    """A real solver run out of iterations (the C++ restatement of the GPU algorithm behind the same C ABI, so
    this runs without a GPU; max_iters far below what the windows need) -> every window ITER_LIMIT -> every window
    re-solved by the reference."""
    from oracle import cpu_pdhg
    sc = FakeScenario(n_windows=3)
    solver = cpu_pdhg.CpuPdhgSolver(threads=2, max_iters=64)
    try:
        dropin.batched_optimize_problem_loop(sc, solver=solver, exporter=FakeExporter([]))
    finally:
        solver.close()
    assert len(sc.reference_solves) == 3
    assert sc.dervet_hip_report.as_dict()["retried_status"] == {"optimal_inaccurate": 3}
    assert all(prob.status == "optimal" for _, prob, _, _ in sc.saved)


def test_cases_loop_batches_independent_cases_and_steps_coupled_ones_in_lockstep():
    journal = []
    cases_ = [FakeScenario(n_windows=3, scen=0, journal=journal),
              FakeScenario(n_windows=3, scen=1, degrade=True, journal=journal),
              FakeScenario(n_windows=2, scen=2, degrade=True, journal=journal),
              FakeScenario(n_windows=2, scen=3, journal=journal)]
    solver = CpuStandInSolver()
    plans = dropin.batched_cases_loop(cases_, solver=solver, exporter=FakeExporter([]))
    # independent cases: all 5 windows in one call; coupled: one call per window position (2, 2, 1 windows)
    assert solver.calls == [5, 2, 2, 1]
    assert [len(p) for p in plans] == [3, 3, 2, 2]
    # lockstep: a coupled case's window k is saved before any coupled case sets up window k + 1
    coupled = [e for e in journal if e[0] in (1, 2)]
    for k in (1, 2):
        first_setup_k = min(i for i, e in enumerate(coupled) if e[1] == "setup" and e[2] == k)
        last_save_prev = max(i for i, e in enumerate(coupled) if e[1] == "save" and e[2] == k - 1)
        assert last_save_prev < first_setup_k
    for c in cases_:
        assert [w for w, *_ in c.saved] == list(range(len(c.lps)))
        for w, prob, err, _ in c.saved:
            assert err is None and prob.value == pytest.approx(_highs(c.lps[w]).obj, rel=1e-9)


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


class FakeMarketScenario(FakeScenario):
    """Usecase 3 golden market days (binary = 1): the reference solve is the MILP (HiGHS MILP on the restatement,
    pinned to the golden objectives by tests/test_market_oracle.py)."""

    def __init__(self, days, name="es"):
        super().__init__(n_windows=len(days))
        wins, _ = cases.market_windows(name, relax=False)
        self.wins = [wins[d] for d in days]

    def set_up_optimization(self, opt_period, annuity_scalar=1, ignore_der_costs=False):
        self.log.append(("setup", int(opt_period)))
        for der in self.ders:
            der.variables_dict = {"window": int(opt_period)}
        return {"win": self.wins[opt_period]}, ["c"], opt_period

    def solve_optimization(self, functions, constraints):
        self.reference_solves.append(functions["win"])
        h = window_lp.solve_highs_milp(functions["win"])
        return types.SimpleNamespace(status="optimal", value=h["obj"], x=h["x"]), functions, None


class FakeMilpExporter:
    """What CvxpyExporter does with a boolean window: None (reference path) unless relax_milp, else the ECOS_BB
    data exported with relax=True."""

    def __init__(self, relax_milp):
        self.relax_milp = relax_milp

    def export(self, functions, constraints):
        if not self.relax_milp:
            return None
        data, col = ecos_forms.ecos_bb_market_form(functions["win"], seed=3)
        return dropin.CvxpyWindow(export.ecos_to_window(data, relax=True), ecos_forms.FakeProblem(data, col))


@pytest.mark.parametrize("relax", [False, True])
def test_milp_windows_relaxed_only_on_opt_in(relax):
    """north_star: MILP windows stay on the reference path, and the GPU solves their LP relaxation only when the
    user opts in.  Off: every day goes to the reference MILP solve (golden objective).  On: every day is solved as
    its LP relaxation by the batched solver, and each relaxed optimum is <= the golden MILP objective."""
    days = [5, 120, 250]
    sc = FakeMarketScenario(days)
    solver = CpuStandInSolver()
    dropin.batched_optimize_problem_loop(sc, solver=solver, exporter=FakeMilpExporter(relax), relax_milp=relax)
    rep = sc.dervet_hip_report.as_dict()
    assert [w for w, *_ in sc.saved] == [0, 1, 2]
    for (w, prob, err, _), win in zip(sc.saved, sc.wins):
        gold = float(win["golden_objective"].sum())
        assert err is None and prob.status == "optimal"
        if relax:
            assert prob.value <= gold + 1e-9 * max(1.0, abs(gold))
        else:
            assert prob.value == pytest.approx(gold, rel=1e-7, abs=1e-7)
    if relax:
        assert solver.calls == [3] and rep["relaxed"] == 3 and rep["gpu"] == 3 and not sc.reference_solves
    else:
        assert solver.calls == [] and rep["reference"] == 3 and len(sc.reference_solves) == 3


def test_install_passes_the_opt_in_through():
    mod = types.SimpleNamespace(MicrogridScenario=FakeScenario)
    cls = dropin.install(mod, relax_milp=True)
    assert cls.dervet_hip_options[1:] == (True, True)
    cls2 = dropin.install(mod)      # re-installed with the default (no relaxation) over the reference class
    assert cls2 is not cls and cls2.__bases__[0] is FakeScenario and cls2.dervet_hip_options[1:] == (False, True)


def test_cvxpy_exporter_requires_cvxpy():
    try:
        import cvxpy  # noqa: F401
    except ImportError:
        with pytest.raises(ImportError):
            dropin.CvxpyExporter()

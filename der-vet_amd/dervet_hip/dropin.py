"""Drop-in batched window loop beneath DER-VET's ``MicrogridScenario``.

Reference loop (dervet/MicrogridScenario.py:281-320, serial over windows):

    for opt_period in self.optimization_levels.predictive.unique():
        functions, constraints, sub_index = self.set_up_optimization(opt_period, annuity_scalar=alpha, ...)
        if not len(constraints) and not len(functions.values()): continue
        cvx_problem, obj_expressions, cvx_error_msg = self.solve_optimization(functions, constraints)   # :319
        self.save_optimization_results(opt_period, sub_index, cvx_problem, obj_expressions, cvx_error_msg)

``batched_optimize_problem_loop`` keeps the same preamble and the same per-window
``set_up_optimization`` / ``save_optimization_results`` calls, in the same order, but replaces the
per-window ``solve_optimization`` by ONE ``BatchSolver.solve`` over every LP window:

  1. set up every window with the unchanged ``set_up_optimization`` and export it immediately
     (``CvxpyExporter``: cvxpy ``get_problem_data`` -> canonical LP), keeping that window's DER
     ``variables_dict`` objects (CVXPY variables are re-created per window, ElectricVehicles.py:96-122);
  2. solve all exported windows in one batch on the GPU;
  3. per window, in order: re-point each DER's ``variables_dict``, write the solution into the CVXPY
     variables, and call the unchanged ``save_optimization_results``.

Windows that are not LPs (binary / integer variables: MILP, ESSSizing.py:82-138) are solved by the
reference ``solve_optimization`` in their place in the order.  Scenarios whose windows are coupled through
saved results (battery degradation, Battery.py:87-110; sizing, MicrogridScenario.py:361-363) run the
reference loop unchanged.  ``DERVET.solve`` hard-codes ``MicrogridScenario`` (dervet/DERVET.py:76), so
``install`` patches that name with the batched subclass.
"""
import numpy as np

from . import _lib
from .solver import BatchSolver, WindowLP

STATUS_TO_CVXPY = _lib.STATUS_NAMES  # DVH status -> cvxpy status string read by save_optimization_results


class CvxpyExporter:
    """(functions, constraints) of one window -> WindowLP via CVXPY's ECOS canonicalisation.

    ECOS data: min c'x + offset  s.t.  A x = b,  G x + s = h,  s in K.  An LP window has a purely
    nonnegative cone (dims.q / dims.e empty), i.e.  G x <= h  ->  K_I = -G, q_I = -h.
    """

    def __init__(self):
        import cvxpy as cvx  # noqa: F401  (absent in this container; the native builder is used there)
        self.cvx = cvx

    def export(self, functions, constraints):
        cvx = self.cvx
        prob = cvx.Problem(cvx.Minimize(sum(functions.values())), constraints)
        if any(v.attributes.get("boolean") or v.attributes.get("integer") for v in prob.variables()):
            return None  # MILP: stays on the reference path
        data, chain, inverse = prob.get_problem_data(cvx.ECOS)
        dims = data["dims"]
        if getattr(dims, "soc", None) or getattr(dims, "exp", 0):
            return None
        import scipy.sparse as sp
        A = sp.csr_matrix(data["A"]) if data.get("A") is not None else sp.csr_matrix((0, len(data["c"])))
        G = sp.csr_matrix(data["G"]) if data.get("G") is not None else sp.csr_matrix((0, len(data["c"])))
        K = sp.vstack([A, -G]).tocsr()
        q = np.concatenate([np.asarray(data.get("b", np.zeros(A.shape[0])), float).ravel(),
                            -np.asarray(data["h"], float).ravel()])
        n = len(data["c"])
        lp = WindowLP.from_csr(K, q, np.asarray(data["c"], float), np.full(n, -np.inf), np.full(n, np.inf),
                               A.shape[0], float(data.get("offset", 0.0)))
        return _CvxpyWindow(prob, chain, inverse, lp, A.shape[0])


class _CvxpyWindow:
    def __init__(self, prob, chain, inverse, lp, m_eq):
        self.prob, self.chain, self.inverse, self.lp, self.m_eq = prob, chain, inverse, lp, m_eq

    def unpack(self, res):
        """Write a WindowResult into the CVXPY variables (same path ECOS results take)."""
        y = res.y
        sol = {"x": res.x, "y": y[:self.m_eq], "z": -y[self.m_eq:],
               "info": {"exitFlag": 0 if res.status == 0 else -1, "pcost": res.obj, "iter": res.iters}}
        self.prob.unpack_results(sol, self.chain, self.inverse)
        return self.prob


def windows_are_independent(scenario):
    """Batched solve is valid when no window's setup depends on an earlier window's saved results."""
    poi = scenario.poi
    if getattr(poi, "is_sizing_optimization", False):
        return False
    for der in getattr(poi, "der_list", []):
        if getattr(der, "incl_cycle_degrade", False) or getattr(der, "yearly_degrade", 0):
            return False
    return True


def batched_optimize_problem_loop(scenario, solver=None, exporter=None, **kwargs):
    """Batched ``MicrogridScenario.optimize_problem_loop`` (dervet/MicrogridScenario.py:281-320)."""
    sa, poi = scenario.service_agg, scenario.poi
    # ---- preamble, verbatim in effect (:289-307)
    scenario.system_requirements = sa.identify_system_requirements(poi.der_list, scenario.opt_years,
                                                                   scenario.frequency)
    alpha = 1
    if poi.is_sizing_optimization:
        alpha = scenario.cost_benefit_analysis.annuity_scalar(scenario.opt_years)
    if sa.post_facto_reliability_only():
        sa.value_streams["Reliability"].use_soc_init = True
    if sa.post_facto_reliability_only_and_user_defined_constraints():
        sa.value_streams["Reliability"].use_user_const = True
    if not scenario.opt_engine:
        return
    ignore = sa.post_facto_reliability_only()
    if not windows_are_independent(scenario):
        for opt_period in scenario.optimization_levels.predictive.unique():
            functions, constraints, sub_index = scenario.set_up_optimization(opt_period, annuity_scalar=alpha,
                                                                             ignore_der_costs=ignore)
            if not len(constraints) and not len(functions.values()):
                continue
            prob, obj, err = scenario.solve_optimization(functions, constraints)
            scenario.save_optimization_results(opt_period, sub_index, prob, obj, err)
        return
    exporter = exporter or CvxpyExporter()
    # ---- 1. set up + export every window
    plan = []
    for opt_period in scenario.optimization_levels.predictive.unique():
        functions, constraints, sub_index = scenario.set_up_optimization(opt_period, annuity_scalar=alpha,
                                                                         ignore_der_costs=ignore)
        if not len(constraints) and not len(functions.values()):
            continue
        saved_vars = {der: getattr(der, "variables_dict", None) for der in getattr(poi, "active_ders", [])}
        win = exporter.export(functions, constraints)
        plan.append((opt_period, sub_index, functions, constraints, saved_vars, win))
    # ---- 2. one batched GPU solve for the LP windows
    lp_idx = [i for i, p in enumerate(plan) if p[5] is not None]
    results = {}
    if lp_idx:
        own = solver is None
        solver = solver or BatchSolver(0)
        try:
            res = solver.solve([plan[i][5].lp for i in lp_idx])
        finally:
            if own:
                solver.close()
        results = dict(zip(lp_idx, res))
    # ---- 3. write back and save, window by window, in the reference order
    for i, (opt_period, sub_index, functions, constraints, saved_vars, win) in enumerate(plan):
        for der, vd in saved_vars.items():
            if vd is not None:
                der.variables_dict = vd
        if win is None:  # MILP / non-LP window: the reference solve, in place
            prob, obj, err = scenario.solve_optimization(functions, constraints)
        else:
            r = results[i]
            prob = win.unpack(r)
            obj = functions
            err = None if r.status == _lib.OPTIMAL else f"dervet_hip: window solve status {r.status_name}"
        scenario.save_optimization_results(opt_period, sub_index, prob, obj, err)
    return plan


def make_batched_scenario_class(base, solver_factory=None):
    """Subclass of the reference ``MicrogridScenario`` whose window loop is batched on the GPU."""

    class BatchedMicrogridScenario(base):
        def optimize_problem_loop(self, **kwargs):
            solver = solver_factory() if solver_factory else None
            try:
                return batched_optimize_problem_loop(self, solver=solver, **kwargs)
            finally:
                if solver is not None:
                    solver.close()

    BatchedMicrogridScenario.__name__ = "BatchedMicrogridScenario"
    return BatchedMicrogridScenario


def install(dervet_module=None):
    """Patch dervet.DERVET.MicrogridScenario (hard-coded at dervet/DERVET.py:76) with the batched class."""
    if dervet_module is None:
        import dervet.DERVET as dervet_module  # noqa: N813
    base = dervet_module.MicrogridScenario
    if getattr(base, "__name__", "") == "BatchedMicrogridScenario":
        return base
    cls = make_batched_scenario_class(base)
    dervet_module.MicrogridScenario = cls
    return cls

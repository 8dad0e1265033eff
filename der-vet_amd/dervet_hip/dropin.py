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
     (``CvxpyExporter``: cvxpy ``get_problem_data(ECOS)`` -> ``export.ecos_to_window``: presolve + band
     canonicalisation), keeping that window's DER ``variables_dict`` objects (CVXPY variables are re-created per
     window, ElectricVehicles.py:96-122);
  2. solve all exported windows in one batch on the GPU;
  3. per window, in order: re-point each DER's ``variables_dict``, hand the solution to CVXPY exactly as ECOS's
     would arrive (``ExportedWindow.ecos_solution`` -> ``Problem.unpack_results``), and call the unchanged
     ``save_optimization_results``.  Statuses map to ECOS exit flags (infeasible 1, unbounded 2, iteration limit
     10 = optimal_inaccurate); a numerical failure, on which CVXPY would raise SolverError, skips
     ``unpack_results`` and is saved with its error message (errors travel as ``cvx_error_msg``,
     MicrogridScenario.py:319-320); the loop goes on either way.

Windows that are not LPs (binary / integer variables: MILP, ``binary`` = 1 in Model_Parameters_Template_DER.csv:17,
e.g. ElectricVehicles.py:120-122) are solved by the reference ``solve_optimization`` in their place in the order,
unless the user opts in with ``relax_milp=True`` (``install(relax_milp=True)``, ``CvxpyExporter(relax_milp=True)``):
then the window is exported through ``get_problem_data(cvx.ECOS_BB)`` and the GPU solves its LP relaxation (boolean
columns boxed to [0, 1], integrality dropped; export.ecos_to_window), whose objective bounds the MILP's from below.

Failure detection: a window the GPU leaves without a certified optimum -- iteration limit,
numerical failure, or an infeasibility / unboundedness verdict -- is re-solved by the reference
``solve_optimization`` in place (``retry_failed``, default on), so that DER-VET receives exactly what its own solve
of that window gives; ``LoopReport`` counts GPU, reference (MILP / non-LP) and retried windows.  With
``retry_failed=False`` the GPU verdict is saved as ECOS would report it (iteration limit -> optimal_inaccurate).  Scenarios whose windows are coupled through
saved results (battery degradation, Battery.py:87-110; sizing, MicrogridScenario.py:361-363) cannot batch their
own windows; ``batched_cases_loop`` batches them ACROSS scenarios instead: window k of every case in one GPU
call, saved before any case sets up window k + 1 (the serial case loop of dervet/DERVET.py:75-83, in lockstep).
``DERVET.solve`` hard-codes ``MicrogridScenario`` (dervet/DERVET.py:76), so ``install`` patches that name with
the batched subclass; ``install(batch_cases=True)`` also replaces ``DERVET.solve`` (DERVET.py:72-90) so that the
windows of every sensitivity case reach the GPU in one batch (``make_batched_dervet_solve``).

Every window is saved with the state its own set-up left: the active-DER list ``poi.grab_active_ders`` chose for
its year (MicrogridScenario.py:342, MicrogridPOI.py:85-91) and its DERs' ``variables_dict``, restored before the
save and before an in-place reference solve (the reference saves each window right after setting it up).
"""
import collections
import time

from . import _lib
from .export import ExportError, ecos_to_window
from .solver import BatchSolver

STATUS_TO_CVXPY = _lib.STATUS_NAMES  # DVH status -> cvxpy status string read by save_optimization_results


class CvxpyExporter:
    """(functions, constraints) of one window -> ExportedWindow via CVXPY's ECOS canonicalisation (ECOS_BB for a
    mixed-integer window when ``relax_milp``; without it such a window stays on the reference path)."""

    def __init__(self, relax_milp=False):
        import cvxpy as cvx  # noqa: F401  (absent in this container; tests drive ecos_to_window directly)
        self.cvx = cvx
        self.relax_milp = bool(relax_milp)

    def export(self, functions, constraints):
        cvx = self.cvx
        prob = cvx.Problem(cvx.Minimize(sum(functions.values())), constraints)
        mip = any(v.attributes.get("boolean") or v.attributes.get("integer") for v in prob.variables())
        if mip and not self.relax_milp:
            return None  # MILP: stays on the reference path
        # ECOS_BB's data carries bool_vars_idx / int_vars_idx (CVXPY 1.0.31 ECOS_BB.apply); its inversion is ECOS's
        data, chain, inverse = prob.get_problem_data(cvx.ECOS_BB if mip else cvx.ECOS)
        try:
            ew = ecos_to_window(data, relax=mip)
        except ExportError:
            return None  # not an LP the solver takes (cones, infeasible presolve): the reference solve
        return CvxpyWindow(ew, prob, chain, inverse)


class CvxpyWindow:
    """An exported window and the CVXPY objects its solution goes back into."""

    def __init__(self, ew, prob=None, chain=None, inverse=None):
        self.ew, self.prob, self.chain, self.inverse = ew, prob, chain, inverse

    @property
    def lp(self):
        return self.ew.lp

    def unpack(self, res):
        """-> (problem, cvx_error_msg), as the reference's solve would leave them: the result goes through CVXPY's
        own ECOS inversion (``unpack_results``) -- optimal / optimal_inaccurate write the variables, infeasible /
        unbounded set the status and value as an ECOS result would -- except a numerical failure, for which
        CVXPY would raise SolverError inside ``prob.solve``: the problem stays unsolved and the message is the
        window's cvx_error_msg (MicrogridScenario.py:319-320)."""
        if res.status == _lib.NUMERICAL:
            return self.prob, f"dervet_hip: window solve status {res.status_name} (solver error)"
        self.prob.unpack_results(self.ew.ecos_solution(res), self.chain, self.inverse)
        return self.prob, None


RETRY_STATUSES = (_lib.ITER_LIMIT, _lib.NUMERICAL, _lib.PRIMAL_INFEASIBLE, _lib.DUAL_INFEASIBLE)


class LoopReport:
    """Where a loop's windows were solved: ``gpu`` (saved from the batched solve, ``relaxed`` of them MILP
    relaxations), ``reference`` (MILP / non-LP windows solved by ``solve_optimization`` in place) and ``retried``
    (GPU windows without a certified optimum, re-solved by ``solve_optimization``; ``retried_status`` counts them
    by the cvxpy status string of the GPU verdict)."""

    def __init__(self):
        self.gpu = self.relaxed = self.reference = self.retried = 0
        self.retried_status = {}

    def as_dict(self):
        return dict(gpu=self.gpu, relaxed=self.relaxed, reference=self.reference, retried=self.retried,
                    retried_status=dict(self.retried_status))

    def __repr__(self):
        return f"LoopReport({self.as_dict()})"


def windows_are_independent(scenario):
    """Batched solve is valid when no window's setup depends on an earlier window's saved results."""
    poi = scenario.poi
    if getattr(poi, "is_sizing_optimization", False):
        return False
    for der in getattr(poi, "der_list", []):
        if getattr(der, "incl_cycle_degrade", False) or getattr(der, "yearly_degrade", 0):
            return False
    return True


def _preamble(scenario):
    """MicrogridScenario.optimize_problem_loop :289-307 in effect; returns (alpha, ignore_der_costs) or None when
    the optimizer is off."""
    sa, poi = scenario.service_agg, scenario.poi
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
        return None
    return alpha, sa.post_facto_reliability_only()


WindowPlan = collections.namedtuple(
    "WindowPlan", "opt_period sub_index functions constraints saved_vars win active_ders")
WindowPlan.__doc__ = """One window between its set-up and its save: what ``set_up_optimization`` returned, the
variables_dict of each active DER (re-created per window), the export (None: reference solve) and the window's own
active-DER list (``poi.grab_active_ders(sub_index)``, MicrogridScenario.py:342 / MicrogridPOI.py:85-91)."""


def _setup_export(scenario, opt_period, alpha, ignore, exporter):
    """set_up_optimization of one window + its export; None for a window with nothing to optimize (:316-318)."""
    functions, constraints, sub_index = scenario.set_up_optimization(opt_period, annuity_scalar=alpha,
                                                                     ignore_der_costs=ignore)
    if not len(constraints) and not len(functions.values()):
        return None
    active = getattr(scenario.poi, "active_ders", None)
    active = None if active is None else list(active)
    saved_vars = {der: getattr(der, "variables_dict", None) for der in (active or [])}
    return WindowPlan(opt_period, sub_index, functions, constraints, saved_vars,
                      exporter.export(functions, constraints), active)


def _restore_window_state(scenario, plan):
    """Put back what this window's set-up left on the scenario before anything of the reference reads it: the
    window's active-DER list (the save iterates ``poi.active_ders``, MicrogridScenario.py:361 and storagevet's save
    through ``super()`` at :360; a DER not operational in this window's year -- construction year, end of life --
    must not be saved, DERExtension.py:116-125) and each of those DERs' ``variables_dict``.  The reference loop
    saves each window right after its set-up, so this is the state its save sees."""
    if plan.active_ders is not None:
        scenario.poi.active_ders = list(plan.active_ders)
    for der, vd in plan.saved_vars.items():
        if vd is not None:
            der.variables_dict = vd


def _solve_plans(plans, solver):
    """One batched solve over the LP windows of `plans` (list of plan tuples); returns {index: WindowResult}."""
    lp_idx = [i for i, p in enumerate(plans) if p.win is not None]
    if not lp_idx:
        return {}
    own = solver is None
    solver = solver or BatchSolver(0)
    try:
        res = solver.solve([plans[i].win.lp for i in lp_idx])
    finally:
        if own:
            solver.close()
    return dict(zip(lp_idx, res))


def _save(scenario, plan, r, report, retry_failed=True):
    opt_period, sub_index, functions, constraints, _, win, _ = plan
    _restore_window_state(scenario, plan)  # before the in-place reference solves too
    if win is None:  # MILP / non-LP window: the reference solve, in place
        prob, obj, err = scenario.solve_optimization(functions, constraints)
        report.reference += 1
    elif retry_failed and r.status in RETRY_STATUSES:  # no certified optimum: the reference solve, in place
        prob, obj, err = scenario.solve_optimization(functions, constraints)
        report.retried += 1
        report.retried_status[r.status_name] = report.retried_status.get(r.status_name, 0) + 1
    else:
        prob, err = win.unpack(r)
        obj = functions
        report.gpu += 1
        report.relaxed += int(bool(getattr(win.ew, "relaxed", False)))
    scenario.save_optimization_results(opt_period, sub_index, prob, obj, err)


def batched_optimize_problem_loop(scenario, solver=None, exporter=None, relax_milp=False, retry_failed=True,
                                  **kwargs):
    """Batched ``MicrogridScenario.optimize_problem_loop`` (dervet/MicrogridScenario.py:281-320).  Returns the plan
    list; the window accounting is left on ``scenario.dervet_hip_report`` (a LoopReport)."""
    report = LoopReport()
    scenario.dervet_hip_report = report
    pre = _preamble(scenario)
    if pre is None:
        return None
    alpha, ignore = pre
    if not windows_are_independent(scenario):  # coupled windows: the reference loop, unchanged
        for opt_period in scenario.optimization_levels.predictive.unique():
            functions, constraints, sub_index = scenario.set_up_optimization(opt_period, annuity_scalar=alpha,
                                                                             ignore_der_costs=ignore)
            if not len(constraints) and not len(functions.values()):
                continue
            prob, obj, err = scenario.solve_optimization(functions, constraints)
            report.reference += 1
            scenario.save_optimization_results(opt_period, sub_index, prob, obj, err)
        return None
    exporter = exporter or CvxpyExporter(relax_milp)
    plan = [p for p in (_setup_export(scenario, w, alpha, ignore, exporter)
                        for w in scenario.optimization_levels.predictive.unique()) if p is not None]
    results = _solve_plans(plan, solver)
    for i, p in enumerate(plan):
        _save(scenario, p, results.get(i), report, retry_failed)
    return plan


def batched_cases_loop(scenarios, solver=None, exporter=None, relax_milp=False, retry_failed=True):
    """The optimize_problem_loop of several cases (dervet/DERVET.py:75-83) batched on the GPU.

    Independent cases (``windows_are_independent``) put all their windows into one batch.  Coupled cases
    (degradation / sizing) advance in lockstep: window position k of every coupled case is set up, solved in one
    batch and saved (so each case's degradation update runs) before any coupled case sets up position k + 1.
    Returns the plans per case, in case order; each case's accounting is on its ``dervet_hip_report``."""
    exporter = exporter or CvxpyExporter(relax_milp)
    own = solver is None
    solver = solver or BatchSolver(0)
    try:
        live, indep, coupled = [], [], []
        for s in scenarios:
            s.dervet_hip_report = LoopReport()
            pre = _preamble(s)
            if pre is None:
                live.append(None)
                continue
            live.append(pre)
            (indep if windows_are_independent(s) else coupled).append(len(live) - 1)
        plans = {i: [] for i in range(len(scenarios))}
        # every window of every independent case: one batch
        flat = []
        for i in indep:
            s = scenarios[i]
            alpha, ignore = live[i]
            for w in s.optimization_levels.predictive.unique():
                p = _setup_export(s, w, alpha, ignore, exporter)
                if p is not None:
                    flat.append((i, p))
        res = _solve_plans([p for _, p in flat], solver)
        for k, (i, p) in enumerate(flat):
            _save(scenarios[i], p, res.get(k), scenarios[i].dervet_hip_report, retry_failed)
            plans[i].append(p)
        # coupled cases: window position by window position across the cases
        periods = {i: list(scenarios[i].optimization_levels.predictive.unique()) for i in coupled}
        for pos in range(max((len(v) for v in periods.values()), default=0)):
            step = []
            for i in coupled:
                if pos < len(periods[i]):
                    alpha, ignore = live[i]
                    p = _setup_export(scenarios[i], periods[i][pos], alpha, ignore, exporter)
                    if p is not None:
                        step.append((i, p))
            res = _solve_plans([p for _, p in step], solver)
            for k, (i, p) in enumerate(step):
                _save(scenarios[i], p, res.get(k), scenarios[i].dervet_hip_report, retry_failed)
                plans[i].append(p)
        return [plans[i] for i in range(len(scenarios))]
    finally:
        if own:
            solver.close()


def make_batched_scenario_class(base, solver_factory=None, relax_milp=False, retry_failed=True, exporter_factory=None):
    """Subclass of the reference ``MicrogridScenario`` whose window loop is batched on the GPU."""

    class BatchedMicrogridScenario(base):
        def optimize_problem_loop(self, **kwargs):
            solver = solver_factory() if solver_factory else None
            exporter = exporter_factory() if exporter_factory else None
            try:
                return batched_optimize_problem_loop(self, solver=solver, exporter=exporter, relax_milp=relax_milp,
                                                     retry_failed=retry_failed, **kwargs)
            finally:
                if solver is not None:
                    solver.close()

    BatchedMicrogridScenario.__name__ = "BatchedMicrogridScenario"
    BatchedMicrogridScenario.dervet_hip_options = (solver_factory, bool(relax_milp), bool(retry_failed))
    return BatchedMicrogridScenario


def make_batched_dervet_solve(dervet_module, solver_factory=None, relax_milp=False, retry_failed=True,
                              case_batch=None, exporter_factory=None):
    """``DERVET.solve`` (dervet/DERVET.py:72-90) with every case's windows in one batched solve.

    The reference runs its cases one after the other -- preamble, ``optimize_problem_loop``, ``add_instance`` --
    so the GPU would see one case's 12-36 windows per call (DERVET.py:75-83).  This version runs each case's
    unchanged preamble (``MicrogridScenario(value)``, ``set_up_poi_and_service_aggregator``, ``initialize_cba``,
    ``fill_and_drop_extra_data``, ``sizing_module``: :76-80), then ``batched_cases_loop`` over the cases
    (independent cases: every window of every case in one solve; degradation / sizing-coupled cases in lockstep by
    window position), then ``MicrogridResult.add_instance(key, run)`` in the reference's key order and
    ``sensitivity_summary()`` (:83-85).  ``case_batch`` bounds how many cases are held at once (None: all); the
    scenarios of one batch are alive together, which is the memory this costs over the serial loop.  A case's
    results are handed to ``add_instance`` after the batch is solved instead of right after its own loop; each
    ``MicrogridResult`` instance is built from its own scenario object, so what it reads is the same."""
    mod = dervet_module

    def solve(self):
        starts = time.time()
        keys = list(self.cases.keys())
        step = len(keys) if not case_batch else int(case_batch)
        for lo in range(0, len(keys), max(step, 1)):
            chunk = keys[lo:lo + max(step, 1)]
            runs = []
            for key in chunk:
                run = mod.MicrogridScenario(self.cases[key])
                run.set_up_poi_and_service_aggregator()
                run.initialize_cba()
                run.fill_and_drop_extra_data()
                run.sizing_module()
                runs.append(run)
            solver = solver_factory() if solver_factory else None
            exporter = exporter_factory() if exporter_factory else None
            try:
                batched_cases_loop(runs, solver=solver, exporter=exporter, relax_milp=relax_milp,
                                   retry_failed=retry_failed)
            finally:
                if solver is not None:
                    solver.close()
            for key, run in zip(chunk, runs):
                mod.MicrogridResult.add_instance(key, run)
        mod.MicrogridResult.sensitivity_summary()
        tell = getattr(mod, "TellUser", None)
        if tell is not None:
            tell.info(f"DERVET runtime: {time.time() - starts}")
        return mod.MicrogridResult

    solve.dervet_hip_batched = True
    return solve


def install(dervet_module=None, relax_milp=False, retry_failed=True, solver_factory=None, batch_cases=False,
            case_batch=None, exporter_factory=None):
    """Patch dervet.DERVET.MicrogridScenario (hard-coded at dervet/DERVET.py:76) with the batched class.
    ``relax_milp``: the user's opt-in to GPU LP relaxations of binary = 1 windows (north_star); off, MILP windows stay
    on the reference solve.  ``retry_failed``: re-solve windows without a certified GPU optimum by the reference.
    ``batch_cases``: also patch ``DERVET.solve`` (DERVET.py:72-90) so that every case's windows go to the GPU
    together (``make_batched_dervet_solve``; ``case_batch`` cases at a time); off, the reference's serial case loop
    is kept (and a previous ``batch_cases`` install is undone)."""
    if dervet_module is None:
        import dervet.DERVET as dervet_module  # noqa: N813
    base = dervet_module.MicrogridScenario
    if getattr(base, "__name__", "") == "BatchedMicrogridScenario":
        if base.dervet_hip_options == (solver_factory, bool(relax_milp), bool(retry_failed)):
            cls = base
        else:
            base = base.__bases__[0]  # re-install with the new options over the reference class
            cls = None
    else:
        cls = None
    if cls is None:
        cls = make_batched_scenario_class(base, solver_factory, relax_milp, retry_failed, exporter_factory)
        dervet_module.MicrogridScenario = cls
    driver = getattr(dervet_module, "DERVET", None)
    if driver is not None:
        if not hasattr(driver, "_dervet_hip_reference_solve"):
            driver._dervet_hip_reference_solve = driver.solve
        if batch_cases:
            driver.solve = make_batched_dervet_solve(dervet_module, solver_factory, relax_milp, retry_failed,
                                                     case_batch, exporter_factory)
        else:
            driver.solve = driver._dervet_hip_reference_solve
    return cls

"""Battery cycle / calendar degradation and the degradation-coupled window sweep (SURVEY.md 8b eligibility, 8e:
"with degradation on, windows of one scenario are solved as sequential batched steps").

DER-VET's Battery (dervet/MicrogridDER/Battery.py:69-110) degrades its energy capacity after every optimization
window through storagevet's BatteryTech degradation module (absent from the reference snapshot, so the model below
is a restatement of its published behaviour; parity UNPINNED):

  * calendar: yearly_degrade % per year, pro rata over the window's days (Model_Parameters_Template_DER.csv:63);
  * cycling (incl_cycle_degrade, :64): rainflow counting of the window's SOE profile (the `rainflow` 3.0.0 package,
    requirements.txt:22; ASTM E1049-85), each cycle's depth = range / rated energy looked up in the cycle-life
    table (data/battery_cycle_life.csv: "Cycle Depth Upper Limit", "Cycle Life Value" -- the first row whose upper
    limit is >= the depth), damage = sum of count / cycle life, scaled by the capacity the table's end-of-life
    condition stands for (1 - cycle_life_table_eol_condition / 100, :65);
  * degrade_perc accumulates; the effective energy capacity is rated x (1 - degrade_perc) (its SOE bounds and
    target follow); when it falls to state_of_health x rated (:90) a replaceable battery is reset to nameplate
    (Battery.py:100-110).

Window k of a scenario therefore depends on the dispatch of its windows 0..k-1, but scenarios are independent:
``DegradationSweep`` solves window position k of EVERY scenario in one batched GPU call, updates every scenario's
capacity from its solved SOE profile (vectorised across scenarios), and only then builds position k + 1 -- the
lockstep loop the drop-in runs for CVXPY windows (dropin.batched_cases_loop), here with the native builder.
"""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def cycle_life_table(path=None):
    """(upper limits, cycle life values) of a DER-VET cycle-life CSV (default: the reference's default table,
    data/battery_cycle_life.csv -- Model_Parameters_Template_DER.csv:66 -- shipped as dervet_hip/data/)."""
    if path is None:
        path = os.path.join(HERE, "data", "battery_cycle_life.csv")
    d = np.loadtxt(path, delimiter=",", skiprows=1)
    return d[:, 0].copy(), d[:, 1].copy()


def _life(depth, upper, life):
    idx = np.minimum(np.searchsorted(upper, depth, side="left"), len(upper) - 1)
    return life[idx]


def cycle_damage(ene, e_rated, upper, life):
    """Sum over rainflow cycles of count / cycle_life(range / e_rated) for every row of ene [S, T] (SOE profiles,
    kWh), cycles taken in extraction order (oracle/rainflow_ref.py restates the counting scalar-wise).  All rows are
    counted in lock step: one pass over the T columns with per-row stacks."""
    x = np.asarray(ene, np.float64)
    S, T = x.shape
    e_rated = np.broadcast_to(np.asarray(e_rated, np.float64), (S,))
    dmg = np.zeros(S)
    if T < 2:
        return dmg
    rows = np.arange(S)
    stack = np.empty((S, T + 1))
    base = np.zeros(S, np.int64)   # first live stack slot (half cycles drop the first point)
    top = np.zeros(S, np.int64)    # one past the last

    def add(mask, rng, count):
        dmg[mask] += count / _life(rng / e_rated[mask], upper, life)

    def emit(mask, vals):
        """Push vals (rows in mask) and apply the three-point rule until it stops for every row."""
        r = rows[mask]
        stack[r, top[r]] = vals
        top[r] += 1
        act = r
        while len(act):
            act = act[top[act] - base[act] >= 3]
            if not len(act):
                break
            t = top[act]
            X = np.abs(stack[act, t - 1] - stack[act, t - 2])
            Y = np.abs(stack[act, t - 2] - stack[act, t - 3])
            go = X >= Y
            act, t, Y = act[go], t[go], Y[go]
            if not len(act):
                break
            half = (t - base[act]) == 3
            m = np.zeros(S, bool)
            m[act[half]] = True
            if half.any():
                add(m, Y[half], 0.5)
                base[act[half]] += 1
            full = ~half
            if full.any():
                f = act[full]
                m[:] = False
                m[f] = True
                add(m, Y[full], 1.0)
                tf = top[f]
                stack[f, tf - 3] = stack[f, tf - 1]
                top[f] -= 2

    # reversals, streamed: the first point, every confirmed turning point, the last point
    emit(np.ones(S, bool), x[:, 0])
    cur = x[:, 1].copy()
    d_last = cur - x[:, 0]
    for j in range(2, T):
        xn = x[:, j]
        active = xn != cur
        d = xn - cur
        rev = active & (d_last * d < 0)
        if rev.any():
            emit(rev, cur[rev])
        cur = np.where(active, xn, cur)
        d_last = np.where(active, d, d_last)
    emit(np.ones(S, bool), x[:, T - 1])
    # what is left on the stacks: half cycles, in order
    span = top - base
    for k in range(int(span.max()) - 1):
        m = span - 1 > k
        if not m.any():
            break
        r = rows[m]
        rng = np.abs(stack[r, base[r] + k + 1] - stack[r, base[r] + k])
        add(m, rng, 0.5)
    return dmg


class Degradation:
    """Degradation state of S batteries (vectorised).

    incl_cycle_degrade = False turns the whole module off, calendar loss included: dervet gates the degradation
    calls on it (Battery.py:82, :101), and the reference's own test pins it -- 041-no_Degradation_Test_MP.csv has
    yearly_degrade = 10 with incl_cycle_degrade = 0 and test_2finances.py:102-104 asserts the 2017 and 2022
    avoided energy charges are equal (tests/test_degradation_ref.py)."""

    def __init__(self, e_rated, yearly_degrade=0.0, incl_cycle_degrade=True, table=None, eol_condition=80.0,
                 state_of_health=73.0, replaceable=True):
        self.e_rated = np.asarray(e_rated, np.float64).copy()
        S = len(self.e_rated)
        self.yearly = np.broadcast_to(np.asarray(yearly_degrade, np.float64), (S,)).copy()
        self.cycle = bool(incl_cycle_degrade)
        self.upper, self.life = table if table is not None else cycle_life_table()
        self.eol = float(eol_condition)
        self.soh = np.broadcast_to(np.asarray(state_of_health, np.float64), (S,)).copy() / 100.0
        self.replaceable = np.broadcast_to(np.asarray(replaceable, bool), (S,)).copy()
        self.degrade_perc = np.zeros(S)
        self.replacements = np.zeros(S, np.int64)
        self.skipped = np.zeros(S, np.int64)  # windows whose dispatch was not used (status not OPTIMAL)
        self.years_degraded = [set() for _ in range(S)]  # Battery.py:104 years_system_degraded

    def capacity(self):
        """Effective energy capacity (kWh) the next window is built with."""
        return np.maximum(self.e_rated * (1.0 - self.degrade_perc), 0.0)

    def age(self, days):
        """Calendar loss only, e.g. from the operation year's start to the first window (Battery.py:84-85)."""
        if self.cycle and days > 0:
            self.degrade_perc += self.yearly / 100.0 * (days / 365.0)

    def update(self, ene, days, valid=None, year=None):
        """After a window of `days` days with SOE profiles ene [S, T]: returns this window's degradation [S].
        valid [S] (default all): rows whose dispatch is usable; the others take the calendar loss only (a window
        that is infeasible or failed numerically has no SOE profile to count) and are counted in ``skipped``.
        year: the window's first year, recorded when a battery reaches its state of health (Battery.py:102-104)."""
        S = len(self.e_rated)
        if not self.cycle:
            return np.zeros(S)
        d = self.yearly / 100.0 * (days / 365.0)
        ok = np.ones(S, bool) if valid is None else np.asarray(valid, bool)
        if ok.any():
            cyc = np.zeros(S)
            cyc[ok] = cycle_damage(np.asarray(ene)[ok], self.e_rated[ok], self.upper, self.life)
            d = d + cyc * (1.0 - self.eol / 100.0)
        self.skipped += ~ok
        self.degrade_perc += d
        reached = self.capacity() <= self.e_rated * self.soh
        if year is not None:
            for i in np.nonzero(reached)[0]:
                self.years_degraded[i].add(int(year))
        worn = reached & self.replaceable
        self.degrade_perc[worn] = 0.0
        self.replacements += worn
        return d


class DegradationSweep:
    """Window positions solved in order, every scenario's window of a position in one batched solve.

    build(k, capacity [S]) -> list of WindowGroup for window position k (the scenarios' windows, in scenario order,
    e.g. ``lambda k, E: scenarios.config4(ids, E=E, only=[k])``); positions: the window ids in time order; dt: hours
    per step."""

    def __init__(self, build, positions, degradation, dt=1.0, builder=None, years=None):
        self.build, self.positions, self.deg, self.dt = build, list(positions), degradation, float(dt)
        self.builder = builder
        self.years = years  # position -> the window's first year (replacement years, Battery.py:104), optional

    def run(self, solver, device="cuda:0"):
        """Returns per position {k, iters [S], status [S], obj [S], degradation [S], capacity_before [S], ene [S, T],
        x (each window's primal solution)}.
        A solver with ``solve_packed`` (BatchSolver) gets the position's batch resident in HBM; any other solver
        with ``solve(lps)`` (e.g. the CPU restatement) gets WindowLPs.  When build returns device-builder specs
        (``scenarios.config4(..., spec=True)``) the windows are expanded on the GPU (lp/gpu_builder.py; ``builder``
        then names the BatchSolver whose handle builds them, default: solver)."""
        from .lp import builder, gpu_builder
        out = []
        for k in self.positions:
            cap = self.deg.capacity()
            groups = self.build(k, cap)
            if hasattr(solver, "solve_packed") and device is not None:
                import torch
                if groups and isinstance(groups[0], gpu_builder.BatteryGroupSpec):
                    dev = gpu_builder.pack_specs_device(groups, self.builder or solver, device)
                    d = gpu_builder.desc_of(groups)[0]
                else:
                    pb = builder.pack_groups(groups)
                    dev = pb.to_torch(device).alloc_outputs()
                    d = np.asarray(pb.desc)
                solver.solve_packed(dev)
                torch.cuda.synchronize()
                x = dev.x.cpu().numpy()
                ist = dev.istats.cpu().numpy()
                obj = dev.stats.cpu().numpy()[:, 0]
                del dev
                T = int(d[0, 2]) - 1
                ene = np.stack([x[int(r[6]) + 2 * T:int(r[6]) + 3 * T] for r in d])
                xs = [x[int(r[6]):int(r[6]) + int(r[0])] for r in d]
            else:
                lps = [lp for g in groups for lp in builder.group_window_lps(g)]
                res = solver.solve(lps)
                ist = np.array([[r.status, r.iters] for r in res])
                obj = np.array([r.obj for r in res])
                T = lps[0].m_eq - 1
                ene = np.stack([r.x[2 * T:3 * T] for r in res])
                xs = [np.asarray(r.x) for r in res]
            # only OPTIMAL dispatch is counted (an infeasible window's x is no SOE profile; VERDICT r04:
            # nor is an ITER_LIMIT one, which failed the KKT test) -- the others are counted in Degradation.skipped
            valid = ist[:, 0] == 0
            if not valid.all():  #  a skipped window gets calendar loss only: say so, it biases wear low
                import warnings
                warnings.warn(f"degradation sweep, window position {k}: {int((~valid).sum())} of {len(valid)} windows "
                              f"not OPTIMAL (statuses {sorted(set(int(v) for v in ist[~valid, 0]))}); their cycle wear "
                              "is not counted (Degradation.skipped)", RuntimeWarning, stacklevel=2)
            deg = self.deg.update(ene, T * self.dt / 24.0, valid=valid,
                                  year=None if self.years is None else self.years[k])
            out.append(dict(k=k, iters=ist[:, 1], status=ist[:, 0], obj=obj, degradation=deg, capacity_before=cap,
                            ene=ene, x=xs))
        return out

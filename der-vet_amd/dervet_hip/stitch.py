"""Coarse-to-fine start for one long window (BASELINE config 3: the 5-minute annual window, T = 105,120).

The long window goes to the grid-wide large-LP path, whose PDHG needs tens of thousands of iterations from a
cold start.  Its sub-windows (e.g. the 365 days of the year, each returning to the SOE target) are small
battery windows that the batched band kernel solves together in a few milliseconds, and their solutions
concatenated are a feasible, near-optimal point of the long window (it only drops the end-of-sub-window SOE
targets).  Monthly sub-windows (the long window's own demand-charge periods) carry their DCM epigraph duals over too:
the long window's DCM row of step t for its k-th charge covering t starts from the sub-window's row of the same step
and rank.  ``solve_stitched`` solves the sub-windows as one batch, stitches their primal and dual solutions
into the long window's layout and starts the long window from there (``dvh_options.warm_start``).

Layout (lp/builder.py battery_group): x = [ch (T), dis (T), ene (T), tau (J)]; rows
0 (ene_0 = target), 1..T-1 (SOE recurrence of step t-1), T (last step back to target), then the >= rows
(DCM epigraph: tau_j - net_t >= base_t).  Sub-window s covering steps [a, a + T_s) maps its rows 1..T_s - 1
onto the long window's rows a + 1 .. a + T_s - 1 and its final row onto row a + T_s (the recurrence across
the boundary, or the final row for the last sub-window).  tau_j is set to the smallest value its >= rows allow
at the stitched (ch, dis); the DCM duals start from the sub-windows' duals of the same (step, charge rank) rows where
a sub-window has them (monthly sub-windows), else at zero.
"""
import numpy as np


def _check_battery(g):
    if g.G != 1:
        raise ValueError("stitching works on single-window groups")
    if g.n != 3 * g.T + g.J or g.m_eq != g.T + 1:
        raise ValueError(f"not a battery (+ DCM) window layout: n={g.n}, m_eq={g.m_eq}, T={g.T}, J={g.J}")


def _dcm_rows(g):
    """(step t, rank k among the DCM rows of step t, row index) of every DCM epigraph row of window group g: the >= rows
    whose entries are ch_t, dis_t and one tau column (builder.battery_group's first >= block)."""
    T, out, seen = g.T, [], {}
    if not g.J:
        return out
    for r in range(g.m_eq, g.m):
        cols = g.indices[g.indptr[r]:g.indptr[r + 1]]
        if len(cols) < 3 or not (cols[0] < T and T <= cols[1] < 2 * T and 3 * T <= cols[2] < 3 * T + g.J):
            break
        t = int(cols[0])
        k = seen.get(t, 0)
        seen[t] = k + 1
        out.append((t, k, r))
    return out


def stitched_start(long, subs, sub_x, sub_y, dcm_duals=False):
    """Starting point (x0, y0) of the long window `long` (WindowGroup, G = 1) from the solutions (sub_x[s],
    sub_y[s]) of its consecutive sub-windows `subs` (WindowGroups, G = 1, covering the long window's steps
    in order)."""
    import scipy.sparse as sp
    _check_battery(long)
    T = long.T
    if sum(g.T for g in subs) != T:
        raise ValueError("sub-windows do not cover the long window")
    x0 = np.zeros(long.n)
    y0 = np.zeros(long.m)
    a = 0
    for s, g in enumerate(subs):
        _check_battery(g)
        Ts = g.T
        xs, ys = np.asarray(sub_x[s], np.float64), np.asarray(sub_y[s], np.float64)
        for blk in range(3):  # ch, dis, ene
            x0[blk * T + a: blk * T + a + Ts] = xs[blk * Ts: blk * Ts + Ts]
        if s == 0:
            y0[0] = ys[0]
        y0[a + 1: a + Ts] = ys[1: Ts]
        y0[a + Ts] = ys[Ts]
        a += Ts
    if long.J and dcm_duals:
        # DCM duals: rows of the long window keyed by (global step, rank of the charge among those covering it).  The
        # rank identifies a charge only where both windows cover the step with the same number of charges (ADVICE r05:
        # an extra or missing charge would shift the ranks); a step where the counts differ starts from 0 instead.
        sub_dual, sub_count = {}, {}
        a = 0
        for s, g in enumerate(subs):
            ys = np.asarray(sub_y[s], np.float64)
            for t, k, r in _dcm_rows(g):
                sub_dual[(a + t, k)] = ys[r]
                sub_count[a + t] = sub_count.get(a + t, 0) + 1
            a += g.T
        long_rows = list(_dcm_rows(long))
        long_count = {}
        for t, _, _ in long_rows:
            long_count[t] = long_count.get(t, 0) + 1
        for t, k, r in long_rows:
            y0[r] = sub_dual.get((t, k), 0.0) if sub_count.get(t, 0) == long_count[t] else 0.0
    if long.J:
        K = sp.csr_matrix((long.data[0], long.indices, long.indptr), shape=(long.m, long.n))
        ge = K[long.m_eq:]
        rest = ge[:, :3 * T] @ x0[:3 * T]
        tc = ge[:, 3 * T:].tocoo()
        need = (long.q[0, long.m_eq:][tc.row] - rest[tc.row]) / tc.data
        tau = np.full(long.J, -np.inf)
        np.maximum.at(tau, tc.col, need)
        tau[~np.isfinite(tau)] = 0.0
        x0[3 * T:] = np.clip(tau, long.l[0, 3 * T:], long.u[0, 3 * T:])
    return x0, y0


def solve_stitched(solver, long, subs, dcm_duals=False):
    """Solve the long window from the stitched solution of its sub-windows.  Returns (result of the long
    window, results of the sub-windows, {"subs_ms", "long_ms"} kernel times)."""
    from .lp import builder
    lps = [builder.group_window_lps(g)[0] for g in subs]
    sres = solver.solve(lps)
    subs_ms = solver.timing()["total_ms"]
    x0, y0 = stitched_start(long, subs, [r.x for r in sres], [r.y for r in sres], dcm_duals)
    w0 = solver.options().warm_start
    solver.set_options(warm_start=1)
    try:
        res = solver.solve([builder.group_window_lps(long)[0]], start=[(x0, y0)])[0]
    finally:
        solver.set_options(warm_start=w0)
    return res, sres, {"subs_ms": subs_ms, "long_ms": solver.timing()["total_ms"]}

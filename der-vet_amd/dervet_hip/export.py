"""ECOS-form window export -> canonical dvh LP, and the way back (SURVEY.md section 8b, Appendix A last bullet).

The reference solves each window with ``cvx.Problem(Minimize(sum(functions)), constraints).solve()`` inside
storagevet ``Scenario.solve_optimization`` (called at dervet/MicrogridScenario.py:319).  CVXPY 1.0.31
(requirements.txt:2) canonicalises that problem for ECOS as

    min c'x + offset   s.t.   A x = b,   G x + s = h,  s >= 0          (``prob.get_problem_data(cvx.ECOS)``)

with every variable bound written as a G row, the battery's reservation columns (uch / udis / uene) pinned to
zero by equality rows, the SOE start ``ene[0] = target`` a one-entry equality row and the DCM ``max`` an epigraph
column of CVXPY's own.  Solved as is, such a window is a generic CSR LP with ~3T one-entry rows.

``ecos_to_window`` turns it into the solver's canonical form (include/dervet_hip.h) in two steps:

1. presolve (exact): one-entry G rows become column bounds (the tightest kept, its row remembered), one-entry
   A rows fix their column, fixed columns are substituted out (rhs and objective offset), rows left without a
   free column are checked and dropped; repeated until nothing changes.
2. band canonicalisation: if what is left is the battery (+ DCM) window -- equality rows forming one chain over
   the SOE columns (each in two of them), two more columns per chain row (ch / dis, lower bound 0), >= rows of
   (ch_t, dis_t, tau_j) with free tau columns -- the columns and rows are permuted into the layout the
   battery-banded kernel verifies on the device (dvh_band.hip): x = [ch(T), dis(T), ene(T), tau(J)], row 0
   ``ene_0 = target``, rows 1..T the SOE chain, then the DCM rows.  The chain's first SOE column was fixed by the
   start row and substituted out in step 1; it is put back (column + its one-entry row) so the chain has its
   initial row.  Either end of the chain may serve as the start (the LP is the same up to relabelling the steps);
   the end whose original row held the pinned column of largest |value| is taken.  A window of any other shape
   keeps the presolved generic form (ELL / generic kernels).

Mixed-integer windows (binary = 1, ``Model_Parameters_Template_DER.csv:17``: boolean ``on_c`` / ``on_d`` / ICE ``on``
variables, ``ElectricVehicles.py:120-122``) are exported through CVXPY's ``get_problem_data(cvx.ECOS_BB)``, whose data
dict carries ``bool_vars_idx`` / ``int_vars_idx`` (the column of every boolean / integer entry).  They are refused
(``ExportError``: the reference solve, in place) unless the caller opts in with ``relax=True``; then integrality is
dropped, every boolean column gets the box [0, 1] (intersected with any bound rows), integer columns keep their
rows' bounds, and the window is the MILP's LP relaxation -- a lower bound on the reference's MILP objective.

``ExportedWindow.ecos_solution(result)`` maps a solver result back to the dict ECOS returns ({x, y, z, s, info}),
which CVXPY's ECOS ``invert`` / ``Problem.unpack_results`` consume: x in the original column order (fixed columns
at their values); ECOS duals from the solver's (c - K'y - lambda = 0 with K = [A; -G]): y_ECOS = -y_E, z = y_I for
kept rows, and for one-entry rows the part of the column's reduced cost that ECOS's stationarity
c + A'y + G'z = 0 leaves to them; ``info`` with exitFlag / pcost (without the offset, which ``invert`` adds) /
dcost / iter / timing as ECOS 2.0.7 fills it.
"""
from dataclasses import dataclass, field

import numpy as np
import scipy.sparse as sp

from . import _lib
from .solver import WindowLP

# dvh status -> ECOS 2.0.7 exitFlag (ECOS_OPTIMAL 0, ECOS_PINF 1, ECOS_DINF 2, ECOS_INACC_OFFSET + 0 = 10 "optimal
# inaccurate", ECOS_NUMERICS -4); CVXPY 1.0.31 maps 0 -> optimal, 1 -> infeasible, 2 -> unbounded,
# 10 -> optimal_inaccurate, negative -> solver_error
EXIT_FLAG = {_lib.OPTIMAL: 0, _lib.PRIMAL_INFEASIBLE: 1, _lib.DUAL_INFEASIBLE: 2, _lib.ITER_LIMIT: 10,
             _lib.NUMERICAL: -4}
SOLUTION_PRESENT = (_lib.OPTIMAL, _lib.ITER_LIMIT)
KIND_A, KIND_G, KIND_ADDED = 0, 1, 2


class ExportError(ValueError):
    """The exported problem is not a window LP the solver takes (the window falls back to the reference solve)."""


def _dims_nonneg(dims, n_g):
    """Checks that every G row is in the nonnegative cone (an LP): no second-order or exponential cones."""
    if dims is None:
        return
    get = (lambda k: dims.get(k)) if isinstance(dims, dict) else (lambda k: getattr(dims, k, None))
    soc = get("q") if get("q") is not None else (get("soc") or [])
    exp = get("e") if get("e") is not None else (get("exp") or 0)
    if len(soc) or exp:
        raise ExportError("not an LP (second-order or exponential cone rows)")
    lin = get("l") if get("l") is not None else get("nonpos")
    if lin is not None and int(lin) != n_g:
        raise ExportError("G rows outside the nonnegative cone")


@dataclass
class ExportedWindow:
    """One window: the canonical LP handed to the solver and the maps back to the ECOS form."""
    lp: WindowLP
    c: np.ndarray               # ECOS objective (without offset)
    offset: float
    A: sp.csr_matrix
    b: np.ndarray
    G: sp.csr_matrix
    h: np.ndarray
    col_src: np.ndarray         # ECOS column of each LP column (-1: an added neutral column)
    row_kind: np.ndarray        # KIND_A: ECOS A row; KIND_G: ECOS G row (the LP >= row is -G); KIND_ADDED: added row
    row_src: np.ndarray         # ECOS row of each LP row (-1 for KIND_ADDED)
    fixed_val: np.ndarray       # value of each ECOS column the presolve substituted out (NaN: in the LP)
    pin_row: np.ndarray         # A row that fixed the column (-1: none)
    lb_row: np.ndarray          # one-entry G row of the column's tightest lower bound (-1: none)
    ub_row: np.ndarray          # ... upper bound
    banded: bool
    meta: dict = field(default_factory=dict)

    @property
    def n(self):
        return len(self.c)

    @property
    def relaxed(self):
        """True for the LP relaxation of a mixed-integer window (``ecos_to_window(..., relax=True)``)."""
        return bool(self.meta.get("relaxed_bool", 0) or self.meta.get("relaxed_int", 0))

    def x_full(self, x):
        """LP solution -> ECOS column order (substituted columns at their values)."""
        out = np.where(np.isnan(self.fixed_val), 0.0, self.fixed_val)
        ok = self.col_src >= 0
        out[self.col_src[ok]] = np.asarray(x)[ok]
        return out

    def duals(self, y):
        """LP duals (dvh convention) -> ECOS (y, z).  A relaxed boolean column's [0, 1] box has no ECOS row: what
        its multiplier carries is dropped (CVXPY reports no duals for a mixed-integer problem anyway)."""
        ya = np.zeros(self.A.shape[0])
        z = np.zeros(self.G.shape[0])
        y = np.asarray(y)
        k = self.row_kind
        ya[self.row_src[k == KIND_A]] = -y[k == KIND_A]
        z[self.row_src[k == KIND_G]] = np.maximum(y[k == KIND_G], 0.0)
        # rows the presolve took out: ECOS stationarity c + A'y + G'z = 0, column by column; what the kept rows
        # leave of it (the column's reduced cost) goes to the column's pin row, else to its active bound row
        rho = self.c + self.A.T @ ya + self.G.T @ z
        for j in np.nonzero(self.pin_row >= 0)[0]:
            r = self.pin_row[j]
            ya[r] -= rho[j] / self.A[r, j]
            rho[j] = 0.0
        for side, rows in ((rho < 0.0, self.ub_row), (rho > 0.0, self.lb_row)):
            for j in np.nonzero(side & (rows >= 0))[0]:
                r = rows[j]
                z[r] = max(z[r] - rho[j] / self.G[r, j], 0.0)
        return ya, z

    def ecos_solution(self, res, setup_s=0.0, solve_s=0.0):
        """The dict ``ecos.solve`` returns for this window, from a solver.WindowResult."""
        info = {"exitFlag": EXIT_FLAG.get(res.status, -4), "iter": int(res.iters),
                "infostring": f"dervet_hip: {res.status_name}",
                "timing": {"runtime": float(setup_s + solve_s), "tsetup": float(setup_s), "tsolve": float(solve_s)},
                "pres": float(res.primal_res_rel), "dres": float(res.dual_res_rel), "gap": float(res.gap_rel),
                "pinf": int(res.status == _lib.PRIMAL_INFEASIBLE), "dinf": int(res.status == _lib.DUAL_INFEASIBLE)}
        x = self.x_full(res.x)
        ya, z = self.duals(res.y)
        info["pcost"] = float(self.c @ x)                  # ECOS's objective excludes the offset (invert adds it)
        info["dcost"] = float(-self.b @ ya - self.h @ z)
        return {"x": x, "y": ya, "z": z, "s": self.h - self.G @ x, "info": info}


def _csr(M, n):
    if M is None:
        return sp.csr_matrix((0, n))
    M = sp.csr_matrix(M, dtype=np.float64)
    M.sum_duplicates()
    M.eliminate_zeros()
    M.sort_indices()
    return M


class _Presolved:
    pass


def presolve(c, offset, A, b, G, h, tol=1e-9, lo0=None, hi0=None):
    """Step 1 of the module docstring.  Returns a _Presolved with the reduced LP pieces and the maps.  ``lo0`` /
    ``hi0``: column bounds known before the rows are read (the [0, 1] box of a relaxed boolean column); a bound row
    replaces them only where it is tighter."""
    n = len(c)
    P = _Presolved()
    lo = np.full(n, -np.inf) if lo0 is None else np.array(lo0, np.float64)
    hi = np.full(n, np.inf) if hi0 is None else np.array(hi0, np.float64)
    lb_row, ub_row, pin_row = np.full(n, -1), np.full(n, -1), np.full(n, -1)
    fixed = np.full(n, np.nan)
    keep_a, keep_g = np.ones(A.shape[0], bool), np.ones(G.shape[0], bool)
    Ac, Gc = A.tocsc(), G.tocsc()
    ra, rg = b.copy(), h.copy()          # right-hand sides with the substituted columns moved over
    c0 = float(offset)
    scale = 1.0 + max(np.abs(b).max(initial=0.0), np.abs(h).max(initial=0.0))
    row_a = np.repeat(np.arange(A.shape[0]), np.diff(A.indptr))
    row_g = np.repeat(np.arange(G.shape[0]), np.diff(G.indptr))

    def fix(j, v):
        nonlocal c0
        fixed[j] = v
        c0 += c[j] * v
        for M, rhs in ((Ac, ra), (Gc, rg)):
            p0, p1 = M.indptr[j], M.indptr[j + 1]
            rhs[M.indices[p0:p1]] -= M.data[p0:p1] * v

    def live_entries(M, rows, keep):
        isfix = ~np.isnan(fixed)
        live = ~isfix[M.indices]
        cnt = np.bincount(rows[live], minlength=M.shape[0])
        return np.where(keep, cnt, -1), live

    changed = True
    while changed:
        changed = False
        for M, rows, keep, rhs, eq in ((A, row_a, keep_a, ra, True), (G, row_g, keep_g, rg, False)):
            cnt, _ = live_entries(M, rows, keep)
            for r in np.nonzero(cnt == 0)[0]:
                if (abs(rhs[r]) if eq else -rhs[r]) > tol * scale:
                    raise ExportError(f"infeasible ({'A' if eq else 'G'} row {r} left with rhs {rhs[r]:.3g})")
                keep[r] = False
                changed = True
        cnt, live = live_entries(A, row_a, keep_a)
        for r in np.nonzero(cnt == 1)[0]:
            p = np.arange(A.indptr[r], A.indptr[r + 1])
            p = p[live[p] & np.isnan(fixed[A.indices[p]])]
            if len(p) != 1:
                continue  # its column was fixed by an earlier row of this pass: checked next pass
            j = A.indices[p[0]]
            keep_a[r] = False
            pin_row[j] = r
            fix(j, ra[r] / A.data[p[0]])
            changed = True
        cnt, live = live_entries(G, row_g, keep_g)
        for r in np.nonzero(cnt == 1)[0]:
            p = np.arange(G.indptr[r], G.indptr[r + 1])
            p = p[live[p] & np.isnan(fixed[G.indices[p]])]
            if len(p) != 1:
                continue
            j, g = G.indices[p[0]], G.data[p[0]]
            v = rg[r] / g
            keep_g[r] = False
            if g > 0 and v < hi[j]:
                hi[j], ub_row[j] = v, r
            elif g < 0 and v > lo[j]:
                lo[j], lb_row[j] = v, r
            changed = True
        free = np.isnan(fixed)
        fin = np.isfinite(lo) & np.isfinite(hi)
        gap = np.where(fin, hi - lo, np.inf)
        for j in np.nonzero(free & fin & (gap <= tol * (1.0 + np.abs(np.where(fin, lo, 0.0)))))[0]:
            if hi[j] < lo[j] - tol * (1.0 + abs(lo[j])):
                raise ExportError(f"infeasible bounds on column {j}")
            fix(j, 0.5 * (lo[j] + hi[j]))
            changed = True
    isfix = ~np.isnan(fixed)
    bad = isfix & ((fixed < lo - tol * (1 + np.abs(lo))) | (fixed > hi + tol * (1 + np.abs(hi))))
    if bad.any():
        raise ExportError(f"fixed column {int(np.nonzero(bad)[0][0])} outside its bounds")
    live_cols = np.nonzero(~isfix)[0]
    if len(live_cols) == 0:
        raise ExportError("every column fixed by the presolve")
    ea, eg = np.nonzero(keep_a)[0], np.nonzero(keep_g)[0]
    P.K = sp.vstack([A[ea][:, live_cols], -G[eg][:, live_cols]]).tocsr()
    P.K.sort_indices()
    P.q = np.concatenate([ra[ea], -rg[eg]])
    P.m_eq = len(ea)
    P.kind = np.concatenate([np.full(len(ea), KIND_A), np.full(len(eg), KIND_G)]).astype(np.int64)
    P.src = np.concatenate([ea, eg]).astype(np.int64)
    P.cols, P.c0, P.lo, P.hi = live_cols, c0, lo, hi
    P.fixed, P.pin_row, P.lb_row, P.ub_row = fixed, pin_row, lb_row, ub_row
    return P


def integer_columns(data):
    """(boolean columns, integer columns) of an ECOS_BB data dict (empty for an ECOS one)."""
    def idx(key):
        v = data.get(key)
        return np.zeros(0, np.int64) if v is None else np.unique(np.asarray(v, np.int64).ravel())
    return idx("bool_vars_idx"), idx("int_vars_idx")


def ecos_to_window(data, tol=1e-9, band=True, relax=False):
    """CVXPY ECOS / ECOS_BB data dict {c, offset, A, b, G, h, dims[, bool_vars_idx, int_vars_idx]} of one window ->
    ExportedWindow.  A mixed-integer window raises ExportError unless ``relax`` (module docstring)."""
    c = np.asarray(data["c"], np.float64).ravel()
    n = len(c)
    A, G = _csr(data.get("A"), n), _csr(data.get("G"), n)
    b = np.zeros(A.shape[0]) if data.get("b") is None else np.asarray(data["b"], np.float64).ravel()
    h = np.zeros(G.shape[0]) if data.get("h") is None else np.asarray(data["h"], np.float64).ravel()
    _dims_nonneg(data.get("dims"), G.shape[0])
    offset = float(np.asarray(data.get("offset", 0.0), np.float64).ravel()[0]) if data.get("offset") is not None \
        else 0.0
    bools, ints = integer_columns(data)
    lo0 = hi0 = None
    if len(bools) or len(ints):
        if not relax:
            raise ExportError(f"mixed-integer window ({len(bools)} boolean, {len(ints)} integer columns): "
                              "the reference MILP solve (opt in to its LP relaxation with relax=True)")
        if (len(bools) and (bools.min() < 0 or bools.max() >= n)) or (len(ints) and (ints.min() < 0 or ints.max() >= n)):
            raise ExportError("integer column index outside the problem")
        lo0, hi0 = np.full(n, -np.inf), np.full(n, np.inf)
        lo0[bools], hi0[bools] = 0.0, 1.0
    P = presolve(c, offset, A, b, G, h, tol, lo0, hi0)
    base = dict(c=c, offset=offset, A=A, b=b, G=G, h=h, pin_row=P.pin_row, lb_row=P.lb_row, ub_row=P.ub_row,
                meta={"relaxed_bool": int(len(bools)), "relaxed_int": int(len(ints))})
    if band:
        w = _band(P, base)
        if w is not None:
            return w
    cl = P.cols
    lp = WindowLP.from_csr(P.K, P.q, c[cl], P.lo[cl], P.hi[cl], P.m_eq, P.c0)
    return ExportedWindow(lp=lp, col_src=cl, row_kind=P.kind, row_src=P.src, fixed_val=P.fixed, banded=False,
                          **base)


def _band(P, base):
    """Step 2 of the module docstring on the presolved LP, or None when it is not the battery (+ DCM) window."""
    K, q, m_eq = P.K, P.q, P.m_eq
    m, nl = K.shape
    if m_eq < 2:
        return None
    cl = P.cols
    lo, hi, c = P.lo[cl], P.hi[cl], base["c"][cl]
    E = K[:m_eq]
    deg_e = np.bincount(E.indices, minlength=nl)
    deg_i = np.bincount(K.indices[K.indptr[m_eq]:], minlength=nl)
    chain = deg_e == 2
    rows_of = [E.indices[E.indptr[r]:E.indptr[r + 1]] for r in range(m_eq)]
    nchain = np.array([int(chain[cols].sum()) for cols in rows_of])
    nside = np.array([int((deg_e[cols] == 1).sum()) for cols in rows_of])
    if not (np.all((nchain == 1) | (nchain == 2)) and np.all(nside == 2) and
            np.all(np.diff(E.indptr) == nchain + 2)):
        return None
    T = m_eq
    ends = np.nonzero(nchain == 1)[0]
    if len(ends) != 2 or int(chain.sum()) != T - 1:
        return None
    rows_in = [[] for _ in range(nl)]
    for r, cols in enumerate(rows_of):
        for j in cols[chain[cols]]:
            rows_in[j].append(r)
    # the column to restore before the first chain row: one the presolve fixed through a pin row, that sat in the
    # end row's original A row and in no other kept row
    A, Ac = base["A"], base["A"].tocsc()
    Gc = base["G"].tocsc()
    kept_a = set(P.src[P.kind == KIND_A].tolist())
    kept_g = set(P.src[P.kind == KIND_G].tolist())
    best = []
    for e in ends:
        r0 = int(P.src[e])
        for j in A.indices[A.indptr[r0]:A.indptr[r0 + 1]]:
            if np.isnan(P.fixed[j]) or P.pin_row[j] < 0:
                continue
            others = set(Ac.indices[Ac.indptr[j]:Ac.indptr[j + 1]].tolist()) & kept_a
            if others != {r0} or set(Gc.indices[Gc.indptr[j]:Gc.indptr[j + 1]].tolist()) & kept_g:
                continue
            best.append((-abs(P.fixed[j]), int(e), int(j)))
    if best:
        best.sort()
        _, start, restore = best[0]
    else:
        start, restore = int(ends[0]), -1
    # walk the chain
    order, ecols, sides = [], [], []
    r, prev = start, -1
    while True:
        cols = rows_of[r]
        order.append(r)
        sides.append(cols[deg_e[cols] == 1])
        nxt = [j for j in cols[chain[cols]] if j != prev]
        if len(order) == T:
            if nxt:
                return None
            break
        if len(nxt) != 1:
            return None
        j = nxt[0]
        ecols.append(j)
        r2 = [x for x in rows_in[j] if x != r]
        if len(r2) != 1:
            return None
        prev, r = j, r2[0]
    if len(set(order)) != T:
        return None
    # >= rows: (ch_t, dis_t, tau_j) with tau free and in no equality row; ch / dis with lower bound 0
    taus = np.nonzero((deg_e == 0) & np.isinf(lo) & np.isinf(hi))[0]
    if len(taus) > 4 or np.any((deg_e == 0) & ~np.isin(np.arange(nl), taus)) or np.any(deg_i[chain] > 0):
        return None
    step_of = np.full(nl, -1)
    for t, sc in enumerate(sides):
        step_of[sc] = t
    is_tau = np.zeros(nl, bool)
    is_tau[taus] = True
    mi = m - m_eq
    seen = np.zeros(T, bool)
    for i in range(m_eq, m):
        cols = K.indices[K.indptr[i]:K.indptr[i + 1]]
        if len(cols) != 3 or int(is_tau[cols].sum()) != 1:
            return None
        st = step_of[cols[~is_tau[cols]]]
        if len(st) != 2 or st[0] < 0 or st[0] != st[1] or seen[st[0]]:
            return None
        seen[st[0]] = True
    if mi > 0 and len(taus) == 0:
        return None
    ch = np.array([s[0] for s in sides])
    dis = np.array([s[1] for s in sides])
    if np.any(lo[ch] != 0.0) or np.any(lo[dis] != 0.0):
        return None
    # assemble [ch(T), dis(T), ene(T) = (restored, chain columns), tau(J)] x [init row, chain rows, >= rows]
    J = len(taus)
    n_b = 3 * T + J
    perm = np.concatenate([ch, dis, [-1], np.asarray(ecols, np.int64), taus]).astype(np.int64)
    inv = np.full(nl, -1)
    okp = perm >= 0
    inv[perm[okp]] = np.nonzero(okp)[0]
    j0 = 2 * T
    if restore >= 0:
        pr = int(P.pin_row[restore])
        v = float(P.fixed[restore])
        pin_coef = float(A[pr, restore])
        coef_first = float(A[int(P.src[start]), restore])
        init_rhs = float(base["b"][pr])
    else:  # no such column: a neutral column pinned to 0 by its own row
        pr, v, pin_coef, coef_first, init_rhs = -1, 0.0, 1.0, 1.0, 0.0
    rows_b, cols_b, vals_b, qb = [0], [j0], [pin_coef], [init_rhs]
    for k, r in enumerate(order):
        p0, p1 = K.indptr[r], K.indptr[r + 1]
        rows_b += [1 + k] * (p1 - p0)
        cols_b += inv[K.indices[p0:p1]].tolist()
        vals_b += K.data[p0:p1].tolist()
        qr = q[r]
        if k == 0:
            rows_b.append(1)
            cols_b.append(j0)
            vals_b.append(coef_first)
            qr += coef_first * v          # the substitution of the restored column, undone
        qb.append(qr)
    for k, i in enumerate(range(m_eq, m)):
        p0, p1 = K.indptr[i], K.indptr[i + 1]
        rows_b += [T + 1 + k] * (p1 - p0)
        cols_b += inv[K.indices[p0:p1]].tolist()
        vals_b += K.data[p0:p1].tolist()
        qb.append(q[i])
    Kb = sp.csr_matrix((vals_b, (rows_b, cols_b)), shape=(T + 1 + mi, n_b))
    cb, lb, ub = np.zeros(n_b), np.zeros(n_b), np.zeros(n_b)
    src = np.full(n_b, -1, np.int64)
    src[okp] = cl[perm[okp]]
    cb[okp], lb[okp], ub[okp] = c[perm[okp]], lo[perm[okp]], hi[perm[okp]]
    fixed = P.fixed.copy()
    c0 = P.c0
    if restore >= 0:
        src[j0] = restore
        cb[j0] = base["c"][restore]
        lb[j0], ub[j0] = P.lo[restore], P.hi[restore]   # its own bounds; the init row pins it
        c0 -= base["c"][restore] * v                     # its objective is back in c
        fixed[restore] = np.nan
    else:
        lb[j0], ub[j0] = -np.inf, np.inf
    kind = np.concatenate([[KIND_A if pr >= 0 else KIND_ADDED], P.kind[order], P.kind[m_eq:]]).astype(np.int64)
    rsrc = np.concatenate([[pr], P.src[order], P.src[m_eq:]]).astype(np.int64)
    pin_row = base["pin_row"].copy()
    if restore >= 0:
        pin_row[restore] = -1          # its pin row is the LP's init row now
    lp = WindowLP.from_csr(Kb, np.asarray(qb, np.float64), cb, lb, ub, T + 1, c0, structure=1)
    return ExportedWindow(lp=lp, col_src=src, row_kind=kind, row_src=rsrc, fixed_val=fixed, banded=True,
                          **dict(base, pin_row=pin_row, meta=dict(base["meta"], T=T, J=J, restored=restore)))

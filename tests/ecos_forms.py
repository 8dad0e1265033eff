"""Test infrastructure: window LPs in the form CVXPY 1.0.31 hands ECOS, and CVXPY's ECOS result inversion.

cvxpy / ecos / storagevet are absent here, so the export path is exercised on ECOS-shaped
data dicts written the way CVXPY would emit the storagevet battery window (parity unpinned against a live
CVXPY: the shape is restated, not captured):

  variables  ene, dis, ch, uene, udis, uch (T each; the reservation columns exist without markets, golden
             "Charge Option (kW)" ~ -7e-14 in timeseries_resultsuc3_es_step2.csv:2) and CVXPY's epigraph column
             of each DCM max, stacked in a shuffled block order (CVXPY orders by variable id)
  A rows     in storagevet's constraint order: the end-of-window row
             (target - ene[-1]) - dt rte ch[-1] + dt dis[-1] - uene[-1] + dt sdr ene[-1] = 0, the SOE recurrence
             ene[1:] - ene[:-1] - dt rte ch[:-1] + dt dis[:-1] - uene[:-1] + dt sdr ene[:-1] = 0, the start
             ene[0] = target, then the reservation pins uene = udis = uch = 0 (one-entry rows)
  G rows     every bound as a one-entry row (ene <= max, -ene <= -min, ch <= P_ch, -ch <= 0, dis, ...), then the
             DCM epigraph rows ch_t - dis_t - tau_j <= -(load - gen)_t
  offset     the constant part (fixed O&M, the retail charge of the uncontrollable load)

``invert`` restates CVXPY 1.0.31's ECOS ``invert`` (cvxpy/reductions/solvers/conic_solvers/ecos_conif.py) plus
``Problem.unpack_results``'s error check: the status from info['exitFlag'], solve / setup time from
info['timing'], the optimal value info['pcost'] + the offset, primal x and the duals y (A rows), z (G rows).
"""
import numpy as np
import scipy.sparse as sp

ECOS_STATUS = {0: "optimal", 1: "infeasible", 2: "unbounded", 10: "optimal_inaccurate",
               11: "infeasible_inaccurate", 12: "unbounded_inaccurate", -1: "solver_error", -2: "solver_error",
               -3: "solver_error", -4: "solver_error", -7: "solver_error"}
SOLUTION_PRESENT = ("optimal", "optimal_inaccurate")


class SolverError(Exception):
    pass


def invert(solution, offset):
    """CVXPY 1.0.31 ECOS.invert + unpack_results' error check -> dict(status, value, x, y, z, attr)."""
    info = solution["info"]
    status = ECOS_STATUS[info["exitFlag"]]
    attr = {"solve_time": info["timing"]["tsolve"], "setup_time": info["timing"]["tsetup"],
            "num_iters": info["iter"]}
    if status == "solver_error":
        raise SolverError("Solver 'ECOS' failed. Try another solver.")
    if status in SOLUTION_PRESENT:
        return dict(status=status, value=info["pcost"] + offset, x=np.asarray(solution["x"]),
                    y=np.asarray(solution["y"]), z=np.asarray(solution["z"]), attr=attr)
    return dict(status=status, value=np.inf if status.startswith("infeasible") else -np.inf, x=None, y=None, z=None,
                attr=attr)


def ecos_form(olp, dt, eta, sdr, target, seed=0, pins="rows"):
    """ECOS data dict of the oracle LP ``olp`` (oracle.window_lp.build, battery [+ DCM] window), and
    col[o] = ECOS column of oracle column o (layout [ch, dis, ene, tau])."""
    rng = np.random.default_rng(seed)
    T, J = olp["T"], olp["J"]
    blocks = [("ene", T), ("dis", T), ("ch", T), ("uene", T), ("udis", T), ("uch", T)] + \
             [(f"tau{j}", 1) for j in range(J)]
    order = rng.permutation(len(blocks))
    off, pos = {}, 0
    for k in order:
        name, size = blocks[k]
        off[name] = pos
        pos += size
    n = pos
    col = np.concatenate([off["ch"] + np.arange(T), off["dis"] + np.arange(T), off["ene"] + np.arange(T),
                          np.array([off[f"tau{j}"] for j in range(J)], np.int64)])
    ene, ch, dis, uene = (lambda t, k=k: off[k] + t for k in ("ene", "ch", "dis", "uene"))
    rows, cols, vals, b = [], [], [], []

    def row(entries, rhs):
        r = len(b)
        for cc, vv in entries:
            rows.append(r)
            cols.append(cc)
            vals.append(vv)
        b.append(rhs)

    k = T - 1
    row([(ene(k), -(1.0 - dt * sdr)), (ch(k), -dt * eta), (dis(k), dt), (uene(k), -1.0)], -target)
    for t in range(T - 1):
        row([(ene(t + 1), 1.0), (ene(t), -(1.0 - dt * sdr)), (ch(t), -dt * eta), (dis(t), dt), (uene(t), -1.0)], 0.0)
    row([(ene(0), 1.0)], target)
    if pins == "rows":
        for name in ("uene", "udis", "uch"):
            for t in range(T):
                row([(off[name] + t, 1.0)], 0.0)
    A = sp.csr_matrix((vals, (rows, cols)), shape=(len(b), n))
    rows, cols, vals, h = [], [], [], []

    def grow(entries, rhs):
        r = len(h)
        for cc, vv in entries:
            rows.append(r)
            cols.append(cc)
            vals.append(vv)
        h.append(rhs)

    lo, hi = olp["l"], olp["u"]
    for name, o in (("ene", 2 * T), ("ch", 0), ("dis", T)):
        for t in range(T):
            if np.isfinite(hi[o + t]):
                grow([(off[name] + t, 1.0)], hi[o + t])
            if np.isfinite(lo[o + t]):
                grow([(off[name] + t, -1.0)], -lo[o + t])
    if pins == "bounds":  # the reservation columns pinned through bounds instead (0 <= u <= 0)
        for name in ("uene", "udis", "uch"):
            for t in range(T):
                grow([(off[name] + t, 1.0)], 0.0)
                grow([(off[name] + t, -1.0)], 0.0)
    K, q, m_eq = olp["K"].tocsr(), olp["q"], olp["m_eq"]
    for i in range(m_eq, K.shape[0]):  # oracle >= row K_i x >= q_i  ->  -K_i x <= -q_i
        p0, p1 = K.indptr[i], K.indptr[i + 1]
        grow([(col[K.indices[p]], -K.data[p]) for p in range(p0, p1)], -q[i])
    G = sp.csr_matrix((vals, (rows, cols)), shape=(len(h), n))
    c = np.zeros(n)
    c[col] = olp["c"]
    data = {"c": c, "offset": float(olp["c0"]), "A": A.tocsc(), "b": np.asarray(b), "G": G.tocsc(),
            "h": np.asarray(h), "dims": {"l": len(h), "q": [], "e": 0}}
    return data, col


def highs_ecos(data):
    """Solve an ECOS data dict with HiGHS; returns (obj incl. offset, x, y_ecos, z) (ECOS dual convention
    c + A'y + G'z = 0, z >= 0)."""
    from scipy.optimize import linprog
    res = linprog(data["c"], A_ub=data["G"], b_ub=data["h"], A_eq=data["A"], b_eq=data["b"],
                  bounds=[(None, None)] * len(data["c"]), method="highs",
                  options={"primal_feasibility_tolerance": 1e-9, "dual_feasibility_tolerance": 1e-9})
    assert res.status == 0, res.message
    return res.fun + data["offset"], res.x, -res.eqlin.marginals, -res.ineqlin.marginals


def oracle_lp_of(lp):
    """solver.WindowLP in the builder / oracle band layout -> (oracle LP dict, dt, eta, sdr, target)."""
    T = lp.m_eq - 1
    K = sp.csr_matrix((lp.data, lp.indices, lp.indptr), shape=(lp.m, lp.n))
    p = lp.indptr[T]  # final row: dt eta ch, -dt dis, (1 - dt sdr) ene
    dt = -float(lp.data[p + 1])
    eta = float(lp.data[p]) / dt
    sdr = (1.0 - float(lp.data[p + 2])) / dt
    olp = dict(K=K, q=lp.q, c=lp.c, c0=lp.c0, l=lp.l, u=lp.u, m_eq=lp.m_eq, T=T, J=lp.n - 3 * T)
    return olp, dt, eta, sdr, float(lp.q[0])


class FakeProblem:
    """The cvx.Problem surface the drop-in touches: unpack_results(solution, chain, inverse_data) through the
    restated ECOS inversion; status / value / x as CVXPY leaves them."""

    def __init__(self, data, col):
        self.data, self.col = data, col
        self.status, self.value, self.x, self.duals = None, None, None, None

    def unpack_results(self, solution, chain, inverse_data):
        r = invert(solution, self.data["offset"])
        self.status, self.value, self.x = r["status"], r["value"], r["x"]
        self.duals = (r["y"], r["z"])


def ecos_bb_market_form(win, seed=0):
    """ECOS_BB data dict of a binary = 1 market-day window (oracle.window_lp market window) as CVXPY 1.0.31 would
    emit it for the reference's MILP: the build() LP without the relaxation row plus storagevet's boolean on_c / on_d
    (ElectricVehicles.py:120-122 pattern) with ch_t <= P_ch on_c_t, dis_t <= P_dis on_d_t, on_c_t + on_d_t <= 1,
    columns shuffled (CVXPY orders by variable id), every bound a one-entry G row, the boolean columns listed in
    ``bool_vars_idx`` (ECOS_BB.apply) and NOT boxed by any row (integrality is what bounds them).  Returns
    (data, col) with col[o] = ECOS column of build() column o; the on_c / on_d columns are col[n:n + 2T]."""
    from oracle import window_lp
    rng = np.random.default_rng(seed)
    lp = window_lp.build(dict(win, binary_relax=False))
    K, q, m_eq, off = lp["K"].tocsr(), lp["q"], lp["m_eq"], lp["layout"]
    n, T = K.shape[1], int(win["T"])
    N = n + 2 * T
    col = rng.permutation(N)
    Ke = K[:m_eq].tocoo()
    A = sp.csr_matrix((Ke.data, (Ke.row, col[Ke.col])), shape=(m_eq, N))
    rows, cols, vals, h = [], [], [], []

    def grow(entries, rhs):
        r = len(h)
        for cc, vv in entries:
            rows.append(r)
            cols.append(cc)
            vals.append(vv)
        h.append(rhs)

    for o in range(n):
        if np.isfinite(lp["u"][o]):
            grow([(col[o], 1.0)], lp["u"][o])
        if np.isfinite(lp["l"][o]):
            grow([(col[o], -1.0)], -lp["l"][o])
    for i in range(m_eq, K.shape[0]):
        p0, p1 = K.indptr[i], K.indptr[i + 1]
        grow([(col[K.indices[p]], -K.data[p]) for p in range(p0, p1)], -q[i])
    b = win["bat"]
    for t in range(T):
        grow([(col[off["ch"] + t], 1.0), (col[n + t], -float(b["Pch"]))], 0.0)
        grow([(col[off["dis"] + t], 1.0), (col[n + T + t], -float(b["Pdis"]))], 0.0)
        grow([(col[n + t], 1.0), (col[n + T + t], 1.0)], 1.0)
    G = sp.csr_matrix((vals, (rows, cols)), shape=(len(h), N))
    c = np.zeros(N)
    c[col[:n]] = lp["c"]
    data = {"c": c, "offset": float(lp["c0"]), "A": A.tocsc(), "b": np.asarray(q[:m_eq], np.float64),
            "G": G.tocsc(), "h": np.asarray(h), "dims": {"l": len(h), "q": [], "e": 0},
            "bool_vars_idx": [int(j) for j in col[n:]], "int_vars_idx": []}
    return data, col

"""ORACLE (test infrastructure only): numpy restatement of the batched PDHG algorithm the HIP kernels run.

This is *our* algorithm (the reference solves the window LP with ECOS / GLPK through CVXPY,
``dervet/MicrogridScenario.py:319``); it exists so that tests can compare the GPU solver's iterates,
iteration counts and statuses with an independent host implementation of the same arithmetic.
The LP-level oracle is HiGHS (``oracle.window_lp.solve_highs``).

Algorithm (restarted reflected Halpern PDHG, PDLP-family):
  LP:  min c'x + c0   s.t.  K_E x = q_E,  K_I x >= q_I,  l <= x <= u
  1. diagonal preconditioning: ``ruiz_iters`` Ruiz inf-norm passes, then one Pock-Chambolle (alpha=1) pass:
        Kt = Dr K Dc,  ct = Dc c,  qt = Dr q,  lt = l / Dc,  ut = u / Dc
  2. step: eta = step_safety / ||Kt||_2 (power iteration, ``power_iters`` steps from the all-ones vector);
     tau = eta / w, sigma = eta * w, primal weight w0 = ||ct|| / ||qt|| (1 if either is 0)
  3. PDHG operator T(x, y):  x+ = proj_[lt,ut](x - tau (ct - Kt'y));  y+ = proj_Y(y + sigma (qt - Kt(2x+ - x)))
     with proj_Y clamping the >= rows' duals at 0.
  4. reflected Halpern step:  z_{k+1} = (k+1)/(k+2) ((1+rho) T(z_k) - rho z_k) + 1/(k+2) z_anchor
  5. every ``check_every`` iterations (termination every ``kkt_every`` such checks): fixed-point residual r = ||z_k - T(z_k)||_w  with
     ||(dx,dy)||_w^2 = w ||dx||^2 + ||dy||^2 / w; restart when r <= b_suff r0, or (r <= b_nec r0 and
     r > r_prev), or k >= b_art * total; on restart z_anchor = z = T(z_k) and the primal weight moves
     halfway (in log space) towards ||dy|| / ||dx|| of the anchor change.
     Termination uses the relative KKT error of the unscaled candidate T(z_k):
        ||primal res||_2 <= eps (1 + ||q||_2),  ||dual res||_2 <= eps (1 + ||c||_2),
        |pobj - dobj| <= eps (1 + |pobj| + |dobj|).
"""
import numpy as np

OPTIMAL, PRIMAL_INFEASIBLE, DUAL_INFEASIBLE, ITER_LIMIT, NUMERICAL = 0, 1, 2, 3, 4

# defaults mirror dvh_default_options (der-vet_amd/csrc/dvh_api.cpp)
DEFAULTS = dict(eps=1e-6, max_iters=100000, check_every=32, kkt_every=4, ruiz_iters=10, power_iters=64,
                step_safety=0.998, rho=1.0, b_suff=0.2, b_nec=0.8, b_art=0.1, theta=1.0, eps_obj=1e-6)


def precondition(K, ruiz_iters):
    """Returns (Dr, Dc) with Kt = diag(Dr) K diag(Dc)."""
    import scipy.sparse as sp
    K = sp.csr_matrix(K)
    m, n = K.shape
    Dr = np.ones(m)
    Dc = np.ones(n)
    A = abs(K).tocsr()
    for _ in range(ruiz_iters):
        S = sp.diags(Dr) @ A @ sp.diags(Dc)
        rmax = np.asarray(S.max(axis=1).todense()).ravel()
        cmax = np.asarray(S.max(axis=0).todense()).ravel()
        Dr /= np.sqrt(np.where(rmax > 0, rmax, 1.0))
        Dc /= np.sqrt(np.where(cmax > 0, cmax, 1.0))
    S = sp.diags(Dr) @ A @ sp.diags(Dc)
    rs = np.asarray(S.sum(axis=1)).ravel()
    cs = np.asarray(S.sum(axis=0)).ravel()
    Dr /= np.sqrt(np.where(rs > 0, rs, 1.0))
    Dc /= np.sqrt(np.where(cs > 0, cs, 1.0))
    return Dr, Dc


def power_norm(Kt, iters):
    """sigma_max(Kt) from `iters` steps of v <- Kt'(Kt v) from v0 = 1/sqrt(n) (no per-step normalisation,
    as the ELL kernel does it): sigma^2 = |v_iters| / |v_iters-1|."""
    n = Kt.shape[1]
    v = np.ones(n) / np.sqrt(n)
    prev = v
    for _ in range(iters):
        prev = v
        v = Kt.T @ (Kt @ v)
    a, b = np.linalg.norm(prev), np.linalg.norm(v)
    return np.sqrt(b / a) if a > 0 and b > 0 else 1.0


def solve(lp, opts=None, trace=None):
    """lp: dict(K csr, q, c, c0, l, u, m_eq).  Returns dict(x, y, obj, status, iters, kkt)."""
    import scipy.sparse as sp
    o = dict(DEFAULTS)
    o.update(opts or {})
    K = sp.csr_matrix(lp["K"])
    m, n = K.shape
    m_eq = int(lp["m_eq"])
    q, c, l, u = (np.asarray(lp[k], float) for k in ("q", "c", "l", "u"))
    c0 = float(lp.get("c0", 0.0))
    Dr, Dc = precondition(K, o["ruiz_iters"])
    Kt = (sp.diags(Dr) @ K @ sp.diags(Dc)).tocsr()
    KtT = Kt.T.tocsr()
    ct, qt = Dc * c, Dr * q
    lt, ut = l / Dc, u / Dc
    # power_iters = 0: use the Pock-Chambolle bound ||Kt||_2 <= 1 instead of an estimate
    eta = o["step_safety"] / (power_norm(Kt, o["power_iters"]) if o["power_iters"] > 0 else 1.0)
    nc, nq = np.linalg.norm(ct), np.linalg.norm(qt)
    w = nc / nq if (nc > 1e-10 and nq > 1e-10) else 1.0
    q_norm, c_norm = np.linalg.norm(q), np.linalg.norm(c)
    finite_l, finite_u = np.isfinite(l), np.isfinite(u)

    def T(x, y):
        tau, sigma = eta / w, eta * w
        xp = np.clip(x - tau * (ct - KtT @ y), lt, ut)
        yp = y + sigma * (qt - Kt @ (2 * xp - x))
        yp[m_eq:] = np.maximum(yp[m_eq:], 0.0)
        return xp, yp

    def kkt(xs, ys):
        x = Dc * xs
        y = Dr * ys
        r = q - K @ x
        r[m_eq:] = np.maximum(r[m_eq:], 0.0)
        rc = c - K.T @ y
        lam = np.where(finite_l & finite_u, rc,
                       np.where(finite_l, np.maximum(rc, 0), np.where(finite_u, np.minimum(rc, 0), 0.0)))
        rd = rc - lam
        pobj = c @ x + c0
        dobj = q @ y + np.sum(np.where(finite_l, l, 0) * np.maximum(lam, 0)) + \
            np.sum(np.where(finite_u, u, 0) * np.minimum(lam, 0)) + c0
        return dict(pres=np.linalg.norm(r), dres=np.linalg.norm(rd), pobj=pobj, dobj=dobj,
                    xnorm=np.linalg.norm(x), ynorm=np.linalg.norm(y), rdx=float(np.sum(np.abs(rd) * np.abs(x))),
                    pres_rel=np.linalg.norm(r) / (1 + q_norm), dres_rel=np.linalg.norm(rd) / (1 + c_norm),
                    gap_rel=abs(pobj - dobj) / (1 + abs(pobj) + abs(dobj)))

    def obj_ok(i):
        # objective-error estimate (eps_obj > 0): |pobj - dobj| + ||y||_2 ||r_p||_2 + sum_j |r_d,j| |x_j|
        # <= eps_obj (1 + |pobj|) (the last term: what the dual objective can overstate the optimum by; the kernels'
        # kkt_done, csrc/dvh_device.h, since round 4)
        if not o["eps_obj"] > 0.0:
            return True
        return abs(i["pobj"] - i["dobj"]) + i["ynorm"] * i["pres"] + i["rdx"] <= o["eps_obj"] * (1.0 + abs(i["pobj"]))

    # warm start (dvh_options.warm_start): unscaled x0 / y0 moved into the scaled space; optional w0
    x = np.clip(np.asarray(o["x0"], float) / Dc if o.get("x0") is not None else np.zeros(n), lt, ut)
    y = np.asarray(o["y0"], float) / Dr if o.get("y0") is not None else np.zeros(m)
    y[m_eq:] = np.maximum(y[m_eq:], 0.0)
    if o.get("w0"):
        w = float(o["w0"])
    elif o.get("x0") is not None:
        # the band kernels' warm-start weight: geometric mean of the data's and the start's ||y~|| / ||x~||
        # (der-vet_amd/csrc/dvh_band.hip)
        nx, ny = float(x @ x), float(y @ y)
        if nx > 1e-20 and ny > 1e-20:
            w = np.sqrt(np.sqrt(ny / nx) * w)
    xa, ya = x.copy(), y.copy()
    k = 0
    r0 = None
    r_prev = None
    status = ITER_LIMIT
    it = 0
    rho = o["rho"]
    info = None
    last = (x, y)
    while it < o["max_iters"]:
        xp, yp = T(x, y)
        it += 1
        if it % o["check_every"] == 0:
            dx, dy = x - xp, y - yp
            r = np.sqrt(w * (dx @ dx) + (dy @ dy) / w)
            if it % (o["check_every"] * o["kkt_every"]) == 0 or it + o["check_every"] > o["max_iters"]:
                info = kkt(xp, yp)
                last = (xp, yp)
                if trace is not None:
                    trace.append((it, k, w, r, info["pres_rel"], info["dres_rel"], info["gap_rel"]))
                if info["pres_rel"] <= o["eps"] and info["dres_rel"] <= o["eps"] and info["gap_rel"] <= o["eps"] \
                        and obj_ok(info):
                    x, y = xp, yp
                    status = OPTIMAL
                    break
            if r0 is None:
                r0 = r
            restart = (r <= o["b_suff"] * r0) or (r <= o["b_nec"] * r0 and r_prev is not None and r > r_prev) \
                or (k + 1 >= o["b_art"] * it)
            if restart:
                ddx, ddy = np.linalg.norm(xp - xa), np.linalg.norm(yp - ya)
                if ddx > 1e-10 and ddy > 1e-10:
                    w = np.exp(o["theta"] * np.log(ddy / ddx) + (1 - o["theta"]) * np.log(w))
                x, y = xp, yp
                xa, ya = xp.copy(), yp.copy()
                k = 0
                r0 = r
                r_prev = None
                continue
            r_prev = r
        cb = 1.0 / (k + 2)
        ca = 1.0 - cb
        x = ca * ((1 + rho) * xp - rho * x) + cb * xa
        y = ca * ((1 + rho) * yp - rho * y) + cb * ya
        k += 1
    xs, ys = (x, y) if status == OPTIMAL else last
    info = kkt(xs, ys)
    xo = Dc * xs
    return dict(x=xo, y=Dr * ys, obj=float(c @ xo + c0), status=status, iters=it, kkt=info, w=w)

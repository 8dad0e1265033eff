"""Vectorised builder of DER-VET dispatch-window LPs for many windows at once (native export path).

Emits exactly the LP that storagevet's ``Scenario.set_up_optimization`` + CVXPY hand to the solver at
``dervet/MicrogridScenario.py:319`` for the in-scope DER / value-stream set (SURVEY.md section 8a rows
a3-a10, Appendix A), in the canonical form of include/dervet_hip.h (equalities first, then >= rows):

  x = [ch(T), dis(T), ene(T), tau(J)]                              (battery: ESSSizing.py:223-278)
  row 0            ene_0 = target                                  (target = soc_target * E)
  rows 1..T-1      -dt eta ch_t + dt dis_t - (1 - dt sdr) ene_t + ene_{t+1} = 0
  row T            dt eta ch_{T-1} - dt dis_{T-1} + (1 - dt sdr) ene_{T-1} = target
  >= rows          -ch_t + dis_t + tau_j >= L_t - G_t + hp          for t in M_j   (DCM epigraph)
  bounds           0 <= ch <= P_ch, 0 <= dis <= P_dis, max(llsoc E, a_min) <= ene <= min(ulsoc E, a_max)
  objective keys   'retailETS', 'DCM', 'DA', '<es> fixed_om', '<es> var_om'  (golden objective_values columns)

Windows that share (T, J, demand masks) share one CSR pattern; values broadcast over the G windows of a
group, so a 10,000-scenario x 12-month sweep is built with a handful of array operations.
"""
from dataclasses import dataclass, field

import numpy as np

from ..packed import PackedBatch


@dataclass
class WindowGroup:
    """G windows with one CSR pattern."""
    T: int
    J: int
    m_eq: int
    indptr: np.ndarray      # int32 [m+1]
    indices: np.ndarray     # int32 [nnz]
    data: np.ndarray        # f64 [G, nnz]
    c: np.ndarray           # f64 [G, n]
    c0: np.ndarray          # f64 [G]
    q: np.ndarray           # f64 [G, m]
    l: np.ndarray           # f64 [G, n]
    u: np.ndarray           # f64 [G, n]
    terms: dict = field(default_factory=dict)   # key -> (coef [G, n], const [G])
    tags: list = field(default_factory=list)    # per-window identifiers (scenario, window)

    @property
    def G(self):
        return self.data.shape[0]

    @property
    def n(self):
        return self.c.shape[1]

    @property
    def m(self):
        return self.q.shape[1]


def _col(a, G, T=None):
    a = np.asarray(a, np.float64)
    if T is None:
        return np.broadcast_to(a, (G,)).astype(np.float64, copy=True) if a.ndim <= 1 else a
    return np.broadcast_to(a, (G, T)).astype(np.float64, copy=False)


def battery_group(T, dt, base_load, bat, retail_price=None, da_price=None, demand_masks=None, demand_prices=None,
                  ene_min=None, ene_max=None, name="es", tags=None, pv_curtail_max=None, ice=None, poi=None,
                  grid_charge=True, pv_gen=None):
    """Build G windows sharing T steps and the demand masks.

    base_load [G, T]  : site load minus fixed generation (kW), hp is added here from ``bat``
    bat               : dict of [G] (or scalar) arrays: E, Pch, Pdis, rte (fraction), sdr (%/h), soc_target,
                        ulsoc, llsoc (fractions), fixedOM ($/kW-yr, charged per window), OMexpenses ($/MWh), hp (kW)
    retail_price, da_price [G, T] ($/kWh) or None
    demand_masks bool [J, T] ; demand_prices [G, J] ($/kW)
    ene_min / ene_max [G, T] aggregate SOE limits (User / Reliability requirements) or None
    pv_curtail_max [G, T]: curtailable PV (IntermittentResourceSizing.py:79-91, curtail = 1): variable
                      0 <= pv_t <= max_t subtracted from the net load (UNPINNED)
    ice               : dict of [G] arrays rated_power, n, min_power, efficiency (gal/kWh), fuel_cost ($/gal),
                      variable_om_cost ($/kWh): storagevet RotatingGenerator rows
                      min_power n on_t <= elec_t <= rated n on_t with on_t in [0, 1] (the opt-in LP relaxation
                      of the binary commitment, RotatingGeneratorSizing.py:110-136; UNPINNED)
    poi               : dict max_import (<= 0 kW), max_export (>= 0 kW), scalars or [G]: storagevet POI interconnection
                      limits (Scenario apply_interconnection_constraints, Schema.json:2123,2194,2199), the net export
                      -(net load) within [max_import, max_export] every step (UNPINNED)
    grid_charge       : False = PV grid_charge 0 (Schema.json:1875): the battery charges from PV only, ch_t <= pv_gen_t
                      (+ pv_t if curtailable); with fixed PV only it tightens ch's upper bound (UNPINNED)
    pv_gen [G, T]     : the fixed PV generation inside base_load (for grid_charge = False)
    Variable order [ch, dis, ene, tau, pv?, elec?, on?]; >= rows: DCM epigraph, per step the two ICE rows, the POI
    import rows, the POI export rows, the charge-from-PV rows (grid_charge = False with curtailable PV).
    """
    base_load = np.atleast_2d(np.asarray(base_load, np.float64))
    G = base_load.shape[0]
    masks = np.zeros((0, T), bool) if demand_masks is None else np.asarray(demand_masks, bool)
    masks = masks[masks.any(axis=1)] if len(masks) else masks
    J = masks.shape[0]
    E = _col(bat["E"], G)
    pch, pdis = _col(bat["Pch"], G), _col(bat["Pdis"], G)
    eta, sdr = _col(bat["rte"], G), _col(bat.get("sdr", 0.0), G) / 100.0
    target = _col(bat.get("soc_target", 1.0), G) * E
    hp = _col(bat.get("hp", 0.0), G)
    base = base_load + hp[:, None]
    n = 3 * T + J
    ich, idis, iene, itau = 0, T, 2 * T, 3 * T
    ipv = ielec = ion = -1
    if pv_curtail_max is not None:
        ipv = n
        n += T
    if ice is not None:
        ielec, ion = n, n + T
        n += 2 * T
    net_extra = [c for c in (ipv, ielec) if c >= 0]  # columns that reduce the net load (-1 coefficient)
    t = np.arange(T)

    # ---- pattern: row lengths 1, 4 x (T-1), 3, then 3 per >= row
    rows_i = [np.nonzero(mk)[0] for mk in masks]
    mI = int(sum(len(r) for r in rows_i))
    w_dcm = 3 + len(net_extra)
    n_poi = 2 * T if poi is not None else 0
    n_gc = T if (not grid_charge and ipv >= 0) else 0
    m = T + 1 + mI + (2 * T if ice is not None else 0) + n_poi + n_gc
    lens = np.concatenate([[1], np.full(T - 1, 4), [3], np.full(mI, w_dcm),
                           np.full(2 * T if ice is not None else 0, 2), np.full(n_poi, w_dcm - 1),
                           np.full(n_gc, 2)]).astype(np.int64)
    indptr = np.zeros(m + 1, np.int64)
    np.cumsum(lens, out=indptr[1:])
    nnz = int(indptr[-1])
    indices = np.empty(nnz, np.int32)
    data = np.empty((G, nnz))
    indices[0] = iene
    data[:, 0] = 1.0
    # recurrence rows (sorted columns: ch_t, dis_t, ene_t, ene_t+1)
    r = indptr[1:T].reshape(-1, 1) + np.arange(4)
    tt = t[:-1]
    indices[r] = np.stack([ich + tt, idis + tt, iene + tt, iene + tt + 1], axis=1)
    data[:, r[:, 0]] = -dt * eta[:, None]
    data[:, r[:, 1]] = dt
    data[:, r[:, 2]] = -(1.0 - dt * sdr)[:, None]
    data[:, r[:, 3]] = 1.0
    # final row
    p = indptr[T]
    indices[p:p + 3] = [ich + T - 1, idis + T - 1, iene + T - 1]
    data[:, p] = dt * eta
    data[:, p + 1] = -dt
    data[:, p + 2] = 1.0 - dt * sdr
    # DCM epigraph rows
    q = np.zeros((G, m))
    q[:, 0] = target
    q[:, T] = target
    row = T + 1
    for j, ti in enumerate(rows_i):
        k = len(ti)
        rr = indptr[row:row + k].reshape(-1, 1) + np.arange(w_dcm)
        indices[rr] = np.stack([ich + ti, idis + ti, np.full(k, itau + j)] + [c0_ + ti for c0_ in net_extra], axis=1)
        data[:, rr[:, 0]] = -1.0
        data[:, rr[:, 1]] = 1.0
        data[:, rr[:, 2]] = 1.0
        for e in range(3, w_dcm):
            data[:, rr[:, e]] = 1.0
        q[:, row:row + k] = base[:, ti]
        row += k
    if ice is not None:
        cap = _col(ice["rated_power"], G) * _col(ice.get("n", 1.0), G)
        pmin = _col(ice.get("min_power", 0.0), G) * _col(ice.get("n", 1.0), G)
        r1 = indptr[row + 2 * t]        # cap on_t - elec_t >= 0
        r2 = indptr[row + 2 * t + 1]    # elec_t - pmin on_t >= 0
        indices[r1], indices[r1 + 1] = ielec + t, ion + t
        indices[r2], indices[r2 + 1] = ielec + t, ion + t
        data[:, r1] = -1.0
        data[:, r1 + 1] = cap[:, None]
        data[:, r2] = 1.0
        data[:, r2 + 1] = -pmin[:, None]
        row += 2 * T
    if poi is not None:  # import: -ch + dis + pv + elec >= base + max_import; export: the negation >= -max_export - base
        for sign, rhs in ((-1.0, base + _col(poi["max_import"], G)[:, None]),
                          (1.0, -_col(poi["max_export"], G)[:, None] - base)):
            rr = indptr[row:row + T].reshape(-1, 1) + np.arange(w_dcm - 1)
            indices[rr] = np.stack([ich + t, idis + t] + [c0_ + t for c0_ in net_extra], axis=1)
            data[:, rr[:, 0]] = sign
            data[:, rr[:, 1]] = -sign
            for e in range(2, w_dcm - 1):
                data[:, rr[:, e]] = -sign
            q[:, row:row + T] = rhs
            row += T
    pvg = np.zeros((G, T)) if pv_gen is None else _col(pv_gen, G, T)
    if n_gc:  # charge from PV only: pv_t - ch_t >= -pv_gen_t
        rr = indptr[row:row + T].reshape(-1, 1) + np.arange(2)
        indices[rr] = np.stack([ich + t, ipv + t], axis=1)
        data[:, rr[:, 0]] = -1.0
        data[:, rr[:, 1]] = 1.0
        q[:, row:row + T] = -pvg
        row += T

    # ---- bounds
    l = np.zeros((G, n))
    u = np.empty((G, n))
    u[:, ich:ich + T] = pch[:, None]
    if not grid_charge and ipv < 0:  # charge from the fixed PV only
        u[:, ich:ich + T] = np.minimum(pch[:, None], pvg)
    u[:, idis:idis + T] = pdis[:, None]
    lo = (_col(bat.get("llsoc", 0.0), G) * E)[:, None] * np.ones((1, T))
    hi = (_col(bat.get("ulsoc", 1.0), G) * E)[:, None] * np.ones((1, T))
    if ene_min is not None:
        lo = np.maximum(lo, _col(ene_min, G, T))
    if ene_max is not None:
        hi = np.minimum(hi, _col(ene_max, G, T))
    l[:, iene:iene + T] = lo
    u[:, iene:iene + T] = hi
    l[:, itau:itau + J] = -np.inf
    u[:, itau:itau + J] = np.inf
    if ipv >= 0:
        u[:, ipv:ipv + T] = _col(pv_curtail_max, G, T)
    if ice is not None:
        u[:, ielec:ielec + T] = np.inf
        u[:, ion:ion + T] = 1.0

    # ---- objective terms
    terms = {}

    def net_term(price):
        pr = _col(price, G, T)
        coef = np.zeros((G, n))
        coef[:, ich:ich + T] = pr * dt
        coef[:, idis:idis + T] = -pr * dt
        for c0_ in net_extra:
            coef[:, c0_:c0_ + T] = -pr * dt
        return coef, (pr * dt * base).sum(axis=1)

    if da_price is not None:
        terms["DA"] = net_term(da_price)
    if J:
        coef = np.zeros((G, n))
        coef[:, itau:itau + J] = np.asarray(demand_prices, np.float64).reshape(G, J)
        terms["DCM"] = (coef, np.zeros(G))
    if retail_price is not None:
        terms["retailETS"] = net_term(retail_price)
    terms[f"{name} fixed_om"] = (np.zeros((G, n)), _col(bat.get("fixedOM", 0.0), G) * pdis)
    coef = np.zeros((G, n))
    coef[:, idis:idis + T] = (_col(bat.get("OMexpenses", 0.0), G) / 1000.0 * dt)[:, None]
    terms[f"{name} var_om"] = (coef, np.zeros(G))
    if ice is not None:
        coef = np.zeros((G, n))
        coef[:, ielec:ielec + T] = ((_col(ice["efficiency"], G) * _col(ice["fuel_cost"], G)
                                     + _col(ice.get("variable_om_cost", 0.0), G)) * dt)[:, None]
        terms["ice fuel_cost"] = (coef, np.zeros(G))
    c = np.zeros((G, n))
    c0 = np.zeros(G)
    for coef, const in terms.values():
        c += coef
        c0 += const
    return WindowGroup(T=T, J=J, m_eq=T + 1, indptr=indptr.astype(np.int32), indices=indices, data=data, c=c, c0=c0,
                       q=q, l=l, u=u, terms=terms, tags=list(tags) if tags is not None else [None] * G)


def _assemble(G, m, blocks):
    """CSR pattern + per-window values from COO blocks (rows [k], cols [k], vals [G, k]): entries sorted by
    (row, col), one pattern shared by the G windows."""
    rows = np.concatenate([np.asarray(r, np.int64) for r, _, _ in blocks])
    cols = np.concatenate([np.asarray(c, np.int64) for _, c, _ in blocks])
    vals = np.concatenate([np.broadcast_to(np.asarray(v, np.float64), (G, len(r))) for r, _, v in blocks], axis=1)
    order = np.lexsort((cols, rows))
    indptr = np.zeros(m + 1, np.int64)
    np.cumsum(np.bincount(rows, minlength=m), out=indptr[1:])
    return indptr.astype(np.int32), cols[order].astype(np.int32), np.ascontiguousarray(vals[:, order])


def market_group(T, dt, bat, da_price, fr, base=None, ene_min=None, ene_max=None, binary_relax=False, name="es",
                 tags=None, reserves=None, lf=None):
    """G windows of battery dispatch with the DA energy term and frequency-regulation reservations (storagevet
    MarketServiceUpAndDown / FrequencyRegulation + EnergyStorage).  Formulation and
    row order as oracle/window_lp.py (pinned to the Usecase 3 goldens: with binaries the restatement reproduces
    every golden daily objective; ``binary_relax`` is the opt-in LP relaxation of binary = 1 windows):

      x = [ch, dis, ene, up_ch, up_dis, down_ch, down_dis]  (T each)
      row 0 ene_0 = target; SOE rows with the energy option dt (rte uch - udis), uch = eou up_ch - eod down_ch,
      udis = eou up_dis - eod down_dis; final row back to target; [CombinedMarket: up = down]
      >= rows per block of T: P_ch - ch - down_ch, P_dis - dis - up_dis, ch - up_ch, dis - down_dis,
      (1 - rte) uch + 2 udis, [regu_max / regu_min], [regd_max / regd_min], [1 - ch / P_ch - dis / P_dis]
      objective keys 'DA', 'regup_prof', 'regdown_prof', 'fr_energy_settlement', '<es> fixed_om', '<es> var_om'

    da_price [G, T]; base [G, T] = load - fixed generation (kW) of the DA net term (zeros: incl_site_load = 0);
    fr: dict eou, eod (scalars), regu_price, regd_price, fr_price [G, T], optional regu_max, regu_min, regd_max,
    regd_min [G, T], combined (bool).

    reserves (optional, parity unpinned): upward-only reserve services (spinning / non-spinning reserve, storagevet
    MarketServiceUp via SpinningReserve / NonspinningReserve, registered at dervet/MicrogridScenario.py:93-94; the
    reference ships no golden result with them active), a list of dicts key ('SR' / 'NSR'), price [G, T] ($/kW),
    duration (h, template column SR/NSR duration), optional max / min [G, T] (ts_constraints).  Each adds
    x blocks [ch_less, dis_more] (T each, >= 0) after the FR blocks; ch_less joins the "ch - up_ch >= 0" row and
    dis_more the "P_dis - dis - up_dis >= 0" row (one shared headroom for every upward service); with a duration
    > 0 one more >= row per step, ene - sum_k duration_k dis_more_k >= lower SOE bound (the energy held back to
    sustain the extra discharge); objective key '<key>' = -price (ch_less + dis_more), per kW like regup_prof.
    lf (optional, parity unpinned): load following (storagevet LoadFollowing, a MarketServiceUpAndDown like FR;
    dervet/MicrogridScenario.py:92), dict eou, eod ([G, T] or scalar: template columns "LF Energy Option Up / Down
    (kWh/kW-hr)"), up_price, down_price, energy_price [G, T], optional up_max, up_min, down_max, down_min [G, T],
    combined.  x blocks [lf_up_ch, lf_up_dis, lf_down_ch, lf_down_dis] after the reserve blocks; its options join
    FR's in the SOE recurrence, the four headroom rows and the option-consistency row; keys 'lf_up_prof',
    'lf_down_prof', 'lf_energy_settlement' as FR's.  With lf the options enter through two free columns (uch, udis)
    appended last, each defined by one equality row per step (see ``agg`` below).
    Without reserves / lf the LP is exactly the pinned DA + FR window."""
    da_price = np.atleast_2d(np.asarray(da_price, np.float64))
    G = da_price.shape[0]
    base = np.zeros((G, T)) if base is None else _col(base, G, T)
    E = _col(bat["E"], G)
    pch, pdis = _col(bat["Pch"], G), _col(bat["Pdis"], G)
    eta, sdr = _col(bat["rte"], G), _col(bat.get("sdr", 0.0), G) / 100.0
    target = _col(bat.get("soc_target", 1.0), G) * E
    eou, eod = float(fr["eou"]), float(fr["eod"])
    combined = bool(fr.get("combined", False))
    ich, idis, iene, iuc, iud, idc, idd = (k * T for k in range(7))
    res = list(reserves or [])
    ires = [((7 + 2 * k) * T, (8 + 2 * k) * T) for k in range(len(res))]  # (ch_less, dis_more) offsets
    n = (7 + 2 * len(res)) * T
    luc = lud = ldc = ldd = -1  # load-following blocks (lf)
    if lf is not None:
        luc, lud, ldc, ldd = (n + k * T for k in range(4))
        n += 4 * T
        LEU, LED = _col(lf["eou"], G, T), _col(lf["eod"], G, T)
    # With LF the options of both services enter the SOE rows through two free aggregate columns
    # uch = sum eou up_ch - eod down_ch, udis = sum eou up_dis - eod down_dis (one equality row each per step):
    # the same LP projected onto the original columns, with 6-entry SOE rows instead of 12, so each ene column
    # sits in short rows only (the small-window ELL kernel's shape) -- without LF the pinned FR form is kept.
    agg = lf is not None
    iuh = iudh = -1
    if agg:
        iuh, iudh = n, n + T
        n += 2 * T
    t = np.arange(T)
    tt = t[:-1]
    one = np.ones((G, 1))
    col = lambda v: np.asarray(v, np.float64).reshape(G, 1) * np.ones((1, len(tt)))
    blocks = [([0], [iene], np.ones((G, 1)))]
    # SOE rows 1..T-1 (step t = row - 1): ene_{t+1} - (1 - dt sdr) ene_t - dt eta ch_t + dt dis_t
    #   - dt eta eou up_ch_t + dt eta eod down_ch_t + dt eou up_dis_t - dt eod down_dis_t = 0
    r = 1 + tt
    opt = ((iuh + tt, -dt * eta[:, None]), (iudh + tt, dt * one)) if agg else (
        (iuc + tt, -dt * eou * eta[:, None]), (idc + tt, dt * eod * eta[:, None]), (iud + tt, dt * eou * one),
        (idd + tt, -dt * eod * one))
    for c0_, v in ((iene + tt + 1, one), (iene + tt, -(1.0 - dt * sdr)[:, None]), (ich + tt, -dt * eta[:, None]),
                   (idis + tt, dt * one)) + opt:
        blocks.append((r, c0_, v * np.ones((1, len(tt)))))
    # final row: (1 - dt sdr) ene + dt eta ch - dt dis + dt (eta uch - udis) = target   (step T-1)
    k = T - 1
    opt = ((iuh + k, dt * eta), (iudh + k, -dt * np.ones(G))) if agg else (
        (iuc + k, dt * eou * eta), (idc + k, -dt * eod * eta), (iud + k, -dt * eou * np.ones(G)),
        (idd + k, dt * eod * np.ones(G)))
    for c0_, v in ((iene + k, 1.0 - dt * sdr), (ich + k, dt * eta), (idis + k, -dt * np.ones(G))) + opt:
        blocks.append(([T], [c0_], np.asarray(v).reshape(G, 1)))
    m = T + 1
    q_eq = [target[:, None], np.zeros((G, T - 1)), target[:, None]]
    if combined:
        for c0_, v in ((iuc, 1.0), (iud, 1.0), (idc, -1.0), (idd, -1.0)):
            blocks.append((m + t, c0_ + t, np.full((G, T), v)))
        q_eq.append(np.zeros((G, T)))
        m += T
    if lf is not None and lf.get("combined"):
        for c0_, v in ((luc, 1.0), (lud, 1.0), (ldc, -1.0), (ldd, -1.0)):
            blocks.append((m + t, c0_ + t, np.full((G, T), v)))
        q_eq.append(np.zeros((G, T)))
        m += T
    if agg:  # uch - sum(eou up_ch - eod down_ch) = 0, udis - sum(eou up_dis - eod down_dis) = 0
        for ia, (u_, d_), (lu_, ld_) in ((iuh, (iuc, idc), (luc, ldc)), (iudh, (iud, idd), (lud, ldd))):
            for c0_, v in ((ia, np.ones((G, 1))), (u_, np.full((G, 1), -eou)), (d_, np.full((G, 1), eod)),
                           (lu_, -LEU), (ld_, LED)):
                blocks.append((m + t, c0_ + t, np.broadcast_to(v, (G, T))))
            q_eq.append(np.zeros((G, T)))
            m += T
    m_eq = m
    q_ge = []

    def ge(entries, rhs):
        nonlocal m
        for c0_, v in entries:
            blocks.append((m + t, c0_ + t, np.broadcast_to(np.asarray(v, np.float64), (G, T))))
        q_ge.append(np.broadcast_to(np.asarray(rhs, np.float64), (G, T)))
        m += T

    xl = (lambda e: [e]) if lf is not None else (lambda e: [])  # LF's entries in the shared rows
    ge([(ich, -1.0), (idc, -1.0)] + xl((ldc, -1.0)), -pch[:, None])
    ge([(idis, -1.0), (iud, -1.0)] + xl((lud, -1.0)) + [(idm, -1.0) for _, idm in ires], -pdis[:, None])
    ge([(ich, 1.0), (iuc, -1.0)] + xl((luc, -1.0)) + [(icl, -1.0) for icl, _ in ires], 0.0)
    ge([(idis, 1.0), (idd, -1.0)] + xl((ldd, -1.0)), 0.0)
    if agg:
        ge([(iuh, (1.0 - eta)[:, None]), (iudh, 2.0)], 0.0)
    else:
        ge([(iuc, ((1.0 - eta) * eou)[:, None]), (idc, (-(1.0 - eta) * eod)[:, None]), (iud, 2.0 * eou),
            (idd, -2.0 * eod)], 0.0)
    # The other rows already imply up_ch + up_dis <= P_ch + P_dis and down_ch + down_dis <= P_ch + P_dis
    # (up_ch <= ch <= P_ch - down_ch, up_dis <= P_dis - dis; down_ch <= P_ch - ch, down_dis <= dis <= P_dis),
    # so a u/d_ts maximum above that is clamped to it: the same feasible set, but without the reference's
    # 9,999,999 kW "no limit" placeholders, which would inflate ||q|| and with it the solver's relative
    # primal tolerance (1e-6 x 7e7 = 70 kW of allowed infeasibility on a Usecase 3 day).
    cap = (pch + pdis)[:, None]
    if fr.get("regu_max") is not None:
        ge([(iuc, -1.0), (iud, -1.0)], -np.minimum(_col(fr["regu_max"], G, T), cap))
        ge([(iuc, 1.0), (iud, 1.0)], _col(fr["regu_min"], G, T))
    if fr.get("regd_max") is not None:
        ge([(idc, -1.0), (idd, -1.0)], -np.minimum(_col(fr["regd_max"], G, T), cap))
        ge([(idc, 1.0), (idd, 1.0)], _col(fr["regd_min"], G, T))
    if binary_relax:
        ge([(ich, (-1.0 / pch)[:, None]), (idis, (-1.0 / pdis)[:, None])], -1.0)
    lo = (_col(bat.get("llsoc", 0.0), G) * E)[:, None] * np.ones((1, T))
    hi = (_col(bat.get("ulsoc", 1.0), G) * E)[:, None] * np.ones((1, T))
    if ene_min is not None:
        lo = np.maximum(lo, _col(ene_min, G, T))
    if ene_max is not None:
        hi = np.minimum(hi, _col(ene_max, G, T))
    for rv, (icl, idm) in zip(res, ires):  # reserve participation limits (ts_constraints), clamped as FR's
        if rv.get("max") is not None:
            ge([(icl, -1.0), (idm, -1.0)], -np.minimum(_col(rv["max"], G, T), cap))
            ge([(icl, 1.0), (idm, 1.0)], _col(rv["min"], G, T))
    if lf is not None:
        if lf.get("up_max") is not None:
            ge([(luc, -1.0), (lud, -1.0)], -np.minimum(_col(lf["up_max"], G, T), cap))
            ge([(luc, 1.0), (lud, 1.0)], _col(lf["up_min"], G, T))
        if lf.get("down_max") is not None:
            ge([(ldc, -1.0), (ldd, -1.0)], -np.minimum(_col(lf["down_max"], G, T), cap))
            ge([(ldc, 1.0), (ldd, 1.0)], _col(lf["down_min"], G, T))
    dur = [float(rv.get("duration", 0.0)) for rv in res]
    if any(d > 0.0 for d in dur):
        ge([(iene, 1.0)] + [(idm, -d) for d, (_, idm) in zip(dur, ires) if d > 0.0], lo)
    indptr, indices, data = _assemble(G, m, blocks)
    q = np.concatenate(q_eq + q_ge, axis=1)

    l = np.zeros((G, n))
    u = np.full((G, n), np.inf)
    u[:, ich:ich + T] = pch[:, None]
    u[:, idis:idis + T] = pdis[:, None]
    if agg:
        l[:, iuh:iuh + 2 * T] = -np.inf
    l[:, iene:iene + T] = lo
    u[:, iene:iene + T] = hi

    terms = {}
    coef = np.zeros((G, n))
    coef[:, ich:ich + T] = da_price * dt
    coef[:, idis:idis + T] = -da_price * dt
    terms["DA"] = (coef, (da_price * dt * base).sum(axis=1))
    pu, pd_, pe = (_col(fr[k], G, T) for k in ("regu_price", "regd_price", "fr_price"))
    coef = np.zeros((G, n))
    coef[:, iuc:iuc + T] = -pu
    coef[:, iud:iud + T] = -pu
    terms["regup_prof"] = (coef, np.zeros(G))
    coef = np.zeros((G, n))
    coef[:, idc:idc + T] = -pd_
    coef[:, idd:idd + T] = -pd_
    terms["regdown_prof"] = (coef, np.zeros(G))
    coef = np.zeros((G, n))
    coef[:, iuc:iuc + T] = -pe * dt * eou
    coef[:, iud:iud + T] = -pe * dt * eou
    coef[:, idc:idc + T] = pe * dt * eod
    coef[:, idd:idd + T] = pe * dt * eod
    terms["fr_energy_settlement"] = (coef, np.zeros(G))
    for rv, (icl, idm) in zip(res, ires):
        coef = np.zeros((G, n))
        pr = _col(rv["price"], G, T)
        coef[:, icl:icl + T] = -pr
        coef[:, idm:idm + T] = -pr
        terms[str(rv["key"])] = (coef, np.zeros(G))
    if lf is not None:
        pu, pd_, pe = (_col(lf[k], G, T) for k in ("up_price", "down_price", "energy_price"))
        for key, blocks_, pr in (("lf_up_prof", (luc, lud), pu), ("lf_down_prof", (ldc, ldd), pd_)):
            coef = np.zeros((G, n))
            for b0 in blocks_:
                coef[:, b0:b0 + T] = -pr
            terms[key] = (coef, np.zeros(G))
        coef = np.zeros((G, n))
        coef[:, luc:luc + T] = -pe * dt * LEU
        coef[:, lud:lud + T] = -pe * dt * LEU
        coef[:, ldc:ldc + T] = pe * dt * LED
        coef[:, ldd:ldd + T] = pe * dt * LED
        terms["lf_energy_settlement"] = (coef, np.zeros(G))
    terms[f"{name} fixed_om"] = (np.zeros((G, n)), _col(bat.get("fixedOM", 0.0), G) * pdis)
    coef = np.zeros((G, n))
    coef[:, idis:idis + T] = (_col(bat.get("OMexpenses", 0.0), G) / 1000.0 * dt)[:, None]
    terms[f"{name} var_om"] = (coef, np.zeros(G))
    c = np.zeros((G, n))
    c0 = np.zeros(G)
    for coef, const in terms.values():
        c += coef
        c0 += const
    return WindowGroup(T=T, J=0, m_eq=m_eq, indptr=indptr, indices=indices, data=data, c=c, c0=c0, q=q, l=l, u=u,
                       terms=terms, tags=list(tags) if tags is not None else [None] * G)


def group_window_lps(g):
    """Per-window solver.WindowLP objects of a group (small batches, tests, the drop-in)."""
    from ..solver import WindowLP
    return [WindowLP(g.indptr, g.indices, g.data[k], g.c[k], g.q[k], g.l[k], g.u[k], g.m_eq, float(g.c0[k]),
                     meta={"tag": g.tags[k]}) for k in range(g.G)]


def pack_groups(groups):
    """Concatenate window groups into one numpy PackedBatch (group order, then window order)."""
    count = sum(g.G for g in groups)
    desc = np.zeros((count, 8), np.int64)
    k = 0
    tr = tz = tn = tm = 0
    for g in groups:
        G, n, m, nnz = g.G, g.n, g.m, len(g.indices)
        kk = np.arange(G, dtype=np.int64)
        desc[k:k + G] = np.stack([np.full(G, n), np.full(G, m), np.full(G, g.m_eq), np.full(G, nnz),
                                  tr + kk * (m + 1), tz + kk * nnz, tn + kk * n, tm + kk * m], axis=1)
        k += G
        tr += G * (m + 1)
        tz += G * nnz
        tn += G * n
        tm += G * m
    cat = lambda f, t: np.concatenate([np.ascontiguousarray(getattr(g, f), t).ravel() for g in groups])
    return PackedBatch(desc=desc,
                       indptr=np.concatenate([np.tile(g.indptr, g.G) for g in groups]).astype(np.int32),
                       indices=np.concatenate([np.tile(g.indices, g.G) for g in groups]).astype(np.int32),
                       data=cat("data", np.float64), c=cat("c", np.float64), c0=cat("c0", np.float64),
                       q=cat("q", np.float64), l=cat("l", np.float64), u=cat("u", np.float64))


def evaluate_terms(g, x):
    """Objective breakdown per window: {key: [G]} for solutions x [G, n] (the objective_values row)."""
    return {k: (coef * x).sum(axis=1) + const for k, (coef, const) in g.terms.items()}

"""Upward reserve services (spinning / non-spinning reserve) on the Usecase 3 daily
market windows.  PARITY UNPINNED: storagevet's MarketServiceUp / SpinningReserve / NonspinningReserve (registered
at dervet/MicrogridScenario.py:93-94) are absent from the reference snapshot and no shipped result has SR / NSR
active, so these tests pin the product builder (dervet_hip.lp.builder.market_group, ``reserves``) against the
independent per-window restatement (oracle/window_lp.py) and against properties any correct formulation has:
zero-price reserves leave the optimum unchanged, paid reserves never raise it, and the optimum respects the
shared headroom and the energy held back for the reserve duration (checked here from the definitions).
Reserve prices are synthetic (fractions of the fixture's Reg Up price), as the fixtures carry no SR / NSR column.
"""
import numpy as np
import pytest

from dervet_hip.lp import builder, scenarios
from oracle import cases, window_lp

CASES = ["es", "es+pv+dg"]
DAYS = [0, 100, 200]


def _signals(name):
    arr, meta = cases.load_market()
    return {k.split("__", 1)[1]: v for k, v in arr.items() if k.startswith(name + "__")}, meta[name]


def reserve_series(sig, pdis, scale=(0.6, 0.3), limits=True):
    """SR / NSR services over the whole fixture year: prices from the Reg Up price, durations 0.5 / 1 h,
    SR participation limited to [0, P_dis / 2] when ``limits``."""
    N = len(sig["da_price"])
    sr = dict(key="SR", price=scale[0] * sig["regu_price"], duration=0.5)
    if limits:
        sr["max"], sr["min"] = np.full(N, 0.5 * pdis), np.zeros(N)
    nsr = dict(key="NSR", price=scale[1] * sig["regu_price"], duration=1.0)
    return [sr, nsr]


def _oracle_window(win, res, n):
    """The oracle window dict of one day with the reserve series sliced to it."""
    s = slice(int(win["index"][0]), int(win["index"][0]) + n)
    w = dict(win)
    w["reserves"] = [dict(r, price=r["price"][s], **({"max": r["max"][s], "min": r["min"][s]}
                                                     if r.get("max") is not None else {})) for r in res]
    return w


@pytest.mark.parametrize("name", CASES)
def test_reserve_builder_matches_oracle(name):
    sig, meta = _signals(name)
    pdis = float(meta["params"]["Battery"]["dis_max_rated"])
    res = reserve_series(sig, pdis)
    g = scenarios.market_days(sig, meta["params"], days=DAYS, reserves=res)
    wins, _ = cases.market_windows(name)
    T = g.T
    assert g.n == 11 * T and set(g.terms) >= {"SR", "NSR", "DA", "regup_prof"}
    for k, d in enumerate(DAYS):
        o = window_lp.build(_oracle_window(wins[d], res, T))
        K = np.zeros((g.m, g.n))
        for r in range(g.m):
            K[r, g.indices[g.indptr[r]:g.indptr[r + 1]]] = g.data[k, g.indptr[r]:g.indptr[r + 1]]
        assert g.m_eq == o["m_eq"] and K.shape == o["K"].shape
        assert np.abs(K - o["K"].toarray()).max() <= 1e-14
        for a, b in ((g.c[k], o["c"]), (g.l[k], o["l"]), (g.u[k], o["u"])):
            assert np.array_equal(a, b) or np.abs(a - b).max() <= 1e-12
        # q equal up to the builder's clamp of participation maxima at P_ch + P_dis (same feasible set)
        hb = window_lp.solve_highs(dict(K=sp_csr(g, k), q=g.q[k], c=g.c[k], c0=float(g.c0[k]), l=g.l[k],
                                        u=g.u[k], m_eq=g.m_eq))
        ho = window_lp.solve_highs(o)
        assert hb["status"] == ho["status"] == 0
        assert abs(hb["obj"] - ho["obj"]) <= 1e-7 * max(abs(ho["obj"]), 1.0), (d, hb["obj"], ho["obj"])


def sp_csr(g, k):
    import scipy.sparse as sp
    return sp.csr_matrix((g.data[k], g.indices, g.indptr), shape=(g.m, g.n))


@pytest.mark.parametrize("name", CASES)
def test_reserve_properties(name):
    sig, meta = _signals(name)
    b = meta["params"]["Battery"]
    pch, pdis = float(b["ch_max_rated"]), float(b["dis_max_rated"])
    base = scenarios.market_days(sig, meta["params"], days=DAYS)
    free = scenarios.market_days(sig, meta["params"], days=DAYS,
                                 reserves=reserve_series(sig, pdis, scale=(0.0, 0.0)))
    paid = scenarios.market_days(sig, meta["params"], days=DAYS, reserves=reserve_series(sig, pdis))
    T = base.T
    for k, d in enumerate(DAYS):
        lp = lambda g: dict(K=sp_csr(g, k), q=g.q[k], c=g.c[k], c0=float(g.c0[k]), l=g.l[k], u=g.u[k],
                            m_eq=g.m_eq)
        h0, hf, hp = (window_lp.solve_highs(lp(g)) for g in (base, free, paid))
        assert h0["status"] == hf["status"] == hp["status"] == 0
        tol = 1e-7 * max(abs(h0["obj"]), 1.0)
        assert abs(hf["obj"] - h0["obj"]) <= tol, (d, hf["obj"], h0["obj"])  # unpaid reserves change nothing
        assert hp["obj"] <= h0["obj"] + tol, (d, hp["obj"], h0["obj"])       # paid reserves never cost
        x = hp["x"]
        blk = lambda i: x[i * T:(i + 1) * T]
        ch, dis, ene, uc, ud = blk(0), blk(1), blk(2), blk(3), blk(4)
        cl = blk(7) + blk(9)
        dm = blk(8) + blk(10)
        ftol = 1e-6 * max(pch, pdis)
        assert np.all(uc + cl <= ch + ftol) and np.all(dis + ud + dm <= pdis + ftol)
        assert np.all(blk(7) + blk(8) <= 0.5 * pdis + ftol)  # SR participation limit
        lo = paid.l[k][2 * T:3 * T]
        assert np.all(ene - 0.5 * blk(8) - 1.0 * blk(10) >= lo - 1e-6 * float(b["ene_max_rated"]))
        # the per-key objective values sum to the objective
        terms = sum(coef[k] @ x + const[k] for coef, const in paid.terms.values())
        assert abs(terms - hp["obj"]) <= 1e-8 * max(abs(hp["obj"]), 1.0)


def test_no_reserves_is_the_pinned_market_lp():
    sig, meta = _signals("es")
    a = scenarios.market_days(sig, meta["params"], days=DAYS)
    b = builder.market_group(a.T, 1.0, dict(E=1.0, Pch=1.0, Pdis=1.0, rte=0.9), np.zeros((1, a.T)),
                             dict(eou=0.3, eod=0.3, regu_price=np.zeros(a.T), regd_price=np.zeros(a.T),
                                  fr_price=np.zeros(a.T)), reserves=[])
    assert a.n == b.n == 7 * a.T
    c = scenarios.market_days(sig, meta["params"], days=DAYS, reserves=None)
    for f in ("indptr", "indices", "data", "q", "c", "l", "u"):
        assert np.array_equal(getattr(a, f), getattr(c, f))


def lf_series(sig, scale=1.0, limits=True, combined=False):
    """Load following over the whole fixture year: prices from the Reg Up / Down prices, energy settled at the
    DA price, per-step energy options around 0.2 kWh/kW-h, participation limited to P_dis / 4 when ``limits``."""
    N = len(sig["da_price"])
    h = np.arange(N)
    d = dict(eou=0.2 + 0.05 * np.sin(h / 7.0), eod=0.2 + 0.05 * np.cos(h / 5.0),
             up_price=scale * 0.8 * sig["regu_price"], down_price=scale * 0.8 * sig["regd_price"],
             energy_price=sig["da_price"], combined=combined)
    return d, limits


def _lf(sig, pdis, **kw):
    d, limits = lf_series(sig, **kw)
    if limits:
        N = len(sig["da_price"])
        d["up_max"] = d["down_max"] = np.full(N, 0.25 * pdis)
        d["up_min"] = d["down_min"] = np.zeros(N)
    return d


@pytest.mark.parametrize("name,combined", [("es", False), ("es+pv+dg", True)])
def test_load_following_builder_matches_oracle(name, combined):
    sig, meta = _signals(name)
    pdis = float(meta["params"]["Battery"]["dis_max_rated"])
    res = reserve_series(sig, pdis)
    lf = _lf(sig, pdis, combined=combined)
    g = scenarios.market_days(sig, meta["params"], days=DAYS, reserves=res, lf=lf)
    wins, _ = cases.market_windows(name)
    T = g.T
    # the builder carries the options through two free aggregate columns (uch, udis) after the oracle's 15 blocks
    assert g.n == 17 * T and {"lf_up_prof", "lf_down_prof", "lf_energy_settlement", "SR"} <= set(g.terms)
    n0 = 15 * T
    for k, d in enumerate(DAYS):
        w = _oracle_window(wins[d], res, T)
        s = slice(d * T, d * T + T)
        w["lf"] = {key: (v[s] if np.ndim(v) else v) for key, v in lf.items()}
        o = window_lp.build(w)
        assert o["K"].shape[1] == n0
        for a, b in ((g.c[k][:n0], o["c"]), (g.l[k][:n0], o["l"]), (g.u[k][:n0], o["u"])):
            assert np.array_equal(a, b) or np.abs(a - b).max() <= 1e-12
        assert not np.any(g.c[k][n0:]) and np.all(np.isneginf(g.l[k][n0:])) and np.all(np.isposinf(g.u[k][n0:]))
        hb = window_lp.solve_highs(dict(K=sp_csr(g, k), q=g.q[k], c=g.c[k], c0=float(g.c0[k]), l=g.l[k],
                                        u=g.u[k], m_eq=g.m_eq))
        ho = window_lp.solve_highs(o)
        assert hb["status"] == ho["status"] == 0
        assert abs(hb["obj"] - ho["obj"]) <= 1e-7 * max(abs(ho["obj"]), 1.0), (d, hb["obj"], ho["obj"])
        # the builder's optimum, restricted to the oracle's columns, is feasible and optimal for the oracle's LP
        xb = hb["x"][:n0]
        assert window_lp.primal_residual_rel(o, xb)[0] <= 1e-8
        assert abs(o["c"] @ xb + o["c0"] - ho["obj"]) <= 1e-7 * max(abs(ho["obj"]), 1.0)


def test_load_following_properties():
    """LF is optional participation: the optimum with it never exceeds the optimum without it (LF = 0 is
    feasible), and raising its capacity prices never raises the optimum.  (Zero-priced LF can still lower the
    optimum: FR's pinned energy-option form, which LF shares, credits up_ch with stored energy and energy revenue
    at once, so there is no "unchanged at price 0" identity to test.)"""
    sig, meta = _signals("es+pv+dg")
    pdis = float(meta["params"]["Battery"]["dis_max_rated"])
    base = scenarios.market_days(sig, meta["params"], days=DAYS)
    cheap = scenarios.market_days(sig, meta["params"], days=DAYS, lf=_lf(sig, pdis, scale=0.5))
    paid = scenarios.market_days(sig, meta["params"], days=DAYS, lf=_lf(sig, pdis))
    for k, d in enumerate(DAYS):
        lp = lambda g: dict(K=sp_csr(g, k), q=g.q[k], c=g.c[k], c0=float(g.c0[k]), l=g.l[k], u=g.u[k],
                            m_eq=g.m_eq)
        h0, hc, hp = (window_lp.solve_highs(lp(g)) for g in (base, cheap, paid))
        assert h0["status"] == hc["status"] == hp["status"] == 0
        tol = 1e-7 * max(abs(h0["obj"]), 1.0)
        assert hc["obj"] <= h0["obj"] + tol, (d, hc["obj"], h0["obj"])
        assert hp["obj"] <= hc["obj"] + tol, (d, hp["obj"], hc["obj"])

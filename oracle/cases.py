"""ORACLE (test infrastructure only): turn the committed golden fixtures into per-window LP inputs.

Window assignment restates storagevet ``Scenario`` ``optimization_levels`` for ``n = month`` / ``n = year``
(one window per calendar month / per year of the hour-beginning index), and the
DCM epigraph grouping is one tau per (month x demand billing period) inside the window (Appendix A).
"""
import json
import os

import numpy as np

from . import tariff as _tariff

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")


def load_case(name):
    arr = dict(np.load(os.path.join(GOLDEN, f"uc2_{name}.npz")))
    with open(os.path.join(GOLDEN, f"uc2_{name}.json")) as f:
        meta = json.load(f)
    return arr, meta


def battery_from_params(p):
    b = p["Battery"]
    return dict(
        name="es",
        E=float(b["ene_max_rated"]), Pch=float(b["ch_max_rated"]), Pdis=float(b["dis_max_rated"]),
        rte=float(b["rte"]) / 100.0, sdr=float(b["sdr"]), soc_target=float(b["soc_target"]) / 100.0,
        ulsoc=float(b["ulsoc"]) / 100.0, llsoc=float(b["llsoc"]) / 100.0,
        fixedOM=float(b["fixedOM"]), OMexpenses=float(b["OMexpenses"]), hp=float(b.get("hp", 0.0)),
    )


def case_windows(name):
    """Per-window LP input dicts (for oracle.window_lp.build) for a golden Usecase2 case."""
    arr, meta = load_case(name)
    p = meta["params"]
    T_all = len(arr["site_load"])
    year = int(p["Scenario"]["opt_years"])
    dt = float(p["Scenario"]["dt"])
    month, he, wd = _tariff.step_calendar(year, T_all, dt)
    price = _tariff.energy_price(meta["tariff"], month, he, wd)
    dem = _tariff.demand_periods(meta["tariff"], month, he, wd)
    gen = np.zeros(T_all)
    if "PV" in p and p["PV"].get("curtail", "0") in ("0", "0.0"):
        gen = float(p["PV"]["rated_capacity"]) * np.nan_to_num(arr["pv_profile"])
    bat = battery_from_params(p)
    if p["Scenario"]["n"] == "month":
        win_id = month - 1
    else:
        win_id = np.zeros(T_all, np.int32)
    wins = []
    for w in np.unique(win_id):
        sel = np.nonzero(win_id == w)[0]
        T = len(sel)
        demand = []
        for _, d, mask in dem:
            for mo in np.unique(month[sel]):
                mm = mask[sel] & (month[sel] == mo)
                if mm.any():
                    demand.append((d, mm))
        wins.append(dict(
            T=T, dt=dt, load=arr["site_load"][sel], gen=gen[sel], retail_price=price[sel], da_price=None,
            demand=demand, ene_min=arr["agg_emin"][sel], ene_max=arr["agg_emax"][sel], bat=bat,
            index=sel,
        ))
    return wins, arr, meta, price


def load_market():
    arr = dict(np.load(os.path.join(GOLDEN, "uc3_market.npz")))
    with open(os.path.join(GOLDEN, "uc3_market.json")) as f:
        meta = json.load(f)
    return arr, meta


def market_windows(name, relax=True):
    """Daily DA + FR window inputs (oracle.window_lp.build) of a Usecase 3 planned golden case (n = 24 steps:
    storagevet ``optimization_levels`` for an integer n are consecutive blocks of n steps), with the golden
    dispatch of each window as a solution vector in the build() layout (x_golden) and the golden objective row.
    Load is not included (incl_site_load = 0); fixed PV generation (curtail = 0) enters the DA net term."""
    arr, meta = load_market()
    m = meta[name]
    p = m["params"]
    key = lambda k: arr[f"{name}__{k}"]
    n = int(p["Scenario"]["n"])
    dt = float(p["Scenario"]["dt"])
    fr = p["FR"]
    bat = battery_from_params(p)
    N = len(key("da_price"))
    wins = []
    for d in range(N // n):
        s = slice(d * n, d * n + n)
        w = dict(T=n, dt=dt, load=np.zeros(n), gen=key("pv_gen")[s], retail_price=None, da_price=key("da_price")[s],
                 demand=[], ene_min=key("agg_emin")[s], ene_max=key("agg_emax")[s], bat=bat,
                 fr=dict(eou=float(fr["eou"]), eod=float(fr["eod"]), regu_price=key("regu_price")[s],
                         regd_price=key("regd_price")[s], fr_price=key("fr_price")[s],
                         combined=fr.get("CombinedMarket", "0") not in ("0", "0.0")),
                 binary_relax=relax and p["Scenario"].get("binary", "0") not in ("0", "0.0"),
                 golden_objective=key("golden_objective")[d], index=np.arange(d * n, d * n + n))
        if fr.get("u_ts_constraints", "0") not in ("0", "0.0"):
            w["fr"]["regu_max"], w["fr"]["regu_min"] = key("regu_max")[s], key("regu_min")[s]
        if fr.get("d_ts_constraints", "0") not in ("0", "0.0"):
            w["fr"]["regd_max"], w["fr"]["regd_min"] = key("regd_max")[s], key("regd_min")[s]
        w["x_golden"] = np.concatenate([key(k)[s] for k in ("golden_ch", "golden_dis", "golden_ene", "golden_up_ch",
                                                            "golden_up_dis", "golden_down_ch", "golden_down_dis")])
        wins.append(w)
    return wins, m["objective_keys"]

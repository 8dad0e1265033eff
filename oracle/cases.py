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

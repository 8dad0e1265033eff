"""Retail tariff -> per-step energy price and demand billing-period masks (vectorised).

Behaviour of storagevet ``Financial.calc_retail_energy_price`` (submodule absent; pinned by the golden
"Tariff Energy Price ($/kWh)" / "Demand Charge Billing Periods" columns of
``test/test_validation_report_sept1/Results/Usecase2/*/step2/timeseries_results*.csv``):
hour-ending he = hb.hour + 1; inclusive month / hour ranges; optional excluded hour range;
``Weekday?`` 1 = Mon-Fri, 0 = Sat-Sun, 2 = all days; energy charges of overlapping periods add up.
"""
import json

import numpy as np


def load_tariff_json(path):
    with open(path) as f:
        return json.load(f)


def calendar(start_year, n_steps, dt_hours=1.0):
    """Vectorised (month, hour_ending, weekday Mon=0, year) of hour-beginning steps from Jan 1 of start_year."""
    t0 = np.datetime64(f"{int(start_year):04d}-01-01T00:00")
    minutes = np.round(np.arange(n_steps) * dt_hours * 60.0).astype("timedelta64[m]")
    ts = t0 + minutes
    days = ts.astype("datetime64[D]")
    months = ts.astype("datetime64[M]")
    years = ts.astype("datetime64[Y]")
    month = (months - years).astype(int) + 1
    hour = ((ts - days).astype("timedelta64[h]")).astype(int)
    weekday = ((days.astype(np.int64) + 3) % 7).astype(np.int32)  # 1970-01-01 was a Thursday (=3)
    year = years.astype(int) + 1970
    return month.astype(np.int32), (hour + 1).astype(np.int32), weekday, year.astype(np.int32)


def _mask(t, k, month, he, wd):
    sel = (month >= t["start_month"][k]) & (month <= t["end_month"][k]) & \
          (he >= t["start_time"][k]) & (he <= t["end_time"][k])
    es, ee = t["excl_start"][k], t["excl_end"][k]
    if es is not None and ee is not None and np.isfinite(es) and np.isfinite(ee):
        sel &= ~((he >= es) & (he <= ee))
    w = int(t["weekday"][k])
    if w == 1:
        sel &= wd < 5
    elif w == 0:
        sel &= wd >= 5
    return sel


def energy_price(t, month, he, wd):
    kinds = np.array([c.strip().lower() for c in t["charge"]])
    vals = np.asarray(t["value"], float)
    masks = np.stack([_mask(t, k, month, he, wd) for k in range(len(vals))]) if len(vals) else np.zeros((0, len(month)), bool)
    e = kinds == "energy"
    return (vals[e][:, None] * masks[e]).sum(axis=0)


def demand_charges(t, month, he, wd):
    """(billing_period ids [P], $/kW [P], masks bool [P, T])."""
    kinds = np.array([c.strip().lower() for c in t["charge"]])
    idx = np.nonzero(kinds == "demand")[0]
    ids = np.asarray(t["billing_period"])[idx]
    vals = np.asarray(t["value"], float)[idx]
    masks = np.stack([_mask(t, k, month, he, wd) for k in idx]) if len(idx) else np.zeros((0, len(month)), bool)
    return ids, vals, masks

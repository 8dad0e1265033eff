"""ORACLE (test infrastructure only): tariff -> per-step retail energy price and demand billing periods.

Restates storagevet ``Financial.calc_retail_energy_price`` (absent submodule; behaviour pinned by the
golden "Tariff Energy Price ($/kWh)" and "Demand Charge Billing Periods" columns of
``test/test_validation_report_sept1/Results/Usecase2/es/step2/timeseries_resultsuc3_es_step2.csv``):

* timestamps are hour-beginning (``Start Datetime (hb)``); tariff hours are hour-ending, he = hb.hour + 1;
* month and hour ranges are inclusive; an optional excluded hour range is removed;
* ``Weekday?`` 1 = Monday-Friday, 0 = Saturday/Sunday, 2 = every day (tariff CSV notes,
  ``data/tariff.csv:2-7``);
* energy charges of all matching periods are summed; demand periods become billing-period masks.

Written as plain per-step Python loops on purpose (independent of the vectorised product version).
"""
import datetime as _dt

import numpy as np


def step_calendar(start_year, n_steps, dt_hours=1.0):
    """(month, hour_ending, weekday[Mon=0]) per hour-beginning step starting Jan 1 00:00 of start_year."""
    t0 = _dt.datetime(int(start_year), 1, 1)
    month = np.empty(n_steps, np.int32)
    he = np.empty(n_steps, np.int32)
    wd = np.empty(n_steps, np.int32)
    for i in range(n_steps):
        ts = t0 + _dt.timedelta(hours=i * dt_hours)
        month[i] = ts.month
        he[i] = ts.hour + 1
        wd[i] = ts.weekday()
    return month, he, wd


def _period_mask(tariff, k, month, he, wd):
    m = (month >= tariff["start_month"][k]) & (month <= tariff["end_month"][k])
    h = (he >= tariff["start_time"][k]) & (he <= tariff["end_time"][k])
    es, ee = tariff["excl_start"][k], tariff["excl_end"][k]
    if es is not None and not np.isnan(es) and ee is not None and not np.isnan(ee):
        h &= ~((he >= es) & (he <= ee))
    w = tariff["weekday"][k]
    if w == 1:
        d = wd < 5
    elif w == 0:
        d = wd >= 5
    else:
        d = np.ones_like(m)
    return m & h & d


def energy_price(tariff, month, he, wd):
    p = np.zeros(len(month))
    for k in range(len(tariff["billing_period"])):
        if tariff["charge"][k] == "energy":
            p[_period_mask(tariff, k, month, he, wd)] += tariff["value"][k]
    return p


def demand_periods(tariff, month, he, wd):
    """List of (billing_period_id, $/kW, bool mask) for the demand charges."""
    out = []
    for k in range(len(tariff["billing_period"])):
        if tariff["charge"][k] == "demand":
            out.append((tariff["billing_period"][k], tariff["value"][k], _period_mask(tariff, k, month, he, wd)))
    return out

"""The reference's degradation test cases as DegradationSweep runs (test helper).

Inputs come from tests/golden/degradation_cases.json (tests/golden/make_fixtures.py extracts them from
test/test_storagevet_features/model_params/{040,041,010}*.csv and their data files): the battery, scenario and value-
stream parameters, the tariff and the cycle-life table.  The 040 / 041 time series has zero site load (checked by the
extractor), so their monthly windows are retail energy time shift on the tariff alone; 010's are DA time shift on
data/hourly_timeseries.csv (the bench fixture's column, checked equal by the extractor).

Both cases are binary = 1 in the reference (MILP on GLPK_MI); the GPU solves the LP relaxation.  With zero load and
non-negative prices, charging and discharging at once only loses energy, so the relaxation's optimum is the MILP's.
"""
import json
import os

import numpy as np

from dervet_hip import degradation
from dervet_hip.lp import builder, scenarios

HERE = os.path.dirname(os.path.abspath(__file__))


def cases():
    with open(os.path.join(HERE, "golden", "degradation_cases.json")) as f:
        return json.load(f)


def battery(case, E):
    b = case["battery"]
    return dict(E=np.asarray(E, np.float64), Pch=float(b["ch_max_rated"]), Pdis=float(b["dis_max_rated"]),
                rte=float(b["rte"]) / 100.0, sdr=float(b["sdr"]), soc_target=float(b["soc_target"]) / 100.0,
                ulsoc=float(b["ulsoc"]) / 100.0, llsoc=float(b["llsoc"]) / 100.0, fixedOM=float(b["fixedOM"]),
                OMexpenses=float(b["OMexpenses"]), hp=float(b["hp"]))


def opt_years(case):
    return [int(y) for y in case["scenario"]["opt_years"].split()]


def sweep(case, spec=False):
    """(DegradationSweep, build) over every monthly window of every opt year, in time order (one scenario)."""
    assert case["scenario"]["n"] == "month" and float(case["scenario"]["dt"]) == 1.0
    b = case["battery"]
    years = opt_years(case)
    tar = case.get("tariff")
    da = scenarios.reference_inputs()["hourly_da_price"] if "DA" in case["value_streams"] else None
    if da is not None:
        assert case["da_price_is_bench_hourly_da_price"] and years == [2017]
    assert case["site_load_zero"]
    T_year = {y: 8784 if (y % 4 == 0 and (y % 100 != 0 or y % 400 == 0)) else 8760 for y in years}

    def build(k, cap):
        y = years[k // 12]
        return scenarios.windows_by_period(y, 1.0, np.zeros((1, T_year[y])), None, battery(case, cap),
                                           tariff_def=tar, da_price=None if da is None else da[None, :],
                                           only=[k % 12], spec=spec)

    deg = degradation.Degradation(
        [float(b["ene_max_rated"])], yearly_degrade=float(b["yearly_degrade"]),
        incl_cycle_degrade=bool(int(b["incl_cycle_degrade"])),
        table=(np.asarray(case["cycle_life"]["upper"]), np.asarray(case["cycle_life"]["life"])),
        eol_condition=float(b["cycle_life_table_eol_condition"]), state_of_health=float(b["state_of_health"]),
        replaceable=bool(int(b["replaceable"])))
    # Battery.py:84-85: calendar loss from the operation year's start to the step before the first window
    first = np.datetime64(f"{years[0]}-01-01T00:00") - np.timedelta64(1, "h")
    op = np.datetime64(f"{int(b['operation_year'])}-01-01T00:00")
    deg.age(max(0.0, float((first + np.timedelta64(1, "h") - op) / np.timedelta64(1, "D"))))
    positions = list(range(12 * len(years)))
    sw = degradation.DegradationSweep(build, positions, deg, years=[years[k // 12] for k in positions])
    return sw, build


def avoided_charges(case, sw, build, out):
    """Per opt year: the avoided energy charge (retailETS without the battery - with it) or, for DA, the DA
    revenue (- the DA term), summed over the year's windows, from each window's solution."""
    years = opt_years(case)
    key = "retailETS" if "retailTimeShift" in case["value_streams"] else "DA"
    res = {y: 0.0 for y in years}
    for p in out:
        g = build(p["k"], p["capacity_before"])[0]
        x = np.asarray(p["x"][0])[None, :]
        with_b = float(builder.evaluate_terms(g, x)[key][0])
        without = float(builder.evaluate_terms(g, np.zeros_like(x))[key][0])
        res[years[p["k"] // 12]] += without - with_b
    return res


class HighsSolver:
    """solve(lps) through the oracle (restated LP + HiGHS): the CPU leg of the degradation-case tests."""

    def solve(self, lps):
        import scipy.sparse as sp

        from oracle import window_lp

        class R:
            pass
        out = []
        for lp in lps:
            m = len(lp.q)
            K = sp.csr_matrix((lp.data, lp.indices, lp.indptr), shape=(m, len(lp.c)))
            h = window_lp.solve_highs(dict(K=K, q=lp.q, c=lp.c, c0=lp.c0, l=lp.l, u=lp.u, m_eq=lp.m_eq))
            r = R()
            r.status, r.iters = (0 if h["status"] == 0 else 4), 0
            r.obj, r.x = h.get("obj", np.nan), h.get("x", np.zeros(len(lp.c)))
            out.append(r)
        return out

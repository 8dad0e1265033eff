"""Battery benefit and CBA present values (oracle/cba.py) pinned to the reference's golden bills / pro forma / NPV
(test/test_validation_report_sept1/Results/Usecase2/{es, es+pv+dg}/step2, tests/golden/uc2_bills.json).
CPU: the restatement against the goldens with HiGHS dispatch; the GPU dispatch is checked in
tests/test_gpu_benefit.py."""
import json
import os

import numpy as np
import pytest

from oracle import cases, cba, window_lp

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "uc2_bills.json")


def bills():
    with open(GOLDEN) as f:
        return json.load(f)


@pytest.mark.parametrize("name", ["es", "es+pv+dg"])
def test_original_charges_and_npv_restatement_match_goldens(name):
    b = bills()[name]
    wins, _, _, _ = cases.case_windows(name)
    for i, w in enumerate(wins):
        e, d = cba.original_charges(w)
        assert e == pytest.approx(b["original_energy_charge"][i], rel=1e-12)
        assert d == pytest.approx(b["original_demand_charge"][i], rel=1e-12)
    # the 2017 avoided charges are the bill differences; the pro forma escalates them; its NPV is the golden row
    ae = np.sum(np.array(b["original_energy_charge"]) - b["energy_charge"])
    ad = np.sum(np.array(b["original_demand_charge"]) - b["demand_charge"])
    assert b["proforma"]["Avoided Energy Charge"][1] == pytest.approx(ae, rel=1e-9)
    assert b["proforma"]["Avoided Demand Charge"][1] == pytest.approx(ad, rel=1e-9)
    n0 = cba.proforma_npv(b)
    for k in ("Avoided Demand Charge", "Avoided Energy Charge", "Lifetime Present Value"):
        assert n0[k] == pytest.approx(b["npv"][k], rel=1e-9), k
    n1 = cba.proforma_npv(b, ae, ad)   # rebuilt from the bills' opt-year values
    for k in ("Avoided Demand Charge", "Avoided Energy Charge", "Lifetime Present Value"):
        assert n1[k] == pytest.approx(b["npv"][k], rel=1e-9), k


def test_highs_dispatch_reproduces_the_golden_benefit():
    b = bills()["es"]
    wins, _, _, _ = cases.case_windows("es")
    for i, w in enumerate(wins[:4]):
        olp = window_lp.build(w)
        h = window_lp.solve_highs(olp)
        oe, od = cba.original_charges(w)
        ben = oe + od - h["terms"]["retailETS"] - h["terms"]["DCM"]
        gold = b["original_energy_charge"][i] + b["original_demand_charge"][i] - b["energy_charge"][i] - \
            b["demand_charge"][i]
        assert ben == pytest.approx(gold, rel=1e-8)
        # obj_no_battery - obj is the same benefit (fixed O&M cancels; the PV-free original adds the PV credit)
        nb = cba.no_battery_objective(olp)
        assert nb - h["obj"] == pytest.approx(ben, rel=1e-9)

"""Battery benefit of the GPU dispatch against the reference's golden bills, pro forma and NPV (VERDICT r01 item 1;
SURVEY.md section 8d "also report error on obj - obj(no battery)", section 8f rank 1 "CBA NPV matches").

The golden Usecase 2 monthly windows (es; es + PV + DG) are built by the product builder and solved on cuda:0
through the C ABI.  Per window, benefit = original bill (site load alone, oracle/cba.py, pinned to the golden
"Original" columns) - (retailETS + DCM of the GPU dispatch), compared with the golden bill difference; the 12
benefits of the opt year against the golden pro forma's 2017 avoided charges; and the pro forma rebuilt from them
(escalated at the value streams' growth rates) against the golden NPV row.

Bars: per-window benefit within 1e-4 relative (the objective is solved to ~1e-6 of a 300 k$ window cost, and
the benefit is ~4-40 k$; measured at most 4.1e-5 with the same algorithm, oracle/cpu_pdhg.cpp, r03), yearly avoided
charges and NPVs within 1e-4.
"""
import numpy as np
import pytest

from dervet_hip import BatchSolver
from dervet_hip.lp import builder, scenarios
from oracle import cases, cba
from test_benefit import bills

pytestmark = pytest.mark.gpu


def gpu_benefits(name):
    wins, arr, meta, _ = cases.case_windows(name)
    bat = cases.battery_from_params(meta["params"])
    p = meta["params"]
    gen = None
    if "PV" in p and p["PV"].get("curtail", "0") in ("0", "0.0"):
        gen = float(p["PV"]["rated_capacity"]) * np.nan_to_num(arr["pv_profile"])
    groups = scenarios.windows_by_period(2017, 1.0, arr["site_load"][None], None if gen is None else gen[None], bat,
                                         tariff_def=meta["tariff"], ene_min=arr["agg_emin"][None],
                                         ene_max=arr["agg_emax"][None])
    lps = [lp for g in groups for lp in builder.group_window_lps(g)]
    with BatchSolver(0) as s:
        res = s.solve(lps)
        assert s.kernel_stats()["band_windows"] == len(lps)
    out = []
    for g, w, r in zip(groups, wins, res):
        assert r.status == 0
        t = builder.evaluate_terms(g, r.x[None, :])
        oe, od = cba.original_charges(w)
        out.append((oe - float(t["retailETS"][0]), od - float(t["DCM"][0])))
    return np.array(out)


@pytest.mark.parametrize("name", ["es", "es+pv+dg"])
def test_gpu_battery_benefit_matches_golden_bills_proforma_and_npv(name):
    b = bills()[name]
    ben = gpu_benefits(name)
    gold_e = np.array(b["original_energy_charge"]) - b["energy_charge"]
    gold_d = np.array(b["original_demand_charge"]) - b["demand_charge"]
    tot, gold = ben.sum(1), gold_e + gold_d
    rel = np.abs(tot - gold) / np.abs(gold)
    assert rel.max() <= 1e-4, rel
    ae, ad = ben[:, 0].sum(), ben[:, 1].sum()
    assert ae + ad == pytest.approx(b["proforma"]["Avoided Energy Charge"][1] + b["proforma"]["Avoided Demand Charge"][1],
                                    rel=1e-4)
    n = cba.proforma_npv(b, ae, ad)
    for k in ("Lifetime Present Value",):
        assert n[k] == pytest.approx(b["npv"][k], rel=1e-4), (k, n[k], b["npv"][k])
    assert n["Avoided Energy Charge"] + n["Avoided Demand Charge"] == pytest.approx(
        b["npv"]["Avoided Energy Charge"] + b["npv"]["Avoided Demand Charge"], rel=1e-4)
    print(f"{name}: max per-window benefit rel err {rel.max():.2e}, lifetime PV {n['Lifetime Present Value']:.2f} "
          f"vs golden {b['npv']['Lifetime Present Value']:.2f}")

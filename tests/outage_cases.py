"""Golden post-facto reliability cases (tests/golden/reliability_cases.*, from the reference's results CSVs)
as oracle inputs and as dervet_hip.reliability.OutageCase, following Reliability.py's choices (:896-905:
SOE at each start from the results' 'Aggregated State of Energy (kWh)', or soc_init x energy rating for
post-facto-reliability-only runs)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load():
    a = np.load(os.path.join(GOLDEN, "reliability_cases.npz"))
    with open(os.path.join(GOLDEN, "reliability_cases.json")) as f:
        meta = json.load(f)
    out = {}
    for name, m in meta.items():
        p = m["params"]
        b, r = p["Battery"], p["Reliability"]
        pv = a[f"{name}__pv_max"] if f"{name}__pv_max" in a.files else None
        out[name] = dict(
            critical_load=a[f"{name}__critical_load"], dt=float(p["Scenario"]["dt"]),
            max_outage_duration=int(float(r["max_outage_duration"])),
            ess=dict(E=float(b["ene_max_rated"]), P_ch=float(b["ch_max_rated"]), P_dis=float(b["dis_max_rated"]),
                     rte=float(b["rte"]) / 100, llsoc=float(b["llsoc"]) / 100, ulsoc=float(b["ulsoc"]) / 100),
            init_soe=a[f"{name}__aggregated_soe"] if f"{name}__aggregated_soe" in a.files else None,
            soc_init=float(r["post_facto_initial_soc"]) / 100,
            pv_max=[pv] if pv is not None else [], pv_nu=[float(r["nu"]) / 100] if pv is not None else [],
            pv_gamma=[float(r["gamma"]) / 100] if pv is not None else [],
            load_shed_pct=a[f"{name}__load_shed_pct"] if r.get("load_shed_percentage") == "1" else None,
            golden_lcp=a[f"{name}__golden_lcp"])
    return out


def oracle_curve(c):
    """(lengths, lcp) from oracle/outage.py for a case dict of load()."""
    from oracle import outage
    e = c["ess"]
    ess = outage.ess_props(e["E"], e["P_ch"], e["P_dis"], e["rte"], e["llsoc"], e["ulsoc"])
    pv = c["pv_max"][0] if c["pv_max"] else None
    cl, gen, pmax, pvar = outage.data_arrays(c["critical_load"], pv, c["pv_nu"][0] if pv is not None else 1.0)
    gamma = c["pv_gamma"][0] if pv is not None else 0.0
    soe = c["init_soe"] if c["init_soe"] is not None else c["soc_init"] * ess["energy rating"]
    L = outage.coverage_lengths(cl, gen, pmax, pvar, gamma, ess, soe, c["max_outage_duration"], c["dt"],
                                c["load_shed_pct"])
    return L, outage.lcp_curve(L, c["max_outage_duration"], c["dt"])

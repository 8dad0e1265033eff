"""GPU: the kernel cascade with its lists formed on the device (csrc/dvh_route.hip, dvh_api.cpp device_cascade) on a
batch that mixes every tier the drop-in can send at once (dervet/DERVET.py:75-83 puts every case's windows in one
batch): Usecase 3 market days, config-4 monthly windows, config-5 LP-relaxed ICE windows, POI + curtailable-PV
windows, annual hourly windows and the 5-minute annual window.  Each tier takes its windows (the next tier is sized for
the windows that reach it: the market days run on the small ELL kernel, the POI windows on the generic one), every window agrees
with HiGHS within 1e-5, and the host waits once per tier that ran.  scripts/ab_cascade.sh compares the same batch bit
for bit with the previous library (profiles/r03g_ab_cascade.log)."""
import numpy as np
import pytest
import scipy.sparse as sp

from dervet_hip.lp import builder, scenarios
from oracle import cases, window_lp

pytestmark = pytest.mark.gpu


def _mixed():
    arr, meta = cases.load_market()
    sig = {k.split("__", 1)[1]: v for k, v in arr.items() if k.startswith("es__")}
    out = [("market", [scenarios.market_days(sig, meta["es"]["params"], days=list(range(0, 365, 9)))]),
           ("config4", scenarios.config4(range(6))), ("config5", scenarios.config5(range(2), years=1))]
    wins, a, m, _ = cases.case_windows("es+pv+dg")
    gen = float(m["params"]["PV"]["rated_capacity"]) * np.nan_to_num(a["pv_profile"])
    out.append(("poi", scenarios.windows_by_period(2017, 1.0, a["site_load"][None], np.zeros_like(gen)[None],
                                                   cases.battery_from_params(m["params"]), tariff_def=m["tariff"],
                                                   ene_min=a["agg_emin"][None], ene_max=a["agg_emax"][None],
                                                   grid_charge=False, pv_curtail_max=(12.0 * gen)[None])[:3]))
    out.append(("annual", scenarios.config4([7], n="year")))
    return out


def test_mixed_batch_takes_every_tier_with_one_wait_per_tier(gpu_solver):
    gs = _mixed()
    lps = [lp for _, gl in gs for g in gl for lp in builder.group_window_lps(g)]
    n = {name: sum(g.G for g in gl) for name, gl in gs}
    res = gpu_solver.solve(lps)
    ks = gpu_solver.kernel_stats()
    assert ks["band_windows"] == n["config4"] + n["config5"], ks
    # the market days are few (<= two per CU) and take the four-wave small ELL variant; the POI windows fit no ELL
    # instantiation and end on the one-window-per-CU generic kernel
    assert ks["ell_windows"] == n["market"] and ks["generic_windows"] == n["poi"], ks
    assert ks["chain_windows"] == n["annual"] and ks["large_windows"] == 0, ks
    # band pass + ICE pass (its refusals' count, then their size classes once set up) + ELL pass read-backs, the
    # medium tier's plan / setup / team hand-offs, the final wait
    assert gpu_solver.host_syncs() <= 4 + 3 + 1, gpu_solver.host_syncs()
    rng = np.random.default_rng(0)
    k = 0
    for name, gl in gs:
        idx = list(range(k, k + n[name]))
        k += n[name]
        for i in sorted(rng.choice(idx, size=min(3, len(idx)), replace=False)):
            lp, r = lps[i], res[i]
            o = dict(K=sp.csr_matrix((lp.data, lp.indices, lp.indptr), shape=(lp.m, lp.n)), q=lp.q, c=lp.c,
                     c0=lp.c0, l=lp.l, u=lp.u, m_eq=lp.m_eq)
            h = window_lp.solve_highs(o)
            assert h["status"] == 0 and r.status == 0, (name, i, r.status_name)
            assert abs(r.obj - h["obj"]) <= 1e-5 * abs(h["obj"]), (name, i, r.obj, h["obj"])
            assert window_lp.primal_residual_rel(o, r.x)[0] <= 1e-6


def test_a_batch_the_band_kernel_takes_whole_waits_once_in_the_cascade(gpu_solver):
    """Host API: the band pass's read-back and the final wait for the results (no per-window host loop)."""
    lps = [lp for g in scenarios.config4(range(30)) for lp in builder.group_window_lps(g)]
    res = gpu_solver.solve(lps)
    assert all(r.status == 0 for r in res)
    assert gpu_solver.kernel_stats()["band_windows"] == 360
    assert gpu_solver.host_syncs() == 2, gpu_solver.host_syncs()


@pytest.mark.parametrize("days", [122, 1095])
def test_market_days_take_the_small_ell_kernel_at_every_batch_size(gpu_solver, days):
    """The four-wave small ELL variant (one column per lane, K and K^T in VGPRs, two windows per CU) takes the DA + FR
    days for few windows as for many (profiles/r05y_market_table.log: 3.6 vs 8.0 ms for 120 days against the generic
    kernel, 5.4 vs 11.3 ms for 1,095 against the round-4 one-wave variant)."""
    arr, meta = cases.load_market()
    names = ("es", "es+pv", "es+pv+dg")
    gl = []
    for nm in names:
        sig = {k.split("__", 1)[1]: v for k, v in arr.items() if k.startswith(nm + "__")}
        gl.append(scenarios.market_days(sig, meta[nm]["params"], name=nm,
                                        days=list(range(0, 365, 3 if days < 365 else 1))[:days // 3 + 1]))
    lps = [lp for g in gl for lp in builder.group_window_lps(g)][:days]
    res = gpu_solver.solve(lps)
    st = gpu_solver.kernel_stats()
    assert st["ell_windows"] == len(lps) and st["variant"] == 5680412, st
    assert all(r.status == 0 for r in res)

"""GPU parity for POI interconnection limits and PV grid_charge = 0 (PARITY UNPINNED formulations,
tests/test_poi_gridcharge.py): the golden es+pv+dg monthly windows with the rows added, built by the product builder
and solved on cuda:0 through the C ABI, against HiGHS on the same LP: objective within 1e-5, primal residual
<= 1e-6.  grid_charge = 0 with fixed PV only tightens ch's bounds (battery-banded kernel); POI rows and the
charge-from-PV rows with curtailable PV are extra >= rows per step: monthly windows of n = 4T + 1 = 2977 columns
with 3-4 entries per column, beyond the ELL kernels' LDS budget (K^T slots 4 x 3072), so they run on the on-chip
generic CSR kernel (same algorithm, one workgroup per window)."""
import numpy as np
import pytest
import scipy.sparse as sp

from dervet_hip.lp import builder, scenarios
from oracle import cases, window_lp

pytestmark = pytest.mark.gpu


def _groups(**kw):
    wins, arr, meta, _ = cases.case_windows("es+pv+dg")
    p = meta["params"]
    gen = float(p["PV"]["rated_capacity"]) * np.nan_to_num(arr["pv_profile"])
    bat = cases.battery_from_params(p)
    if kw.pop("big_curtailable_pv", False):
        kw["pv_curtail_max"] = (12.0 * gen)[None]
        gen = np.zeros_like(gen)
    return scenarios.windows_by_period(2017, 1.0, arr["site_load"][None], gen[None], bat, tariff_def=meta["tariff"],
                                       ene_min=arr["agg_emin"][None], ene_max=arr["agg_emax"][None], **kw)


def _check(groups, res):
    k = 0
    for g in groups:
        for i in range(g.G):
            r = res[k]
            k += 1
            o = dict(K=sp.csr_matrix((g.data[i], g.indices, g.indptr), shape=(g.m, g.n)), q=g.q[i], c=g.c[i],
                     c0=float(g.c0[i]), l=g.l[i], u=g.u[i], m_eq=g.m_eq)
            h = window_lp.solve_highs(o)
            assert h["status"] == 0 and r.status == 0, (k, r.status_name)
            assert abs(r.obj - h["obj"]) <= 1e-5 * abs(h["obj"]), (k, r.obj, h["obj"])
            assert window_lp.primal_residual_rel(o, r.x)[0] <= 1e-6


@pytest.mark.parametrize("variant", ["grid_charge_fixed_pv", "grid_charge_curtailable", "poi_no_export"])
def test_poi_and_grid_charge_windows_match_highs(gpu_solver, variant):
    if variant == "grid_charge_fixed_pv":
        groups = _groups(grid_charge=False)
        path = "band_windows"
    elif variant == "grid_charge_curtailable":
        groups = _groups(grid_charge=False, big_curtailable_pv=True)
        path = None
    else:
        groups = _groups(poi=dict(max_import=-12000.0, max_export=0.0), big_curtailable_pv=True)
        path = None
    lps = [lp for g in groups for lp in builder.group_window_lps(g)]
    res = gpu_solver.solve(lps)
    ks = gpu_solver.kernel_stats()
    if path:
        assert ks[path] == len(lps), ks
    else:
        assert ks["large_windows"] == 0 and ks["band_windows"] + ks["ell_windows"] + ks["generic_windows"] == len(lps), ks
    _check(groups, res)

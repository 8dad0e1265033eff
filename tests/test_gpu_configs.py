"""GPU parity on the BASELINE configurations and on edge cases, through the C ABI.

Each test builds windows with the product builder, solves them on cuda:0 with libdervet_hip and checks
against the oracle (restated LP + HiGHS, oracle/window_lp.py): objective within 1e-5 relative, primal
residual <= 1e-6 (recomputed here from the returned x).  Config 3 (one 105,120-step window) runs on the
grid-wide large-LP path (der-vet_amd/csrc/dvh_large.hip).
"""
import numpy as np
import pytest
import scipy.sparse as sp

from dervet_hip import BatchSolver, SolverError, WindowLP, pack
from dervet_hip.lp import builder, scenarios
from oracle import window_lp

pytestmark = pytest.mark.gpu

OBJ_TOL = 1e-5
PRES_TOL = 1e-6


def _oracle_lp(lp):
    K = sp.csr_matrix((lp.data, lp.indices, lp.indptr), shape=(lp.m, lp.n))
    return dict(K=K, q=lp.q, c=lp.c, c0=lp.c0, l=lp.l, u=lp.u, m_eq=lp.m_eq)


def _check(lps, res, what):
    worst = 0.0
    for k, (lp, r) in enumerate(zip(lps, res)):
        olp = _oracle_lp(lp)
        h = window_lp.solve_highs(olp)
        assert h["status"] == 0
        assert r.status == 0, f"{what} window {k}: {r.status_name} after {r.iters} iterations"
        pres, _ = window_lp.primal_residual_rel(olp, r.x)
        rel = abs(r.obj - h["obj"]) / max(abs(h["obj"]), 1e-9)
        worst = max(worst, rel)
        assert rel <= OBJ_TOL, f"{what} window {k}: objective rel err {rel:.2e}"
        assert pres <= PRES_TOL, f"{what} window {k}: primal residual {pres:.2e}"
    return worst


def _lps(groups):
    return [lp for g in groups for lp in builder.group_window_lps(g)]


def test_config1_da_windows(gpu_solver):
    lps = _lps(scenarios.config1())
    _check(lps, gpu_solver.solve(lps), "config1")


def test_config1_da_plus_retail(gpu_solver):
    lps = _lps(scenarios.config1(with_retail=True))
    _check(lps, gpu_solver.solve(lps), "config1+retail")


def test_config2_36_windows(gpu_solver):
    lps = _lps(scenarios.config2())
    assert len(lps) == 36
    _check(lps, gpu_solver.solve(lps), "config2")
    assert gpu_solver.kernel_stats()["band_windows"] == 36


def test_config4_sample_matches_highs(gpu_solver):
    lps = _lps(scenarios.config4([7, 1234, 9999]))
    _check(lps, gpu_solver.solve(lps), "config4")


def test_config5_band_ice_path(gpu_solver):
    """Config 5 (battery + LP-relaxed ICE + DCM, 744-step windows) takes the ICE variant of the band kernel."""
    g = scenarios.config5([3], years=1)
    lps = _lps([g[0], g[6]])
    res = gpu_solver.solve(lps)
    _check(lps, res, "config5")
    st = gpu_solver.kernel_stats()
    assert st["band_windows"] == 2 and st["variant"] == 9000112, st


def test_config5_band_ice_and_generic_kernels_agree():
    """ICE band kernel vs the generic CSR kernel on config-5 windows: same algorithm, objectives within 1e-7."""
    g = scenarios.config5([7], years=1)
    lps = _lps([g[1], g[9]])
    out = {}
    with BatchSolver(0) as s:
        for path, key in (("default", "band_windows"), ("generic", "generic_windows")):
            s.set_kernel_path(path)
            out[path] = s.solve(lps)
            assert s.kernel_stats()[key] == 2, (path, s.kernel_stats())
    for ra, rc in zip(out["default"], out["generic"]):
        assert ra.status == rc.status == 0
        assert abs(ra.obj - rc.obj) <= 1e-7 * abs(rc.obj)
        assert abs(ra.iters - rc.iters) <= 64


def test_band_ell_and_generic_kernels_agree():
    """The three kernels run the same algorithm on the same scaled LP: objectives within 1e-7, iteration counts
    within two check periods (summation orders differ)."""
    lps = _lps(scenarios.config4([42]))
    out = {}
    with BatchSolver(0) as s:
        for path, key in (("default", "band_windows"), ("ell", "ell_windows"), ("generic", "generic_windows")):
            s.set_kernel_path(path)
            out[path] = s.solve(lps)
            assert s.kernel_stats()[key] == 12, (path, s.kernel_stats())
    for ra, rb, rc in zip(out["default"], out["ell"], out["generic"]):
        assert ra.status == rb.status == rc.status == 0
        assert abs(ra.obj - rc.obj) <= 1e-7 * abs(rc.obj)
        assert abs(rb.obj - rc.obj) <= 1e-7 * abs(rc.obj)
        assert abs(ra.iters - rc.iters) <= 32 and abs(rb.iters - rc.iters) <= 32


@pytest.mark.parametrize("T", [743, 745, 768, 100, 2])
def test_band_kernel_forms_agree(T):
    """The battery band kernel's default form (3 steps per lane, 256 threads, two windows per CU) and its
    one-step-per-lane form (768 threads) run the same iteration; only the tau partial sums are grouped differently.
    Step counts T = 3k + 2 / 3k + 1 leave padding steps inside a lane; T = 768 fills every lane; two demand periods
    (J = 2, 4) take the per-column tau path.  Objectives within 1e-7 of each other (as the other cross-kernel checks;
    the realistic lengths agree to 1e-9) and 1e-5 of HiGHS; iteration counts within two check periods except on the
    degenerate two-step window, where the grouping of the sums moves the restart decisions."""
    rng = np.random.default_rng(T)
    G = 3
    load = 400 + 200 * rng.random((G, T))
    masks = np.zeros((2, T), bool)
    masks[0, : (T + 1) // 2] = True
    masks[1, (T + 1) // 2:] = True
    bat = dict(E=rng.uniform(500, 2000, G), Pch=rng.uniform(100, 400, G), Pdis=rng.uniform(100, 400, G),
               rte=rng.uniform(0.8, 0.95, G), sdr=rng.uniform(0, 1, G), soc_target=rng.uniform(0.3, 0.9, G),
               ulsoc=0.95, llsoc=0.05, fixedOM=10.0, OMexpenses=rng.uniform(0, 5, G))
    groups = [builder.battery_group(T, 1.0, load, bat, retail_price=rng.uniform(0.03, 0.2, (G, T)),
                                    demand_masks=masks[:1], demand_prices=rng.uniform(5, 20, (G, 1))),
              builder.battery_group(T, 1.0, load, bat, retail_price=rng.uniform(0.03, 0.2, (G, T)),
                                    demand_masks=masks, demand_prices=rng.uniform(5, 20, (G, 2)))]
    if T >= 4:  # J = 4 (the kernel's limit): four interleaved demand periods, every step in one of them
        m4 = np.zeros((4, T), bool)
        for j in range(4):
            m4[j, j::4] = True
        groups.append(builder.battery_group(T, 1.0, load, bat, retail_price=rng.uniform(0.03, 0.2, (G, T)),
                                            demand_masks=m4, demand_prices=rng.uniform(5, 20, (G, 4))))
    lps = _lps(groups)
    out = {}
    with BatchSolver(0) as s:
        for path, variant in (("band3", 9002004), ("band1", 9000012)):
            s.set_kernel_path(path)
            out[path] = s.solve(lps)
            st = s.kernel_stats()
            assert st["band_windows"] == len(lps) and st["variant"] == variant, (path, st)
    for ra, rb in zip(out["band3"], out["band1"]):
        assert ra.status == rb.status == 0
        assert abs(ra.obj - rb.obj) <= (1e-9 if T >= 100 else 1e-7) * max(1.0, abs(rb.obj))
        assert T < 100 or abs(ra.iters - rb.iters) <= 64
    _check(lps, out["band3"], f"band form 3, T={T}")


def test_band_kernel_form_follows_batch_size():
    """The default cascade runs a batch of at most one battery window per CU in the one-step form (a lone window
    is faster there) and larger batches in the three-step, two-windows-per-CU form."""
    import torch
    small = _lps(scenarios.config1())
    big = pack(_lps(scenarios.config4(range(30)))).to_torch("cuda:0").alloc_outputs()  # 360 windows > 256 CUs
    with BatchSolver(0) as s:
        _check(small, s.solve(small), "config1 one-step")
        assert s.kernel_stats()["variant"] == 9000012, s.kernel_stats()
        s.solve_packed(big)
        torch.cuda.synchronize()
        st = s.kernel_stats()
        assert st["variant"] == 9002004 and st["band_windows"] == 360, st
        assert (big.istats.cpu().numpy()[:, 0] == 0).all()


@pytest.mark.parametrize("path", ["band1", "band3", "ell"])
def test_kkt_predict_only_delays_termination(path):
    """dvh_options.kkt_predict skips due KKT checks without touching the iterates (restarts depend on the
    fixed-point residual only): every window ends at the same or a later check (later by more than the 4 skipped
    checks where a check the plain run passed is skipped and the next ones fail: the KKT error is not monotone),
    bit-identical where the iteration counts agree, and still passes the same termination test."""
    lps = _lps(scenarios.config4(range(24)))
    s = BatchSolver(0)
    try:
        s.set_kernel_path(path)
        s.set_options(check_every=64, kkt_every=1)
        plain = s.solve(lps)
        s.set_options(kkt_predict=4)
        pred = s.solve(lps)
        assert s.kernel_stats()["ell_windows" if path == "ell" else "band_windows"] == len(lps)
    finally:
        s.close()
    delay = []
    for a, b in zip(plain, pred):
        assert a.status == 0 and b.status == 0
        assert a.iters <= b.iters and (b.iters - a.iters) % 64 == 0, (a.iters, b.iters)
        delay.append(b.iters - a.iters)
        if a.iters == b.iters:
            assert a.obj == b.obj and np.array_equal(a.x, b.x) and np.array_equal(a.y, b.y)
        else:  # both passed the same termination test, at different checks
            assert abs(a.obj - b.obj) <= 2e-6 * max(1.0, abs(a.obj))
    assert np.mean(delay) <= 64, np.mean(delay)
    _check(lps[::23], pred[::23], f"kkt_predict {path}")
    bad = BatchSolver(0)
    try:
        with pytest.raises(SolverError, match="kkt_predict"):
            bad.set_options(kkt_predict=-1)
    finally:
        bad.close()


def test_band_kernel_config1_no_dcm(gpu_solver):
    """Config 1 (DA arbitrage, no demand charge: J = 0, no >= rows) takes the battery-banded kernel."""
    lps = _lps(scenarios.config1())
    _check(lps, gpu_solver.solve(lps), "config1-band")
    assert gpu_solver.kernel_stats()["band_windows"] == len(lps)


def test_packed_device_path_equals_host_path(gpu_solver):
    import torch
    lps = _lps(scenarios.config4([5, 6]))
    host = gpu_solver.solve(lps)
    dev = pack(lps).to_torch("cuda:0").alloc_outputs()
    gpu_solver.solve_packed(dev)
    torch.cuda.synchronize()
    st = dev.stats.cpu().numpy()
    ist = dev.istats.cpu().numpy()
    x = dev.x.cpu().numpy()
    off = 0
    for k, (lp, r) in enumerate(zip(lps, host)):
        assert st[k, 0] == r.obj and ist[k, 0] == r.status and ist[k, 1] == r.iters
        assert np.array_equal(x[off:off + lp.n], r.x)
        off += lp.n


def test_results_are_bitwise_reproducible(gpu_solver):
    lps = _lps(scenarios.config4([11]))
    a = gpu_solver.solve(lps)
    b = gpu_solver.solve(lps)
    for ra, rb in zip(a, b):
        assert np.array_equal(ra.x, rb.x) and np.array_equal(ra.y, rb.y) and ra.iters == rb.iters


def test_randomised_battery_parameters(gpu_solver):
    """Unpinned features: sdr, soc_target, ulsoc/llsoc, hp, curtailable PV, two demand periods."""
    rng = np.random.default_rng(3)
    T, G = 168, 4
    load = 400 + 200 * rng.random((G, T))
    masks = np.zeros((2, T), bool)
    masks[0, ::2] = True
    masks[1, 1::2] = True
    bat = dict(E=rng.uniform(500, 2000, G), Pch=rng.uniform(100, 400, G), Pdis=rng.uniform(100, 400, G),
               rte=rng.uniform(0.8, 0.95, G), sdr=rng.uniform(0, 1, G), soc_target=rng.uniform(0.3, 0.9, G),
               ulsoc=0.95, llsoc=0.05, fixedOM=10.0, OMexpenses=rng.uniform(0, 5, G), hp=rng.uniform(0, 20, G))
    g = builder.battery_group(T, 1.0, load, bat, retail_price=rng.uniform(0.03, 0.2, (G, T)),
                              demand_masks=masks, demand_prices=rng.uniform(5, 20, (G, 2)),
                              pv_curtail_max=rng.uniform(0, 300, (G, T)))
    lps = builder.group_window_lps(g)
    _check(lps, gpu_solver.solve(lps), "random")


def test_tiny_and_equality_only_lps(gpu_solver):
    # min x0 + 2 x1  s.t. x0 + x1 = 1, 0 <= x <= 1  -> obj 1
    lp1 = WindowLP(np.array([0, 2], np.int32), np.array([0, 1], np.int32), np.array([1.0, 1.0]),
                   np.array([1.0, 2.0]), np.array([1.0]), np.zeros(2), np.ones(2), 1, 0.5)
    # min -x  s.t. x >= 0.25 (as a >= row), x <= 1  -> obj -1
    lp2 = WindowLP(np.array([0, 1], np.int32), np.array([0], np.int32), np.array([1.0]), np.array([-1.0]),
                   np.array([0.25]), np.zeros(1), np.ones(1), 0, 0.0)
    r = gpu_solver.solve([lp1, lp2])
    assert r[0].status == 0 and abs(r[0].obj - 1.5) < 1e-6 and abs(r[0].x[0] - 1.0) < 1e-6
    assert r[1].status == 0 and abs(r[1].obj + 1.0) < 1e-6


def test_infeasible_window_is_not_reported_optimal():
    # x0 + x1 = 3 with 0 <= x <= 1: primal infeasible
    lp = WindowLP(np.array([0, 2], np.int32), np.array([0, 1], np.int32), np.array([1.0, 1.0]),
                  np.array([1.0, 1.0]), np.array([3.0]), np.zeros(2), np.ones(2), 1, 0.0)
    with BatchSolver(0, max_iters=4096) as s:
        r = s.solve([lp])[0]
    assert r.status != 0 and r.primal_res_rel > 1e-6


@pytest.mark.parametrize("path", ["default", "ell", "generic"])
def test_crossed_bounds_window_reported_infeasible_on_every_kernel_path(path):
    """A window with l_j > u_j (a reliability requirement above E) is PRIMAL_INFEASIBLE at 0 iterations from the
    setup kernel; no PDHG kernel overwrites it and its neighbours solve as alone (oracle/cpu_pdhg.cpp applies the
    same rule)."""
    import dataclasses
    lps = _lps(scenarios.config4([3]))[:4]
    T = lps[2].m_eq - 1
    bad_l = lps[2].l.copy()
    bad_l[2 * T + 7] = lps[2].u[2 * T + 7] + 10.0
    bad = list(lps)
    bad[2] = dataclasses.replace(lps[2], l=bad_l)
    with BatchSolver(0) as s:
        s.set_kernel_path(path)
        ref = s.solve(lps)
        res = s.solve(bad)
    assert res[2].status_name == "infeasible" and res[2].iters == 0
    for k in (0, 1, 3):
        assert res[k].status == 0 and res[k].obj == ref[k].obj and res[k].iters == ref[k].iters


def test_invalid_inputs_raise_with_message(gpu_solver):
    bad = WindowLP(np.array([0, 1], np.int32), np.array([5], np.int32), np.array([1.0]), np.array([1.0, 1.0]),
                   np.array([1.0]), np.zeros(2), np.ones(2), 1, 0.0)
    with pytest.raises(SolverError, match="column index"):
        gpu_solver.solve([bad])
    nanlp = WindowLP(np.array([0, 1], np.int32), np.array([0], np.int32), np.array([np.nan]), np.array([1.0]),
                     np.array([1.0]), np.zeros(1), np.ones(1), 1, 0.0)
    with pytest.raises(SolverError, match="non-finite"):
        gpu_solver.solve([nanlp])


def _config3_da():
    g = scenarios.config3("da")
    assert g[0].T == 105120
    return g


def test_config3_annual_5min_window_large_path(gpu_solver):
    """BASELINE config 3: one 105,120-step annual window (n = 315,360) on the grid-wide large-LP path (the band
    kernels off, so the medium tier is off too; the default route is the long team, tests/test_gpu_config3.py)."""
    lps = _lps(_config3_da())
    assert lps[0].n == 3 * 105120
    gpu_solver.set_kernel_path("ell")
    try:
        res = gpu_solver.solve(lps)
        assert gpu_solver.kernel_stats()["large_windows"] == 1
    finally:
        gpu_solver.set_kernel_path("default")
    _check(lps, res, "config3")


def test_large_path_with_dcm_columns_in_mixed_batch():
    """An annual hourly window with 12 monthly DCM tau columns batched together with monthly windows: each goes to
    its path -- the medium tier (dvh_chain.hip) by default, the grid-wide large-LP path when the band kernels are off
    -- and all match HiGHS."""
    ri = scenarios.reference_inputs()
    load = ri["multi_der_site_load"][None, :]
    gen = 1000.0 * np.nan_to_num(ri["multi_der_pv_profile"])[None, :]
    annual = scenarios.windows_by_period(2017, 1.0, load, gen, scenarios.config2_battery(), tariff_def=scenarios.tariff(),
                                         n="year")
    lps = _lps(scenarios.config4([3])[:2]) + _lps(annual) + _lps(scenarios.config4([4])[:1])
    assert lps[2].n == 3 * 8760 + 12
    with BatchSolver(0) as s:
        res = s.solve(lps)
        ks = s.kernel_stats()
        assert ks["chain_windows"] == 1 and ks["band_windows"] == 3 and ks["large_windows"] == 0, ks
        _check(lps, res, "mixed")
        s.set_kernel_path("ell")
        res = s.solve(lps)
        ks = s.kernel_stats()
        assert ks["large_windows"] == 1 and ks["ell_windows"] == 3, ks
        _check(lps, res, "mixed-large")


def test_warm_start_from_own_solution_and_neighbour():
    """warm_start: windows started at their own solution need far fewer iterations than cold starts (the
    relative KKT test sits at 1e-6, so a few restart periods are still needed) and end at the HiGHS optimum;
    started from another scenario's solution of the same month they still converge to the HiGHS optimum
    (battery-banded kernel)."""
    lps = _lps(scenarios.config4([11, 12]))
    with BatchSolver(0) as s:
        cold = s.solve(lps)
        s.set_options(warm_start=1)
        own = s.solve(lps, start=[(r.x, r.y) for r in cold])
        assert s.kernel_stats()["band_windows"] == len(lps)
        nb = s.solve(lps, start=[(cold[k ^ 1].x, cold[k ^ 1].y) for k in range(len(lps))])  # other scenario
    assert all(r.status == 0 for r in own)
    assert sum(r.iters for r in own) < 0.6 * sum(r.iters for r in cold), ([r.iters for r in own], [r.iters for r in cold])
    _check(lps, own, "config4-warm-own")
    _check(lps, nb, "config4-warm-neighbour")


def test_multi_device_handle_splits_batch_and_matches_single_device():
    """A handle over several devices (device_mask / dvh_create_devices; device 0 repeated on a one-GPU box) splits a
    host batch into cost-balanced contiguous ranges solved concurrently: results bit-identical to one device, path
    counts summed, an annual window costing as many monthly windows as its nonzeros."""
    from dervet_hip.lp import scenarios as sc
    ri = sc.reference_inputs()
    load = ri["multi_der_site_load"][None, :]
    gen = 1000.0 * np.nan_to_num(ri["multi_der_pv_profile"])[None, :]
    annual = sc.windows_by_period(2017, 1.0, load, gen, sc.config2_battery(), tariff_def=sc.tariff(), n="year")
    lps = _lps(sc.config4(range(6))) + _lps(annual) + _lps(sc.config2())
    with BatchSolver(0) as one:
        r1 = one.solve(lps)
        k1 = one.kernel_stats()
    with BatchSolver(devices=[0, 0, 0]) as three:
        assert three.device_count == 3
        r3 = three.solve(lps)
        k3 = three.kernel_stats()
    for a, b in zip(r1, r3):
        assert a.status == b.status and a.iters == b.iters and a.obj == b.obj
        assert np.array_equal(a.x, b.x) and np.array_equal(a.y, b.y)
    for key in ("band_windows", "ell_windows", "generic_windows", "large_windows"):
        assert k1[key] == k3[key], (key, k1, k3)
    _check(lps[::7], r3[::7], "multi-device")

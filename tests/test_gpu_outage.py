"""GPU reliability sweep (dvh_outage_coverage) vs the oracle and the reference's golden curves: covered
lengths bit-exact per start step, load coverage probability curves bit-exact."""
import numpy as np
import pytest

import outage_cases
from dervet_hip import reliability

pytestmark = pytest.mark.gpu


def _case(c):
    return reliability.OutageCase(critical_load=c["critical_load"], dt=c["dt"],
                                  max_outage_duration=c["max_outage_duration"], ess=c["ess"], init_soe=c["init_soe"],
                                  soc_init=c["soc_init"], pv_max=c["pv_max"], pv_nu=c["pv_nu"],
                                  pv_gamma=c["pv_gamma"], load_shed_pct=c["load_shed_pct"])


def test_golden_cases_bit_exact(gpu_solver):
    cases = outage_cases.load()
    names = sorted(cases)
    lengths, curves = reliability.outage_coverage([_case(cases[n]) for n in names], gpu_solver)
    for n, L, lcp in zip(names, lengths, curves):
        Lo, _ = outage_cases.oracle_curve(cases[n])
        np.testing.assert_array_equal(L, Lo, err_msg=n)
        np.testing.assert_array_equal(lcp, cases[n]["golden_lcp"], err_msg=n)
    dfs = reliability.load_coverage_probability([_case(cases["uc2_es"])], gpu_solver)
    assert list(dfs[0].columns) == ["Load Coverage Probability (%)"] and dfs[0].index.name == "Outage Length (hrs)"
    assert len(dfs[0]) == 80 and dfs[0].index[0] == 1.0


def _random_case(rng, N, dt=1.0, max_out=24, pv=True, dg=True, shed=True, soe_series=True):
    cl = rng.uniform(200.0, 1500.0, N).round(5)
    E = float(rng.uniform(500, 6000))
    ess = dict(E=E, P_ch=E / rng.uniform(2, 6), P_dis=E / rng.uniform(2, 6), rte=float(rng.uniform(0.8, 0.95)),
               llsoc=float(rng.uniform(0, 0.2)), ulsoc=float(rng.uniform(0.85, 1.0)))
    pvs = [np.maximum(0.0, rng.normal(600, 400, N))] if pv else []
    return reliability.OutageCase(
        critical_load=cl, dt=dt, max_outage_duration=max_out, ess=ess,
        init_soe=rng.uniform(0, E, N) if soe_series else None, soc_init=float(rng.uniform(0.3, 1.0)),
        pv_max=pvs, pv_nu=[float(rng.uniform(0.2, 1.0))] if pv else [], pv_gamma=[float(rng.uniform(0.3, 1.0))] if pv else [],
        dg_power=[float(rng.uniform(0, 600))] if dg else [],
        load_shed_pct=rng.choice([100.0, 80.0, 50.0, 30.0], size=max_out) if shed else None)


def _oracle(c):
    from oracle import outage
    dg, pmax, props, pvar, gamma = reliability.der_mix_properties(c)
    gen = np.repeat(dg, len(c.critical_load))
    soe = c.init_soe if c.init_soe is not None else c.soc_init * props["energy rating"]
    L = outage.coverage_lengths(np.asarray(c.critical_load), gen, pmax, pvar, gamma, props, soe,
                                c.max_outage_duration, c.dt, c.load_shed_pct)
    return L, outage.lcp_curve(L, c.max_outage_duration, c.dt)


def test_randomised_cases_bit_exact(gpu_solver):
    """PV (nu, gamma), generators, load-shed multipliers, llsoc / ulsoc limits, SOE series or soc_init, short
    series (N < max outage), dt = 0.5 -- every covered length equals the oracle's."""
    rng = np.random.default_rng(20250217)
    cases = [_random_case(rng, 700), _random_case(rng, 700, pv=False), _random_case(rng, 700, dg=False, shed=False),
             _random_case(rng, 700, soe_series=False), _random_case(rng, 13, max_out=40),
             _random_case(rng, 300, dt=0.5, max_out=12)]
    lengths, curves = reliability.outage_coverage(cases, gpu_solver)
    for k, (c, L, lcp) in enumerate(zip(cases, lengths, curves)):
        Lo, lo = _oracle(c)
        np.testing.assert_array_equal(L, Lo, err_msg=f"case {k}")
        np.testing.assert_array_equal(lcp, lo[:len(lcp)], err_msg=f"case {k}")
        assert len(np.unique(L)) > 1 or k == 4, f"case {k} exercises only one outcome"


def test_invalid_case_raises(gpu_solver):
    bad = reliability.OutageCase(critical_load=np.ones(10), dt=1.0, max_outage_duration=0, ess=dict(E=1, rte=0.9))
    with pytest.raises(Exception, match="max_outage >= dt"):
        reliability.outage_coverage([bad], gpu_solver)


def test_min_soe_bit_exact(gpu_solver):
    """Reliability.min_soe_iterative (the config-5 'Reliability Min State of Energy' requirement) on the golden
    sites and randomized cases: every start's soe_used equals the oracle's (parity unpinned vs the reference:
    no reference run writes this column)."""
    from oracle import outage
    golden = outage_cases.load()
    rng = np.random.default_rng(7)
    cases = [_case(golden["uc2_es+pv"]), _case(golden["ls_w_ls1"]), _random_case(rng, 600),
             _random_case(rng, 400, pv=False, shed=False), _random_case(rng, 9, max_out=30)]
    targets = [4, 4, 6, 3, 12]
    got = reliability.min_soe(cases, targets, gpu_solver)
    for k, (c, tgt, g) in enumerate(zip(cases, targets, got)):
        dg, pmax, props, pvar, gamma = reliability.der_mix_properties(c)
        ref = outage.min_soe(np.asarray(c.critical_load, np.float64), np.repeat(dg, len(pmax)), pmax, pvar, gamma,
                             props, c.soc_init, tgt, c.max_outage_duration, c.dt, c.load_shed_pct)
        np.testing.assert_array_equal(g, ref, err_msg=f"case {k}")
        assert (g >= 0).all()
    assert got[0].max() > 0


def test_config5_min_soe_from_the_gpu_outage_kernel_feeds_the_windows(gpu_solver):
    """BASELINE config 5 end to end (row a10): the 'Reliability Min State of Energy' requirement of each scenario
    is computed by dvh_outage_min_soe (bit-exact with the oracle restatement of Reliability.min_soe_iterative) and
    applied as every window's ene lower bound; the windows solve to the HiGHS optimum on the battery-banded ICE
    kernel.  With the ICE units in the outage mix they carry the critical load alone and the requirement is 0."""
    import scipy.sparse as sp
    from dervet_hip.lp import builder, scenarios
    from oracle import outage, window_lp
    ids = [0, 1, 2]
    ms = scenarios.config5_min_soe(ids, gpu_solver)
    assert ms.shape == (3, 8760) and ms.max() > 0
    for c, g in zip(scenarios.config5_outage_cases(ids), ms):
        dg, pmax, props, pvar, gamma = reliability.der_mix_properties(c)
        ref = outage.min_soe(np.asarray(c.critical_load, np.float64), np.repeat(dg, len(pmax)), pmax, pvar, gamma,
                             props, c.soc_init, 4, c.max_outage_duration, c.dt, c.load_shed_pct)
        np.testing.assert_array_equal(g, ref)
    assert scenarios.config5_min_soe(ids, gpu_solver, count_ice=True).max() == 0.0
    E = scenarios.sweep_parameters(ids)["E"]
    for cap in (False, True):
        groups = scenarios.config5(ids, years=1, min_soe=ms, cap_min_soe=cap)
        lps = [lp for g in groups for lp in builder.group_window_lps(g)]
        res = gpu_solver.solve(lps)
        assert gpu_solver.kernel_stats()["band_windows"] == len(lps)
        k = 0
        seen = set()
        for g in groups:
            T = g.T
            for i in range(g.G):
                r = res[k]
                k += 1
                req = ms[i][g.index]
                # the requirement is the ene lower bound (clipped at E with cap)
                assert np.array_equal(g.l[i][2 * T:3 * T], np.minimum(req, E[i]) if cap else req)
                crossed = not cap and bool((req > E[i]).any())
                if crossed:  # infeasible as stated: reported at once, no iterations
                    assert r.status_name == "infeasible" and r.iters == 0, (k, r.status_name)
                else:
                    assert r.status == 0, (k, r.status_name)
                if (crossed, i) in seen:
                    continue
                seen.add((crossed, i))
                o = dict(K=sp.csr_matrix((g.data[i], g.indices, g.indptr), shape=(g.m, g.n)), q=g.q[i], c=g.c[i],
                         c0=float(g.c0[i]), l=g.l[i], u=g.u[i], m_eq=g.m_eq)
                if crossed:
                    continue  # HiGHS rejects crossed bounds outright; nothing further to compare
                h = window_lp.solve_highs(o)
                assert h["status"] == 0 and abs(r.obj - h["obj"]) <= 1e-5 * abs(h["obj"]), (k, r.obj, h["obj"])
                assert window_lp.primal_residual_rel(o, r.x)[0] <= 1e-6

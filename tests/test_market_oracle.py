"""Market-service windows: DA + frequency regulation, daily, binary = 1.

The reference's storagevet FrequencyRegulation / EnergyStorage formulation is absent; the oracle
restates it (oracle/window_lp.py) and these tests pin that restatement to the reference's own Usecase 3 goldens
(test/test_validation_report_sept1/Results/Usecase3/planned/step2/{es,es+pv,es+pv+dg}: 365 daily windows each,
fixtures tests/golden/uc3_market.* from tests/golden/make_fixtures.py):
  * the objective terms evaluated on the golden dispatch reproduce every golden objective_values row;
  * the golden dispatch is feasible in the restated constraints;
  * the restated MILP (binary on_c / on_d, as GLPK_MI solves it there) reaches the golden optimum exactly, so
    the constraint set is complete (a missing row would let it go lower, an extra one would push it higher);
  * the opt-in LP relaxation (what the GPU solves) is a lower bound of every golden day.
The product's vectorised builder (dervet_hip.lp.builder.market_group) emits the same LP as the oracle.
"""
import numpy as np
import pytest

from dervet_hip.lp import scenarios
from oracle import cases, window_lp

CASES = ["es", "es+pv", "es+pv+dg"]


def _signals(name):
    arr, meta = cases.load_market()
    return {k.split("__", 1)[1]: v for k, v in arr.items() if k.startswith(name + "__")}, meta[name]


@pytest.mark.parametrize("name", CASES)
def test_golden_dispatch_reproduces_objective_rows_and_is_feasible(name):
    wins, keys = cases.market_windows(name)
    assert keys == ["DA", "regup_prof", "regdown_prof", "fr_energy_settlement", "es fixed_om", "es var_om"]
    assert len(wins) == 365
    for d, w in enumerate(wins):
        lp = window_lp.build(dict(w, binary_relax=False))
        terms = window_lp.evaluate_terms(lp, w["x_golden"])
        got = np.array([terms[k] for k in keys])
        assert np.all(np.abs(got - w["golden_objective"]) <= 1e-9 * (1.0 + np.abs(w["golden_objective"]))), (name, d)
        _, viol = window_lp.primal_residual_rel(lp, w["x_golden"])
        assert viol <= 1e-6, (name, d, viol)


@pytest.mark.parametrize("name", CASES)
def test_milp_restatement_reaches_golden_optimum(name):
    wins, _ = cases.market_windows(name)
    for d in range(0, 365, 23):
        r = window_lp.solve_highs_milp(wins[d])
        assert r["status"] == 0
        g = wins[d]["golden_objective"].sum()
        assert abs(r["obj"] - g) <= 1e-9 * (1.0 + abs(g)), (name, d, r["obj"], g)


@pytest.mark.parametrize("name", CASES)
def test_lp_relaxation_bounds_every_golden_day(name):
    wins, _ = cases.market_windows(name)
    gaps = []
    for w in wins:
        h = window_lp.solve_highs(window_lp.build(w))
        assert h["status"] == 0
        g = w["golden_objective"].sum()
        gaps.append((g - h["obj"]) / (1.0 + abs(g)))
    gaps = np.array(gaps)
    assert gaps.min() >= -1e-9
    assert gaps.max() < 5e-3  # the relaxation stays within 0.5 % of the MILP optimum on these cases


@pytest.mark.parametrize("name", CASES)
def test_builder_matches_oracle(name):
    sig, meta = _signals(name)
    days = [0, 1, 100, 200, 364]
    g = scenarios.market_days(sig, meta["params"], days=days)
    wins, keys = cases.market_windows(name)
    for k, d in enumerate(days):
        o = window_lp.build(wins[d])
        K = np.zeros((g.m, g.n))
        for r in range(g.m):
            K[r, g.indices[g.indptr[r]:g.indptr[r + 1]]] = g.data[k, g.indptr[r]:g.indptr[r + 1]]
        assert g.m_eq == o["m_eq"] and K.shape == o["K"].shape
        assert np.abs(K - o["K"].toarray()).max() <= 1e-14
        # u/d_ts maxima above P_ch + P_dis are clamped to it by the builder (an implied bound, same feasible set)
        T = o["T"]
        cap = -(o["u"][0] + o["u"][T])
        qb = np.where(o["q"] < cap, cap, o["q"])
        qb[:o["m_eq"]] = o["q"][:o["m_eq"]]
        for a, b in ((g.q[k], qb), (g.c[k], o["c"]), (g.l[k], o["l"]), (g.u[k], o["u"])):
            assert np.array_equal(a, b) or np.abs(a - b).max() <= 1e-12
        assert abs(g.c0[k] - o["c0"]) <= 1e-9
        x = wins[d]["x_golden"]
        for key in keys:
            coef, const = g.terms[key]
            assert abs(coef[k] @ x + const[k] - wins[d]["golden_objective"][keys.index(key)]) <= 1e-8

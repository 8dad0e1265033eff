"""Battery degradation (dervet_hip/degradation.py; parity UNPINNED: storagevet's BatteryTech module is absent) and
the degradation-coupled sweep on CPU.  Rainflow counting is pinned by ASTM E1049-85's worked example; the vectorised
counter equals the scalar restatement (oracle/rainflow_ref.py) bit for bit; the lockstep sweep (window position k of
every scenario in one batch) equals a scenario-by-scenario serial loop with the same solver."""
import numpy as np
import pytest

from dervet_hip import degradation
from dervet_hip.lp import scenarios
from oracle import rainflow_ref


def test_rainflow_astm_example():
    # ASTM E1049-85, rainflow counting example: loads -2, 1, -3, 5, -1, 3, -4, 4, -2
    got = rainflow_ref.count_cycles([-2, 1, -3, 5, -1, 3, -4, 4, -2])
    assert got == [(3, 0.5), (4, 1.5), (6, 0.5), (8, 1.0), (9, 0.5)]


def test_rainflow_reversals_flat_runs_and_ends():
    assert rainflow_ref.reversals([0, 1, 1, 2, 1, 1, 0, 0, 3]) == [0, 3, 6, 8]
    assert rainflow_ref.cycles([5, 5]) == [(0, 0.5)]


def _oracle_damage(series, e_rated, upper, life):
    d = 0.0
    for r, c in rainflow_ref.cycles(series):
        idx = min(int(np.searchsorted(upper, r / e_rated, side="left")), len(upper) - 1)
        d += c / life[idx]
    return d


def test_vectorised_cycle_damage_equals_scalar_restatement():
    rng = np.random.default_rng(5)
    upper, life = degradation.cycle_life_table()
    S, T = 40, 300
    x = np.cumsum(rng.normal(size=(S, T)), axis=1) * 50 + 2000
    x[:, 50:60] = x[:, 49:50]          # plateaus
    x[3] = 1000.0                       # flat profile: one zero-range half cycle
    x[7, ::2] += 300.0                  # sawtooth
    E = rng.uniform(3000, 6000, S)
    got = degradation.cycle_damage(x, E, upper, life)
    for i in range(S):
        assert got[i] == _oracle_damage(x[i], E[i], upper, life), i


def test_degradation_update_and_replacement():
    upper, life = degradation.cycle_life_table()
    d = degradation.Degradation([1000.0, 1000.0], yearly_degrade=2.0, state_of_health=80.0,
                                replaceable=[True, False], eol_condition=80.0)
    full = np.tile(np.array([0.0, 1000.0]), (2, 10))   # 10 full 100 % cycles (9.5 full + half cycles)
    step = d.update(full, days=30.0)
    cyc = _oracle_damage(full[0], 1000.0, upper, life) * 0.2
    assert step[0] == pytest.approx(0.02 * 30 / 365 + cyc, rel=1e-15)
    for _ in range(400):  # wear both batteries below 80 % state of health
        d.update(full, days=30.0)
    assert d.replacements[0] >= 1 and d.replacements[1] == 0
    assert d.capacity()[1] <= 800.0 and d.capacity()[0] > 800.0


def test_lockstep_sweep_equals_serial_loop_on_cpu_restatement():
    from oracle.cpu_pdhg import CpuPdhgSolver
    ids = [0, 1, 2]
    P = scenarios.sweep_parameters(ids)
    solver = CpuPdhgSolver(threads=3)

    def run(scen, E):
        deg = degradation.Degradation(E, yearly_degrade=1.0)
        sw = degradation.DegradationSweep(lambda k, cap: scenarios.config4(scen, E=cap, only=[k]), [0, 1, 2], deg)
        return sw.run(solver, device=None), deg

    batched, deg = run(ids, P["E"])
    assert all((p["status"] == 0).all() for p in batched)
    assert (deg.degrade_perc > 0).all() and (batched[2]["capacity_before"] < P["E"]).all()
    for i, s in enumerate(ids):
        alone, _ = run([s], P["E"][i:i + 1])
        for pb, pa in zip(batched, alone):
            # same LP, same solver arithmetic: identical dispatch and wear; the objective's constant (numpy's row sum
            # of the fixed net-load cost) may differ in the last bit with the batch shape
            assert np.array_equal(pb["ene"][i], pa["ene"][0]) and pb["iters"][i] == pa["iters"][0]
            assert pb["degradation"][i] == pa["degradation"][0]
            assert pb["obj"][i] == pytest.approx(pa["obj"][0], rel=1e-14)

"""GPU: the degradation-coupled sweep (dervet_hip/degradation.py; parity UNPINNED beyond HiGHS on each window) --
window position k of every scenario in one batched solve, capacities updated from the solved SOE profiles before
position k + 1 is built.  Equals the scenario-by-scenario serial loop on the same GPU bit for bit (dispatch, wear);
every window optimal and within 1e-5 of HiGHS on a sample; the capacity only shrinks."""
import numpy as np
import pytest
import scipy.sparse as sp

from dervet_hip import degradation
from dervet_hip.lp import builder, scenarios
from oracle import window_lp

pytestmark = pytest.mark.gpu


def _sweep(ids, E, solver, positions):
    deg = degradation.Degradation(E, yearly_degrade=2.0)
    sw = degradation.DegradationSweep(lambda k, cap: scenarios.config4(ids, E=cap, only=[k]), positions, deg)
    return sw.run(solver), deg


def test_lockstep_sweep_matches_serial_and_highs(gpu_solver):
    ids = list(range(16))
    P = scenarios.sweep_parameters(ids)
    out, deg = _sweep(ids, P["E"], gpu_solver, range(12))
    assert all((p["status"] == 0).all() for p in out)
    caps = np.stack([p["capacity_before"] for p in out])
    assert (np.diff(caps, axis=0) <= 0).all() and (deg.capacity() < P["E"]).all()
    for i in (0, 7):
        alone, _ = _sweep([ids[i]], P["E"][i:i + 1], gpu_solver, range(12))
        for pb, pa in zip(out, alone):
            assert np.array_equal(pb["ene"][i], pa["ene"][0]) and pb["iters"][i] == pa["iters"][0]
            assert pb["degradation"][i] == pa["degradation"][0]
    # position 6 with the degraded capacities, against HiGHS
    g = scenarios.config4(ids, E=out[6]["capacity_before"], only=[6])[0]
    for i in (0, 5, 11):
        o = dict(K=sp.csr_matrix((g.data[i], g.indices, g.indptr), shape=(g.m, g.n)), q=g.q[i], c=g.c[i],
                 c0=float(g.c0[i]), l=g.l[i], u=g.u[i], m_eq=g.m_eq)
        h = window_lp.solve_highs(o)
        assert abs(out[6]["obj"][i] - h["obj"]) <= 1e-5 * abs(h["obj"])


def test_device_built_sweep_equals_host_built(gpu_solver):
    """The same sweep with every position's windows expanded on the GPU (lp/gpu_builder.py): identical results."""
    ids = list(range(6))
    P = scenarios.sweep_parameters(ids)
    host, dh = _sweep(ids, P["E"], gpu_solver, range(4))
    deg = degradation.Degradation(P["E"], yearly_degrade=2.0)
    sw = degradation.DegradationSweep(lambda k, cap: scenarios.config4(ids, E=cap, only=[k], spec=True), range(4), deg)
    dev = sw.run(gpu_solver)
    for a, b in zip(host, dev):
        for f in ("ene", "iters", "status", "obj", "degradation", "capacity_before"):
            assert np.array_equal(a[f], b[f]), f
    assert np.array_equal(dh.capacity(), deg.capacity())

"""POI interconnection limits and PV grid_charge = 0.

Both live in the absent storagevet (POI.optimization_problem, extended at dervet/MicrogridPOI.py:215-258; PV
``grid_charge``, Schema.json:1875; Scenario ``apply_interconnection_constraints`` / ``max_import`` / ``max_export``,
Schema.json:2123,2194,2199) and no reference result has them active: PARITY UNPINNED.  Restated independently in
oracle/window_lp.py (build: ``poi``, ``grid_charge``) and the product builder; checked here that the builder emits
the oracle's LP entry for entry and that the HiGHS optimum has the properties the rows mean (limits hold, a binding
limit never lowers the cost, charging stays within the PV).  GPU parity: tests/test_gpu_poi.py.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from dervet_hip.lp import builder
from oracle import cases, window_lp


def _window(name="es+pv+dg", k=3):
    wins, _, meta, _ = cases.case_windows(name)
    return wins[k]


def _builder(w, **kw):
    base = w["load"] - w["gen"]
    return builder.battery_group(w["T"], w["dt"], base[None], w["bat"], retail_price=w["retail_price"][None],
                                 demand_masks=[m for _, m in w["demand"]],
                                 demand_prices=np.array([[d for d, _ in w["demand"]]]), ene_min=w["ene_min"][None],
                                 ene_max=w["ene_max"][None], **kw)


def _same(g, o):
    K = sp.csr_matrix((g.data[0], g.indices, g.indptr), shape=(g.m, g.n))
    assert K.shape == o["K"].shape and (K != o["K"]).nnz == 0
    assert np.array_equal(g.q[0], o["q"]) and np.array_equal(g.l[0], o["l"]) and np.array_equal(g.u[0], o["u"])
    assert np.allclose(g.c[0], o["c"], rtol=0, atol=1e-12) and g.c0[0] == pytest.approx(o["c0"], rel=1e-14)


def net_load(o, x, w):
    T = w["T"]
    off = o["layout"]
    net = (w["load"] - w["gen"] + w["bat"].get("hp", 0.0)) + x[off["ch"]:off["ch"] + T] - x[off["dis"]:off["dis"] + T]
    if "pv" in off:
        net = net - x[off["pv"]:off["pv"] + T]
    return net


def test_poi_limits_builder_equals_oracle_and_hold_at_the_optimum():
    """An oversized curtailable PV (12x the case's array, as a curtailable column) exports at midday; max_export = 0
    forbids it: the limit binds (cost rises: the export credit is lost), the net load stays >= 0 and below the
    import limit."""
    w = _window()
    w = dict(w, pv_curtail_max=12.0 * w["gen"], gen=np.zeros(w["T"]))
    free = window_lp.solve_highs(window_lp.build(w))
    o_free = window_lp.build(w)
    assert net_load(o_free, free["x"], w).min() < -100.0            # the free optimum exports
    poi = dict(max_import=-(w["load"].max() + 100.0), max_export=0.0)
    o = window_lp.build(dict(w, poi=poi))
    _same(_builder(w, poi=poi, pv_curtail_max=w["pv_curtail_max"][None]), o)
    h = window_lp.solve_highs(o)
    assert h["status"] == 0
    net = net_load(o, h["x"], w)
    assert net.min() >= -1e-6 and net.max() <= w["load"].max() + 100.0 + 1e-6
    assert h["obj"] > free["obj"] + 1.0
    # a loose limit leaves the optimum unchanged
    loose = window_lp.solve_highs(window_lp.build(dict(w, poi=dict(max_import=-1e6, max_export=1e6))))
    assert loose["obj"] == pytest.approx(free["obj"], rel=1e-9)


def test_poi_limits_with_curtailable_pv_carry_the_pv_column():
    w = _window()
    pvm = np.full(w["T"], 300.0)
    poi = dict(max_import=-9000.0, max_export=0.0)
    o = window_lp.build(dict(w, poi=poi, pv_curtail_max=pvm))
    _same(_builder(w, poi=poi, pv_curtail_max=pvm[None]), o)
    h = window_lp.solve_highs(o)
    assert h["status"] == 0 and net_load(o, h["x"], w).min() >= -1e-6


@pytest.mark.parametrize("curtail", [False, True])
def test_grid_charge_off_charges_from_pv_only(curtail):
    w = _window()
    T = w["T"]
    extra, bextra = {}, {}
    if curtail:
        pvm = np.full(T, 300.0)
        extra, bextra = dict(pv_curtail_max=pvm), dict(pv_curtail_max=pvm[None])
    o = window_lp.build(dict(w, grid_charge=False, **extra))
    _same(_builder(w, grid_charge=False, pv_gen=w["gen"][None], **bextra), o)
    h = window_lp.solve_highs(o)
    free = window_lp.solve_highs(window_lp.build(dict(w, **extra)))
    off = o["layout"]
    ch = h["x"][off["ch"]:off["ch"] + T]
    pv = w["gen"] + (h["x"][off["pv"]:off["pv"] + T] if curtail else 0.0)
    assert h["status"] == 0 and np.all(ch <= pv + 1e-6)
    assert h["obj"] >= free["obj"] - 1e-9 * abs(free["obj"])

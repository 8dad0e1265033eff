"""ECOS-form export (dervet_hip.export) on CVXPY-shaped golden windows (CPU; the GPU half is test_gpu_export.py).

The windows are the reference's golden Usecase 2 monthly windows (test/test_validation_report_sept1/Results/
Usecase2/{es, es+pv+dg}/step2, committed as tests/golden fixtures), written in the form CVXPY 1.0.31 hands ECOS
(tests/ecos_forms.py: bounds as one-entry G rows, zero-pinned reservation columns, the start row, shuffled
column blocks).  Checks: the presolve + band canonicalisation produce the battery-banded layout the GPU kernel
takes, the exported LP has the golden objective (HiGHS), and a solution mapped back has ECOS's sign
conventions (stationarity c + A'y + G'z = 0, z >= 0, complementary slackness, dual objective = primal),
read through a restatement of CVXPY's ECOS inversion.  Parity against a live CVXPY is unpinned (absent here).
"""
import numpy as np
import pytest
import scipy.sparse as sp

import ecos_forms
from dervet_hip import WindowResult, export
from oracle import cases, window_lp


def _golden(name):
    wins, arr, _, _ = cases.case_windows(name)
    return wins, arr


def _exported(w, seed, pins):
    olp = window_lp.build(w)
    b = w["bat"]
    data, col = ecos_forms.ecos_form(olp, w["dt"], b["rte"], b["sdr"] / 100.0, b["soc_target"] * b["E"], seed=seed,
                                     pins=pins)
    return olp, data, col, export.ecos_to_window(data)


def _highs_result(lp):
    K = sp.csr_matrix((lp.data, lp.indices, lp.indptr), shape=(lp.m, lp.n))
    h = window_lp.solve_highs(dict(K=K, q=lp.q, c=lp.c, c0=lp.c0, l=lp.l, u=lp.u, m_eq=lp.m_eq))
    assert h["status"] == 0
    return WindowResult(h["x"], h["y"], h["obj"], 0, 0, 0.0, 0.0, 0.0)


def ecos_kkt(data, sol):
    """Relative ECOS KKT errors of a solution dict: stationarity, primal feasibility, complementarity, gap."""
    A, G, b, h, c = data["A"], data["G"], data["b"], data["h"], data["c"]
    x, y, z = sol["x"], sol["y"], sol["z"]
    stat = np.linalg.norm(c + A.T @ y + G.T @ z) / (1 + np.linalg.norm(c))
    pfeas = np.sqrt(np.sum((A @ x - b) ** 2) + np.sum(np.maximum(G @ x - h, 0) ** 2)) / (
        1 + np.linalg.norm(np.concatenate([b, h])))
    pobj = c @ x + data["offset"]
    dobj = -b @ y - h @ z + data["offset"]
    return dict(stat=stat, pfeas=pfeas, zmin=z.min(initial=0.0), compl=abs(z @ (h - G @ x)) / (1 + abs(pobj)),
                gap=abs(pobj - dobj) / (1 + abs(pobj)), pobj=pobj)


@pytest.mark.parametrize("name", ["es", "es+pv+dg"])
def test_golden_windows_export_to_the_band_layout(name):
    wins, arr = _golden(name)
    for i, w in enumerate(wins):
        olp, data, col, ew = _exported(w, seed=i, pins="rows" if i % 2 == 0 else "bounds")
        lp, T = ew.lp, olp["T"]
        assert ew.banded and lp.n == 3 * T + olp["J"] and lp.m == olp["K"].shape[0] and lp.m_eq == T + 1
        # the layout the band kernel verifies: init row on ene_0, chain rows (ch_t, dis_t, ene_t, ene_t+1)
        assert list(lp.indices[lp.indptr[0]:lp.indptr[1]]) == [2 * T]
        for t in (0, T // 2, T - 2):
            assert sorted(lp.indices[lp.indptr[t + 1]:lp.indptr[t + 2]]) == [t, T + t, 2 * T + t, 2 * T + t + 1]
        assert np.all(lp.l[:2 * T] == 0.0) and np.all(np.isinf(lp.l[3 * T:]))
        r = _highs_result(lp)
        gold = float(arr["golden_objective"][i].sum())
        assert abs(r.obj - gold) <= 1e-9 * abs(gold)
        sol = ew.ecos_solution(r)
        inv = ecos_forms.invert(sol, data["offset"])
        assert inv["status"] == "optimal" and abs(inv["value"] - gold) <= 1e-9 * abs(gold)
        # the primal solution in ECOS order is the oracle's layout through `col`, and feasible
        k = ecos_kkt(data, sol)
        assert k["pfeas"] < 1e-12 and k["stat"] < 1e-12 and k["zmin"] >= 0.0 and k["compl"] < 1e-12
        assert k["gap"] < 1e-9
        assert abs(olp["c"] @ sol["x"][col] + olp["c0"] - gold) <= 1e-9 * abs(gold)


def test_dual_signs_follow_ecos():
    """Kept rows: y_ECOS = -y_E, z = y_I; one-entry rows absorb the reduced costs (the drop-in once
    passed y_E and -y_I, and pcost with the offset already in)."""
    wins, arr = _golden("es")
    olp, data, col, ew = _exported(wins[0], seed=3, pins="rows")
    r = _highs_result(ew.lp)
    sol = ew.ecos_solution(r)
    kA = ew.row_kind == export.KIND_A
    kG = ew.row_kind == export.KIND_G
    assert np.array_equal(sol["y"][ew.row_src[kA]], -r.y[kA])
    assert np.array_equal(sol["z"][ew.row_src[kG]], np.maximum(r.y[kG], 0.0))
    assert sol["info"]["pcost"] == pytest.approx(r.obj - data["offset"], rel=1e-12)
    # the same optimum as HiGHS on the untouched ECOS form (duals are not unique: compare dual objectives)
    h_obj, h_x, h_y, h_z = ecos_forms.highs_ecos(data)
    assert -data["b"] @ sol["y"] - data["h"] @ sol["z"] == pytest.approx(-data["b"] @ h_y - data["h"] @ h_z,
                                                                         rel=1e-9)
    assert ecos_forms.invert(sol, data["offset"])["value"] == pytest.approx(h_obj, rel=1e-10)


def test_status_maps_to_ecos_exit_flags():
    wins, _ = _golden("es")
    _, data, _, ew = _exported(wins[1], seed=1, pins="rows")
    r = _highs_result(ew.lp)
    expect = {0: ("optimal", True), 3: ("optimal_inaccurate", True), 1: ("infeasible", False),
              2: ("unbounded", False)}
    for st, (name, has_x) in expect.items():
        r.status = st
        inv = ecos_forms.invert(ew.ecos_solution(r), data["offset"])
        assert inv["status"] == name and (inv["x"] is not None) == has_x
    r.status = 4  # NUMERICAL -> ECOS_NUMERICS: CVXPY raises SolverError
    with pytest.raises(ecos_forms.SolverError):
        ecos_forms.invert(ew.ecos_solution(r), data["offset"])


def test_other_shapes_keep_the_generic_presolved_form():
    """A window with curtailable PV (extra columns in the DCM rows) is not the band shape: presolved generic LP,
    same optimum."""
    wins, _ = _golden("es")
    w = dict(wins[2], pv_curtail_max=np.full(wins[2]["T"], 300.0))
    olp = window_lp.build(w)
    n = olp["K"].shape[1]
    G = sp.vstack([sp.eye(n, format="csr"), -sp.eye(n, format="csr")]).tocsr()
    h = np.concatenate([olp["u"], -olp["l"]])
    keep = np.isfinite(h)
    K, q, me = olp["K"], olp["q"], olp["m_eq"]
    data = {"c": olp["c"], "offset": olp["c0"], "A": K[:me], "b": q[:me], "G": sp.vstack([G[keep], -K[me:]]),
            "h": np.concatenate([h[keep], -q[me:]]), "dims": {"l": int(keep.sum()) + K.shape[0] - me, "q": [], "e": 0}}
    ew = export.ecos_to_window(data)
    # the start row ene_0 = target fixes ene_0: one column and one row fewer
    assert not ew.banded and ew.lp.n == n - 1 and ew.lp.m == K.shape[0] - 1
    r = _highs_result(ew.lp)
    assert r.obj == pytest.approx(window_lp.solve_highs(olp)["obj"], rel=1e-9)
    k = ecos_kkt(data, ew.ecos_solution(r))
    assert k["stat"] < 1e-9 and k["zmin"] >= 0 and k["gap"] < 1e-9


def test_presolve_detects_inconsistent_rows_and_cones():
    data = {"c": np.array([1.0, 1.0]), "offset": 0.0, "A": sp.csr_matrix([[1.0, 0.0], [1.0, 0.0]]),
            "b": np.array([1.0, 2.0]), "G": sp.csr_matrix((0, 2)), "h": np.zeros(0), "dims": {"l": 0, "q": [], "e": 0}}
    with pytest.raises(export.ExportError):
        export.ecos_to_window(data)
    data = {"c": np.array([1.0]), "offset": 0.0, "A": None, "b": None, "G": sp.csr_matrix([[1.0], [-1.0], [2.0]]),
            "h": np.array([1.0, 0.0, 0.0]), "dims": {"l": 1, "q": [2], "e": 0}}
    with pytest.raises(export.ExportError):
        export.ecos_to_window(data)


# -- mixed-integer windows (binary = 1): refused by default, LP-relaxed on opt-in ----------------------------------
_MARKET_DAYS = {"es": (0, 91, 200, 364), "es+pv": (17, 180), "es+pv+dg": (45, 300)}


@pytest.mark.parametrize("name", sorted(_MARKET_DAYS))
def test_milp_market_day_is_refused_without_opt_in_and_relaxed_with_it(name):
    """Usecase 3 golden days (binary = 1, Model_Parameters_Template_DER.csv:17; goldens are the reference's MILP
    solves): the ECOS_BB form is an ExportError without ``relax``; relaxed, the exported LP's optimum equals the
    relaxed restatement's (window_lp.build(binary_relax=True), HiGHS) and is <= the golden MILP objective, and the
    solution comes back through the ECOS inversion with the relaxed objective."""
    wins, _ = cases.market_windows(name)
    for d in _MARKET_DAYS[name]:
        w = wins[d]
        data, col = ecos_forms.ecos_bb_market_form(w, seed=d)
        with pytest.raises(export.ExportError, match="mixed-integer"):
            export.ecos_to_window(data)
        ew = export.ecos_to_window(data, relax=True)
        assert ew.relaxed and ew.meta["relaxed_bool"] == 2 * w["T"] and not ew.banded
        r = _highs_result(ew.lp)
        ref = window_lp.solve_highs(window_lp.build(dict(w, binary_relax=True)))
        assert abs(r.obj - ref["obj"]) <= 1e-9 * max(1.0, abs(ref["obj"]))
        gold = float(w["golden_objective"].sum())
        assert r.obj <= gold + 1e-9 * max(1.0, abs(gold))
        sol = ew.ecos_solution(r)
        inv = ecos_forms.invert(sol, data["offset"])
        assert inv["status"] == "optimal" and inv["value"] == pytest.approx(r.obj, rel=1e-9, abs=1e-9)
        x = sol["x"]
        bools = np.asarray(data["bool_vars_idx"])
        assert x[bools].min() >= -1e-9 and x[bools].max() <= 1 + 1e-9      # the relaxation's [0, 1] box
        kkt = ecos_kkt(data, sol)
        assert kkt["pfeas"] <= 1e-8


def test_relaxed_bool_box_meets_bound_rows():
    """A boolean column that also has bound rows keeps the tighter of the row and the [0, 1] box; an integer column
    only loses integrality."""
    c = np.array([-1.0, -1.0, 1.0])
    G = sp.csr_matrix(np.array([[1.0, 0, 0], [0, 1.0, 0], [0, 0, -1.0], [1.0, 1.0, 1.0]]))
    h = np.array([0.5, 7.0, -0.25, 10.0])   # x0 <= 0.5 (tighter than 1), x1 <= 7 (looser), x2 >= 0.25
    data = {"c": c, "offset": 0.0, "A": None, "b": None, "G": G, "h": h, "dims": {"l": 4},
            "bool_vars_idx": [0, 1], "int_vars_idx": [2]}
    ew = export.ecos_to_window(data, relax=True)
    assert ew.meta["relaxed_bool"] == 2 and ew.meta["relaxed_int"] == 1
    lo = np.full(3, np.nan)
    hi = np.full(3, np.nan)
    lo[ew.col_src], hi[ew.col_src] = ew.lp.l, ew.lp.u
    assert list(lo) == [0.0, 0.0, 0.25] and list(hi) == [0.5, 1.0, np.inf]
    r = _highs_result(ew.lp)
    assert r.obj == pytest.approx(-1.5 + 0.25)
    with pytest.raises(export.ExportError):
        export.ecos_to_window(dict(data, bool_vars_idx=[5]), relax=True)

"""Post-facto reliability sweep on the GPU: the load coverage probability curve of DER-VET's Reliability value
stream (dervet/MicrogridValueStreams/Reliability.py:876-967 ``load_coverage_probability``), one outage simulated
from every start step of every case in one kernel launch (``dvh_outage_coverage``, csrc/dvh_outage.hip).

``der_mix_properties`` restates ``Reliability.get_der_mix_properties`` (:276-332) for plain DER descriptions
(storagevet's DER objects are not available here), and ``load_coverage_probability`` returns the reference's
DataFrame (index 'Outage Length (hrs)', column 'Load Coverage Probability (%)').  SOE at each outage start
follows the reference's choice (:896-905): the 'Aggregated State of Energy (kWh)' results column, the
'Aggregate Energy Min (kWh)' column for User-constraint-only runs, or soc_init x energy rating
(``init_soe=None``).  Bit-exact with the numpy reference (tests/test_gpu_outage.py); no CPU fallback.
"""
import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _lib


@dataclass
class OutageCase:
    critical_load: np.ndarray                 # [N] kW
    dt: float = 1.0                           # hours per step
    max_outage_duration: int = 24             # hours
    ess: dict = field(default_factory=dict)   # E (kWh), P_ch, P_dis (kW), rte (fraction), llsoc, ulsoc (fractions)
    init_soe: np.ndarray = None               # [N] energy at each outage start; None: soc_init x E
    soc_init: float = 1.0                     # post_facto_initial_soc (fraction)
    pv_max: list = field(default_factory=list)   # [N] arrays, one per PV (maximum generation)
    pv_nu: list = field(default_factory=list)    # nu (fraction) per PV
    pv_gamma: list = field(default_factory=list)  # gamma (fraction) per PV
    dg_power: list = field(default_factory=list)  # max power out (kW) per generator
    n_2: bool = False                         # N-2: drop the largest generator (dg_rating)
    dg_rating: float = 0.0
    load_shed_pct: np.ndarray = None          # [max_outage_duration] % of critical load kept per outage hour


def der_mix_properties(case):
    """(dg_gen, pv_max, props, pv_vari, largest_gamma) as Reliability.get_der_mix_properties (:276-332)."""
    N = len(case.critical_load)
    pv_max = np.zeros(N)
    pv_vari = np.zeros(N)
    gamma = 0.0
    for g, nu, ga in zip(case.pv_max, case.pv_nu, case.pv_gamma):
        g = np.asarray(g, np.float64)
        pv_max += g
        pv_vari += g * nu
        gamma = max(gamma, ga)
    dg = float(sum(case.dg_power))
    if case.n_2:
        dg -= case.dg_rating
    e = case.ess
    props = {"charge max": float(e.get("P_ch", 0.0)), "discharge max": float(e.get("P_dis", 0.0)),
             "operation SOE min": e.get("llsoc", 0.0) * float(e.get("E", 0.0)),
             "operation SOE max": e.get("ulsoc", 1.0) * float(e.get("E", 0.0)),
             "rte": float(e.get("rte", 1.0)), "energy rating": float(e.get("E", 0.0)),
             "pv present": bool(case.pv_max)}
    return dg, pv_max, props, pv_vari, gamma


def _cases_struct(cases):
    arr = (_lib.OutageCase * len(cases))()
    keep, sizes = [], []

    def ptr(a):
        if a is None:
            return None
        a = np.ascontiguousarray(a, np.float64)
        keep.append(a)
        return a.ctypes.data_as(_lib.c_double_p)

    for k, c in enumerate(cases):
        dg, pv_max, props, pv_vari, gamma = der_mix_properties(c)
        N = len(c.critical_load)
        o = arr[k]
        o.n_steps, o.max_outage, o.dt = N, int(c.max_outage_duration), float(c.dt)
        o.critical_load = ptr(c.critical_load)
        o.pv_max = ptr(pv_max) if c.pv_max else None
        o.pv_vari = ptr(pv_vari) if c.pv_max else None
        o.init_soe = ptr(c.init_soe)
        o.load_shed_pct = ptr(c.load_shed_pct)
        o.soe0 = c.soc_init * props["energy rating"]
        o.dg_gen, o.gamma = dg, gamma
        o.soe_min, o.soe_max = props["operation SOE min"], props["operation SOE max"]
        o.charge_max, o.discharge_max, o.rte = props["charge max"], props["discharge max"], props["rte"]
        sizes.append((N, int(c.max_outage_duration / c.dt)))
    return arr, keep, sizes


def outage_coverage(cases, solver):
    """Covered length per start (list of int32 arrays) and the LCP curve per case (list of float arrays)."""
    lib = solver._lib
    arr, keep, sizes = _cases_struct(cases)
    lengths = np.zeros(sum(n for n, _ in sizes), np.int32)
    lcp = np.zeros(sum(L for _, L in sizes), np.float64)
    solver._check(lib.dvh_outage_coverage(solver._h, arr, len(cases), lengths.ctypes.data_as(_lib.c_int32_p),
                                          lcp.ctypes.data_as(_lib.c_double_p)), "dvh_outage_coverage")
    out_l, out_c, a, b = [], [], 0, 0
    for N, L in sizes:
        out_l.append(lengths[a:a + N])
        out_c.append(lcp[b:b + L])
        a += N
        b += L
    return out_l, out_c


def min_soe(cases, target_hours, solver):
    """Reliability.min_soe_iterative (:685-756) per case: [N] minimum SOE (kWh) the ESS must hold at each step
    to ride through a target_hours outage from soc_init x energy rating (the 'Reliability Min State of Energy
    (kWh)' requirement applied to every window as an ene lower bound, :334-354)."""
    lib = solver._lib
    arr, keep, sizes = _cases_struct(cases)
    tgt = np.ascontiguousarray(np.broadcast_to(np.asarray(target_hours, np.int32), (len(cases),)))
    out = np.zeros(sum(n for n, _ in sizes), np.float64)
    solver._check(lib.dvh_outage_min_soe(solver._h, arr, len(cases), tgt.ctypes.data_as(_lib.c_int32_p),
                                         out.ctypes.data_as(_lib.c_double_p)), "dvh_outage_min_soe")
    res, a = [], 0
    for N, _ in sizes:
        res.append(out[a:a + N])
        a += N
    return res


def load_coverage_probability(cases, solver):
    """The reference's DataFrames (Reliability.py:959-967), one per case."""
    import pandas as pd
    _, curves = outage_coverage(cases, solver)
    out = []
    for c, v in zip(cases, curves):
        length = np.arange(c.dt, c.max_outage_duration + c.dt, c.dt)[:len(v)]
        df = pd.DataFrame({"Outage Length (hrs)": length, "Load Coverage Probability (%)": v})
        out.append(df.set_index("Outage Length (hrs)"))
    return out


def last_kernel_ms(solver):
    ms = ctypes.c_double()
    solver._check(solver._lib.dvh_last_outage_ms(solver._h, ctypes.byref(ms)), "dvh_last_outage_ms")
    return ms.value

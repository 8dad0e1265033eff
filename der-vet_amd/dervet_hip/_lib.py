"""ctypes binding of libdervet_hip (include/dervet_hip.h).

The library is the product path: there is no CPU fallback.  Loading fails loudly when the shared object
is missing, and every solve fails loudly when no GPU is present.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# DVH_LIB: an alternative build of the same library (kernel A/B helpers under scripts/)
LIB_PATH = os.environ.get("DVH_LIB") or os.path.join(HERE, "libdervet_hip.so")

DVH_OK, DVH_ERR_ARG, DVH_ERR_HIP, DVH_ERR_UNSUPPORTED = 0, -1, -2, -3
OPTIMAL, PRIMAL_INFEASIBLE, DUAL_INFEASIBLE, ITER_LIMIT, NUMERICAL = 0, 1, 2, 3, 4
STATUS_NAMES = {OPTIMAL: "optimal", PRIMAL_INFEASIBLE: "infeasible", DUAL_INFEASIBLE: "unbounded",
                ITER_LIMIT: "optimal_inaccurate", NUMERICAL: "solver_error"}

c_int32_p = ctypes.POINTER(ctypes.c_int32)
c_double_p = ctypes.POINTER(ctypes.c_double)
c_int64_p = ctypes.POINTER(ctypes.c_int64)


class Options(ctypes.Structure):
    _fields_ = [("eps", ctypes.c_double), ("max_iters", ctypes.c_int32), ("check_every", ctypes.c_int32),
                ("ruiz_iters", ctypes.c_int32), ("power_iters", ctypes.c_int32), ("step_safety", ctypes.c_double),
                ("reflection", ctypes.c_double), ("restart_sufficient", ctypes.c_double),
                ("restart_necessary", ctypes.c_double), ("restart_artificial", ctypes.c_double),
                ("primal_weight_theta", ctypes.c_double), ("verbose", ctypes.c_int32),
                ("kkt_every", ctypes.c_int32), ("warm_start", ctypes.c_int32), ("pad0", ctypes.c_int32),
                ("eps_obj", ctypes.c_double), ("kkt_predict", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


class LP(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("m_eq", ctypes.c_int32), ("m_ineq", ctypes.c_int32), ("nnz", ctypes.c_int32),
                ("indptr", c_int32_p), ("indices", c_int32_p), ("data", c_double_p), ("c", c_double_p),
                ("c0", ctypes.c_double), ("q", c_double_p), ("l", c_double_p), ("u", c_double_p),
                ("structure", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class Result(ctypes.Structure):
    _fields_ = [("x", c_double_p), ("y", c_double_p), ("obj", ctypes.c_double), ("primal_res_rel", ctypes.c_double),
                ("dual_res_rel", ctypes.c_double), ("gap_rel", ctypes.c_double), ("status", ctypes.c_int32),
                ("iters", ctypes.c_int32)]


class Packed(ctypes.Structure):
    _fields_ = [("count", ctypes.c_int32), ("reserved", ctypes.c_int32), ("total_n", ctypes.c_int64),
                ("total_m", ctypes.c_int64), ("total_nnz", ctypes.c_int64), ("total_rows", ctypes.c_int64),
                ("desc", ctypes.c_void_p), ("indptr", ctypes.c_void_p), ("indices", ctypes.c_void_p),
                ("data", ctypes.c_void_p), ("c", ctypes.c_void_p), ("c0", ctypes.c_void_p), ("q", ctypes.c_void_p),
                ("l", ctypes.c_void_p), ("u", ctypes.c_void_p), ("x", ctypes.c_void_p), ("y", ctypes.c_void_p),
                ("stats", ctypes.c_void_p), ("istats", ctypes.c_void_p)]


class OutageCase(ctypes.Structure):
    _fields_ = [("n_steps", ctypes.c_int32), ("max_outage", ctypes.c_int32), ("dt", ctypes.c_double),
                ("critical_load", c_double_p), ("pv_max", c_double_p), ("pv_vari", c_double_p),
                ("init_soe", c_double_p), ("load_shed_pct", c_double_p), ("soe0", ctypes.c_double),
                ("dg_gen", ctypes.c_double), ("gamma", ctypes.c_double), ("soe_min", ctypes.c_double),
                ("soe_max", ctypes.c_double), ("charge_max", ctypes.c_double), ("discharge_max", ctypes.c_double),
                ("rte", ctypes.c_double)]


# symbol -> (restype, argtypes); every symbol declared in include/dervet_hip.h
class BatteryGroup(ctypes.Structure):
    """dvh_battery_group (device-side window builder inputs; pointers are device addresses)."""
    _fields_ = [("T", ctypes.c_int32), ("J", ctypes.c_int32), ("G", ctypes.c_int32), ("mI", ctypes.c_int32),
                ("dt", ctypes.c_double), ("has_retail", ctypes.c_int32), ("has_da", ctypes.c_int32),
                ("has_emin", ctypes.c_int32), ("has_emax", ctypes.c_int32)] + \
               [(f, ctypes.c_void_p) for f in ("dcm_t", "dcm_j", "base", "retail", "da", "demand", "emin", "emax", "E",
                                               "pch", "pdis", "rte", "sdr", "soc_target", "ulsoc", "llsoc", "om",
                                               "c0")] + \
               [("has_ice", ctypes.c_int32), ("pad_ice", ctypes.c_int32)] + \
               [(f, ctypes.c_void_p) for f in ("ice_cap", "ice_pmin", "ice_cost")]



class SweepDraws(ctypes.Structure):
    """dvh_sweep_draws (scenario series generator; seeds host, outputs device)."""
    _fields_ = [("count", ctypes.c_int32), ("steps", ctypes.c_int32), ("n_uniform", ctypes.c_int32),
                ("seeds", ctypes.c_void_p), ("a1", ctypes.c_double), ("innov", ctypes.c_double),
                ("z0", ctypes.c_void_p), ("ar", ctypes.c_void_p), ("uniform", ctypes.c_void_p),
                ("ambiguous", ctypes.c_void_p)]


class WindowSeries(ctypes.Structure):
    """dvh_window_series (the device builder's inputs cut from the scenarios' series; device pointers)."""
    _fields_ = [(f, ctypes.c_int32) for f in ("G", "T", "t0", "rep", "J", "count", "hours")] + \
               [("dt", ctypes.c_double)] + \
               [(f, ctypes.c_void_p) for f in ("rows", "ar", "site_load", "pv_profile", "price", "load_scale",
                                               "price_scale", "pv_rated", "hp", "c0_add", "base", "retail", "c0")]

SYMBOLS = {
    "dvh_version": (ctypes.c_char_p, []),
    "dvh_default_options": (None, [ctypes.POINTER(Options)]),
    "dvh_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(Options), ctypes.POINTER(ctypes.c_void_p)]),
    "dvh_create_devices": (ctypes.c_int, [c_int32_p, ctypes.c_int32, ctypes.POINTER(Options),
                                          ctypes.POINTER(ctypes.c_void_p)]),
    "dvh_device_count": (ctypes.c_int, [ctypes.c_void_p]),
    "dvh_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "dvh_last_error": (ctypes.c_char_p, [ctypes.c_void_p]),
    "dvh_set_options": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Options)]),
    "dvh_solve_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(LP), ctypes.c_int32, ctypes.POINTER(Result)]),
    "dvh_solve_packed_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Packed), ctypes.c_void_p]),
    "dvh_warm_transfer": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Packed), ctypes.c_void_p, ctypes.c_int32]),
    "dvh_warm_transfer_blend": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Packed), ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]),
    "dvh_build_battery_group": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(BatteryGroup), ctypes.POINTER(Packed),
                                               ctypes.c_int32]),
    "dvh_synchronize": (ctypes.c_int, [ctypes.c_void_p]),
    "dvh_series_draws": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(SweepDraws)]),
    "dvh_series_windows": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(WindowSeries)]),
    "dvh_last_timing": (ctypes.c_int, [ctypes.c_void_p, c_double_p]),
    "dvh_last_stats": (ctypes.c_int, [ctypes.c_void_p, c_int32_p]),
    "dvh_last_host_syncs": (ctypes.c_int, [ctypes.c_void_p, c_int32_p]),
    "dvh_last_path_counts": (ctypes.c_int, [ctypes.c_void_p, c_int32_p]),
    "dvh_last_path_counts4": (ctypes.c_int, [ctypes.c_void_p, c_int32_p]),
    "dvh_last_path_counts5": (ctypes.c_int, [ctypes.c_void_p, c_int32_p]),
    "dvh_last_chain_aborts": (ctypes.c_int, [ctypes.c_void_p, c_int32_p]),
    "dvh_last_warning": (ctypes.c_char_p, [ctypes.c_void_p]),
    "dvh_set_kernel_path": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "dvh_set_launch_order": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32]),
    "dvh_outage_coverage": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(OutageCase), ctypes.c_int32, c_int32_p,
                                           c_double_p]),
    "dvh_outage_min_soe": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(OutageCase), ctypes.c_int32, c_int32_p,
                                          c_double_p]),
    "dvh_last_outage_ms": (ctypes.c_int, [ctypes.c_void_p, c_double_p]),
    "dvh_comm_unique_id": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p]),
    "dvh_comm_init": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_char_p]),
    "dvh_comm_info": (ctypes.c_int, [ctypes.c_void_p, c_int32_p]),
    "dvh_gather_results": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                          ctypes.c_void_p]),
}
COMM_ID_BYTES = 128  # DVH_COMM_ID_BYTES

_lib = None


def load(path=None):
    """Load libdervet_hip.so (raises if it was not built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(f"libdervet_hip.so not found at {p}: build it with `python -m dervet_hip.build` "
                           "(there is no CPU fallback)")
    lib = ctypes.CDLL(p)
    for name, (res, args) in SYMBOLS.items():
        if os.environ.get("DVH_LIB") and not hasattr(lib, name):
            continue  # an A/B build of an earlier library (scripts/): the entry points it has
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if path is None:
        _lib = lib
    return lib


def default_options(**kw):
    o = Options()
    load().dvh_default_options(ctypes.byref(o))
    for k, v in kw.items():
        if not hasattr(o, k):
            raise KeyError(f"unknown option {k}")
        setattr(o, k, v)
    return o

"""Scenario / window assembly for the BASELINE.json configurations.

``windows_by_period`` plays the role of storagevet ``Scenario.optimization_levels`` + the per-window
``set_up_optimization`` of dervet/MicrogridScenario.py:322-346 for many scenarios at once: it splits each
scenario's time series into optimization windows (n = 'month' | 'year') and builds one WindowGroup per
window position (all scenarios together, one CSR pattern).

Config 4 (the bench workload): 10,000 perturbations of the config-2 scenario x 12 monthly windows.
Generator (numpy PCG64), per scenario s with seed 20250217 + s, draws in this order:
  load scale ~ LogNormal(0, 0.15); AR(1) innovations e_t ~ N(0,1), t < 8760; price scale ~ U[0.7, 1.3];
  demand charge ~ U[5, 25] $/kW; PV rated ~ U[0, 2000] kW; E ~ U[500, 10000] kWh; duration ~ U[2, 6] h
  (P = E / duration); rte ~ U[0.80, 0.95].
  load_t = base_t * scale * (1 + 0.05 a_t),  a_t = 0.9 a_{t-1} + sqrt(1 - 0.81) e_t,  a_0 = e_0.
"""
import functools
import os

import numpy as np

from . import tariff as _tariff
from .builder import battery_group

DATA = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data")
SEED0 = 20250217


@functools.lru_cache(maxsize=1)
def _reference_arrays():
    with np.load(os.path.join(DATA, "reference_inputs.npz")) as z:
        out = {k: z[k] for k in z.files}
    for v in out.values():
        v.setflags(write=False)  # shared by every caller: read-only
    return out


def reference_inputs():
    """The reference's input series (data/reference_inputs.npz), loaded once per process (read-only arrays)."""
    return dict(_reference_arrays())


def tariff(name="data_tariff"):
    return _tariff.load_tariff_json(os.path.join(DATA, f"tariff_{name}.json"))


def windows_by_period(year, dt, load, gen, bat, tariff_def=None, da_price=None, n="month", ene_min=None,
                      ene_max=None, demand_price_override=None, price_scale=None, tags_prefix=None,
                      pv_curtail_max=None, ice=None, poi=None, grid_charge=True, only=None, spec=False):
    """Split S scenarios' series [S, Tall] into windows; returns a list of WindowGroup (one per window id).

    demand_price_override [S] replaces every demand charge's $/kW (sweep); price_scale [S] scales energy prices.
    poi / grid_charge: POI interconnection limits and PV grid_charge (builder.battery_group; parity unpinned).
    only: window ids to build (None: all), e.g. one window position of a degradation-coupled sweep.
    spec: return the device builder's inputs (gpu_builder.BatteryGroupSpec) instead of host-built groups.
    """
    load = np.atleast_2d(np.asarray(load, np.float64))
    S, Tall = load.shape
    gen = np.zeros_like(load) if gen is None else np.broadcast_to(np.asarray(gen, np.float64), load.shape)
    month, he, wd, yr = _tariff.calendar(year, Tall, dt)
    price = None
    d_ids, d_vals, d_masks = np.zeros(0), np.zeros(0), np.zeros((0, Tall), bool)
    if tariff_def is not None:
        price = np.broadcast_to(_tariff.energy_price(tariff_def, month, he, wd), (S, Tall))
        if price_scale is not None:
            price = price * np.asarray(price_scale, np.float64)[:, None]
        d_ids, d_vals, d_masks = _tariff.demand_charges(tariff_def, month, he, wd)
    if n == "month":
        wid = (yr - yr[0]) * 12 + month - 1
    elif n == "year":
        wid = yr - yr[0]
    else:
        wid = np.arange(Tall) // int(n)
    groups = []
    for w in np.unique(wid):
        if only is not None and int(w) not in only:
            continue
        sel = np.nonzero(wid == w)[0]
        T = len(sel)
        masks, prices = [], []
        for p in range(len(d_vals)):
            for mo in np.unique(month[sel]):
                mk = d_masks[p, sel] & (month[sel] == mo)
                if mk.any():
                    masks.append(mk)
                    dp = np.full(S, d_vals[p]) if demand_price_override is None else np.asarray(demand_price_override)
                    prices.append(dp)
        masks = np.array(masks, bool).reshape(-1, T)
        prices = np.stack(prices, axis=1) if prices else np.zeros((S, 0))
        make = battery_group
        if spec:
            from .gpu_builder import battery_group_spec as make
        g = make(
            T, dt, load[:, sel] - gen[:, sel], bat,
            retail_price=None if price is None else price[:, sel],
            da_price=None if da_price is None else np.broadcast_to(np.asarray(da_price, np.float64), (S, Tall))[:, sel],
            demand_masks=masks, demand_prices=prices,
            ene_min=None if ene_min is None else np.broadcast_to(ene_min, (S, Tall))[:, sel],
            ene_max=None if ene_max is None else np.broadcast_to(ene_max, (S, Tall))[:, sel],
            tags=[(s if tags_prefix is None else tags_prefix[s], int(w)) for s in range(S)],
            pv_curtail_max=None if pv_curtail_max is None else np.broadcast_to(pv_curtail_max, (S, Tall))[:, sel],
            ice=ice, poi=poi, grid_charge=grid_charge, pv_gen=None if grid_charge else gen[:, sel])
        g.index = sel
        groups.append(g)
    return groups


def template_battery():
    """Model_Parameters_Template_DER.csv battery (:50-70): 1000 kWh, 250 kW, rte 85 %, hp 100 kW."""
    return dict(E=1000.0, Pch=250.0, Pdis=250.0, rte=0.85, sdr=0.0, soc_target=1.0, ulsoc=1.0, llsoc=0.0,
                fixedOM=10.0, OMexpenses=0.0, hp=100.0)


def config1(with_retail=False):
    """Template battery, DA energy time shift on data/hourly_timeseries.csv (incl_site_load = 0), monthly."""
    ri = reference_inputs()
    T = len(ri["hourly_da_price"])
    load = np.zeros((1, T))
    if with_retail:
        load = ri["hourly_site_load"][None, :]
    return windows_by_period(2017, 1.0, load, None, template_battery(),
                             tariff_def=tariff("data_tariff") if with_retail else None,
                             da_price=ri["hourly_da_price"][None, :])


def config3(variant="da", n="year"):
    """BASELINE config 3: the 5-minute (dt = 1/12 h, Model_Parameters_Template_DER.csv:4) year of
    test/datasets/000-004-timeseries_5min_negprices.csv (2019, 105,120 steps, 2,375 negative DA prices) with the
    template battery.  variant "da": DA time shift alone, no site load (n = 315,360); "dcm": DA + retailETS + the 12
    monthly demand charges of data/tariff.csv on the file's site load, less the template's fixed PV (100 kW,
    curtail 0, grid_charge 0: Model_Parameters_Template_DER.csv PV rows) with data/multi_der_hourly_timeseries.csv's
    2017 "PV Gen (kW/rated kW)/1" profile held over each hour (n = 315,372, m = 210,241).  n: the window ("year": one
    annual window; an int: sub-windows of that many steps, e.g. 288 = daily, for the stitched start)."""
    ri = reference_inputs()
    T = len(ri["fivemin_da_price"])
    da = ri["fivemin_da_price"][None, :]
    if variant == "da":
        return windows_by_period(2019, 1.0 / 12, np.zeros((1, T)), None, template_battery(), da_price=da, n=n)
    if variant != "dcm":
        raise ValueError(f"config3 variant {variant!r}")
    pv = 100.0 * np.repeat(np.nan_to_num(ri["multi_der_pv_profile"]), 12)[:T]
    return windows_by_period(2019, 1.0 / 12, ri["fivemin_site_load"][None, :], pv[None, :], template_battery(),
                             da_price=da, tariff_def=tariff(), n=n, grid_charge=False)


def config2_battery():
    return dict(E=4000.0, Pch=1000.0, Pdis=1000.0, rte=0.91, sdr=0.0, soc_target=1.0, ulsoc=1.0, llsoc=0.0,
                fixedOM=10.0, OMexpenses=0.0, hp=0.0)


def config2(years=(2017, 2018, 2019), pv_rated=1000.0):
    """Battery + fixed PV + DCM + retailETS on data/multi_der_hourly_timeseries.csv, data/tariff.csv,
    monthly windows over 3 opt years (the same 2017 profile re-used for 2018-19: growth 0)."""
    ri = reference_inputs()
    load = ri["multi_der_site_load"]
    gen = pv_rated * np.nan_to_num(ri["multi_der_pv_profile"])
    groups = []
    for y in years:
        groups += windows_by_period(y, 1.0, load[None, :], gen[None, :], config2_battery(), tariff_def=tariff())
    return groups


def sweep_parameters(scenarios):
    """Per-scenario draws of the config-4 generator (module docstring)."""
    scen = np.asarray(list(scenarios), np.int64)
    S = len(scen)
    out = dict(load_scale=np.empty(S), eps=np.empty((S, 8760)), price_scale=np.empty(S), demand=np.empty(S),
               pv_rated=np.empty(S), E=np.empty(S), duration=np.empty(S), rte=np.empty(S))
    for i, s in enumerate(scen):
        rng = np.random.Generator(np.random.PCG64(SEED0 + int(s)))
        out["load_scale"][i] = rng.lognormal(0.0, 0.15)
        out["eps"][i] = rng.standard_normal(8760)
        out["price_scale"][i] = rng.uniform(0.7, 1.3)
        out["demand"][i] = rng.uniform(5.0, 25.0)
        out["pv_rated"][i] = rng.uniform(0.0, 2000.0)
        out["E"][i] = rng.uniform(500.0, 10000.0)
        out["duration"][i] = rng.uniform(2.0, 6.0)
        out["rte"][i] = rng.uniform(0.80, 0.95)
    return out


def sweep_features(P):
    """Similarity features of sweep scenarios (for dervet_hip.sweep's nearest-seed choice): battery energy
    relative to load (log), battery duration, PV rating relative to load.  GPU study on 48,000 config-4 windows
    (profiles/r01i_seeded_features*.log): warm windows 2,152 -> 2,023 iterations vs battery energy alone."""
    return np.stack([np.log(P["E"] / P["load_scale"]), P["duration"], P["pv_rated"] / P["load_scale"]], axis=1)


@functools.lru_cache(maxsize=1)
def _config4_series(scenarios):
    """The scenarios' draws and hourly load / PV series (kept for the next call: a degradation-coupled sweep builds
    one window position per call from the same series; read-only)."""
    from scipy.signal import lfilter
    ri = reference_inputs()
    P = sweep_parameters(scenarios)
    phi = 0.9
    e = P.pop("eps")
    e[:, 1:] *= np.sqrt(1.0 - phi * phi)
    a = lfilter([1.0], [1.0, -phi], e, axis=1)
    del e
    load = ri["multi_der_site_load"][None, :] * P["load_scale"][:, None] * (1.0 + 0.05 * a)
    gen = P["pv_rated"][:, None] * np.nan_to_num(ri["multi_der_pv_profile"])[None, :]
    for v in list(P.values()) + [load, gen]:
        v.flags.writeable = False
    return P, load, gen


def config4(scenarios, n="month", dt=1.0, E=None, only=None, spec=False):
    """Synthetic sweep windows for the given scenario ids (12 monthly windows each).  n: the optimisation window
    (Model_Parameters_Template_DER.csv:8 `n`: "month", "year" or a step count); dt < 1: sub-hourly steps, the hourly
    series held constant within each hour (Model_Parameters_Template_DER.csv:4 `dt`).  E [S]: the batteries'
    current energy capacity (a degraded battery, dervet_hip.degradation; power ratings stay at the rated E /
    duration); only: window ids to build; spec: the device builder's inputs instead of host-built groups."""
    P, load, gen = _config4_series(tuple(int(s) for s in scenarios))
    Eb = P["E"] if E is None else np.asarray(E, np.float64)
    bat = dict(E=Eb, Pch=P["E"] / P["duration"], Pdis=P["E"] / P["duration"], rte=P["rte"], sdr=0.0,
               soc_target=1.0, ulsoc=1.0, llsoc=0.0, fixedOM=10.0, OMexpenses=0.0, hp=0.0)
    rep = int(round(1.0 / dt))
    if rep > 1:
        load, gen = np.repeat(load, rep, axis=1), np.repeat(gen, rep, axis=1)
    return windows_by_period(2017, dt, load, gen, bat, tariff_def=tariff(), n=n, demand_price_override=P["demand"],
                             price_scale=P["price_scale"], tags_prefix=list(scenarios), only=only, spec=spec)


def reliability_min_soe(critical_load, hours=4.0, dt=1.0, cap=None):
    """Synthetic reliability requirement (BASELINE config 5): energy to carry the critical load for the next
    `hours` hours from every step, min_soe_t = sum_{k=t}^{t+h-1} critical_k dt (the shape of
    Reliability.min_soe_iterative, Reliability.py:685-733, without the outage simulation; UNPINNED)."""
    c = np.atleast_2d(np.asarray(critical_load, np.float64))
    h = int(round(hours / dt))
    cs = np.concatenate([np.zeros((c.shape[0], 1)), np.cumsum(c, axis=1)], axis=1)
    T = c.shape[1]
    idx = np.minimum(np.arange(T) + h, T)
    out = (cs[:, idx] - cs[:, :T]) * dt
    if cap is not None:
        out = np.minimum(out, np.asarray(cap, np.float64).reshape(-1, 1))
    return out


def config5_outage_cases(scenarios, count_ice=False):
    """Per scenario, the DER mix the Reliability value stream simulates outages with (Reliability.min_soe_iterative,
    dervet/MicrogridValueStreams/Reliability.py:685-733, via get_der_mix_properties :276-332): the scenario's
    critical load (data/multi_der_hourly_timeseries.csv "Critical Load (kW)" x its load scale), its battery
    (E, P, rte; soc_init 100 %, template "post_facto_initial_soc"), its PV (rated x profile, template nu 20 % /
    gamma 43 %, Model_Parameters_Template_DER.csv:118-119) and, with count_ice, the ICE units (7 x 750 kW; they
    alone carry the critical load, which makes the requirement zero -- the bench's config 5 leaves them out of the
    outage mix so the 4-h requirement binds)."""
    from ..reliability import OutageCase
    ri = reference_inputs()
    scen = list(scenarios)
    P = sweep_parameters(scen)
    pv = np.nan_to_num(ri["multi_der_pv_profile"])
    cases = []
    for i in range(len(scen)):
        E = float(P["E"][i])
        Pw = E / float(P["duration"][i])
        cases.append(OutageCase(critical_load=ri["multi_der_critical_load"] * float(P["load_scale"][i]), dt=1.0,
                                max_outage_duration=80,
                                ess=dict(E=E, P_ch=Pw, P_dis=Pw, rte=float(P["rte"][i]), llsoc=0.0, ulsoc=1.0),
                                soc_init=1.0, pv_max=[float(P["pv_rated"][i]) * pv], pv_nu=[0.20], pv_gamma=[0.43],
                                dg_power=[750.0] * 7 if count_ice else []))
    return cases


def config5_min_soe(scenarios, solver, target_hours=4, count_ice=False):
    """[S, 8760] 'Reliability Min State of Energy' per scenario, computed on the GPU (dvh_outage_min_soe, the
    Reliability.min_soe_iterative restatement) -- the ene lower bound every config-5 window applies (row a10)."""
    from ..reliability import min_soe
    return np.stack(min_soe(config5_outage_cases(scenarios, count_ice), target_hours, solver))


def config5(scenarios, years=20, start_year=2017, min_soe=None, cap_min_soe=False, spec=False):
    """Battery + fixed PV + LP-relaxed ICE + 4-h reliability min-SOE, retail + DCM, monthly windows over
    `years` opt years (the 2017 profile re-used each year).  Perturbations as config 4 (same seeds) plus
    ICE fuel cost; ICE parameters from the Usecase3 ES+PV+DG model parameters (750 kW x 7 units,
    0.0866 gal/kWh) with a 250 kW minimum stable output per unit so the relaxation binds.
    min_soe [S, 8760]: the reliability requirement (``config5_min_soe``, computed on the GPU); None: the synthetic
    4-h critical-load coverage vector ``reliability_min_soe`` (CPU tests).  Hours whose requirement exceeds the
    battery's energy rating (the restated simulate_outage lets SOE climb past E while it "discharges" a negative
    net load, Reliability.py:543-556) give crossed ene bounds: those windows are infeasible as the reference
    states them and the solver reports PRIMAL_INFEASIBLE without iterating; cap_min_soe=True clips the requirement
    at ulsoc * E instead (the bench's timed horizon, which reports how many windows the clip touched).
    spec: the device builder's inputs (gpu_builder.BatteryGroupSpec, ICE included) instead of host-built groups."""
    from scipy.signal import lfilter
    ri = reference_inputs()
    scen = list(scenarios)
    P = sweep_parameters(scen)
    e = P["eps"].copy()
    e[:, 1:] *= np.sqrt(1.0 - 0.81)
    a = lfilter([1.0], [1.0, -0.9], e, axis=1)
    load = ri["multi_der_site_load"][None, :] * P["load_scale"][:, None] * (1.0 + 0.05 * a)
    gen = P["pv_rated"][:, None] * np.nan_to_num(ri["multi_der_pv_profile"])[None, :]
    E = P["E"]
    bat = dict(E=E, Pch=E / P["duration"], Pdis=E / P["duration"], rte=P["rte"], sdr=0.0, soc_target=1.0,
               ulsoc=1.0, llsoc=0.0, fixedOM=10.0, OMexpenses=0.0, hp=0.0)
    fuel = 2.5 + P["price_scale"]  # U[3.2, 3.8] $/gal, deterministic from the same draws
    ice = dict(rated_power=750.0, n=7.0, min_power=250.0, efficiency=0.086618705, fuel_cost=fuel,
               variable_om_cost=0.0)
    if min_soe is None:
        crit = ri["multi_der_critical_load"][None, :] * P["load_scale"][:, None]
        emin = reliability_min_soe(crit, 4.0, 1.0, cap=E)
    else:
        emin = np.asarray(min_soe, np.float64).reshape(len(scen), -1)
        if cap_min_soe:
            emin = np.minimum(emin, (bat["ulsoc"] * E)[:, None])
    groups = []
    for y in range(years):
        gy = windows_by_period(start_year + y, 1.0, load, gen, bat, tariff_def=tariff(),
                               demand_price_override=P["demand"], price_scale=P["price_scale"],
                               ene_min=emin, ice=ice, tags_prefix=scen, spec=spec)
        if y > 0:  # window ids unique over the horizon (12 y + month): several opt years can share one sweep batch
            for g in gy:
                g.tags = [(t[0], 12 * y + t[1]) for t in g.tags]
        groups += gy
    return groups


# dvh_options for market-service day windows (Usecase 3 style): primal-weight smoothing theta = 0.5 (PDLP's omega
# <- exp(theta log(dy/dx) + (1 - theta) log(omega)) at restarts).  On the 1,095 golden days (algorithm lab, host cores)
# the slowest day takes 5,504 iterations instead of 7,424 and the mean 1,589 instead of 1,799, objectives within 3e-7
# of the theta = 1 solve; a batch of days is latency-bound on its slowest window, so the wall time follows the max.
# Not the library default: on the battery / DCM windows of config 4 theta = 0.5 costs 18 % cold and 6 % warm
# iterations, and config 3's DCM + PV window takes 1.85x as many.
MARKET_OPTIONS = {"primal_weight_theta": 0.5}


def market_days(signals, params, relax=True, days=None, name="es", reserves=None, lf=None):
    """Daily DA + frequency-regulation windows (Usecase 3 style) as one
    market_group.  signals: dict of [N] arrays da_price, regu_price, regd_price, fr_price, agg_emin, agg_emax,
    pv_gen (fixed PV, curtail = 0), regu_max/min, regd_max/min; params: model parameters (Tag -> Key -> value
    strings, as the reference's model-parameter CSV).  Windows are consecutive blocks of n steps
    (``optimization_levels`` for an integer n); ``relax`` applies the opt-in LP relaxation to binary = 1.
    reserves (optional, parity unpinned): upward reserve services as builder.market_group takes them, with
    full-length [N] price / max / min series (template columns "SR Price ($/kW)", "SR Max (kW)", ...).
    lf (optional, parity unpinned): load following as builder.market_group takes it, with full-length [N] series
    (eou / eod may be scalars; combined a bool)."""
    from .builder import market_group
    sc, b, fr = params["Scenario"], params["Battery"], params["FR"]
    n, dt = int(sc["n"]), float(sc["dt"])
    flag = lambda v: str(v).strip() not in ("0", "0.0", "", "no")
    N = len(signals["da_price"]) // n * n
    sel = np.arange(N).reshape(-1, n)
    if days is not None:
        sel = sel[np.asarray(days)]
    blk = lambda k: np.asarray(signals[k], np.float64)[sel]
    bat = dict(E=float(b["ene_max_rated"]), Pch=float(b["ch_max_rated"]), Pdis=float(b["dis_max_rated"]),
               rte=float(b["rte"]) / 100.0, sdr=float(b["sdr"]), soc_target=float(b["soc_target"]) / 100.0,
               ulsoc=float(b["ulsoc"]) / 100.0, llsoc=float(b["llsoc"]) / 100.0, fixedOM=float(b["fixedOM"]),
               OMexpenses=float(b["OMexpenses"]))
    frd = dict(eou=float(fr["eou"]), eod=float(fr["eod"]), regu_price=blk("regu_price"),
               regd_price=blk("regd_price"), fr_price=blk("fr_price"), combined=flag(fr.get("CombinedMarket", 0)))
    if flag(fr.get("u_ts_constraints", 0)):
        frd["regu_max"], frd["regu_min"] = blk("regu_max"), blk("regu_min")
    if flag(fr.get("d_ts_constraints", 0)):
        frd["regd_max"], frd["regd_min"] = blk("regd_max"), blk("regd_min")
    base = -blk("pv_gen") if "pv_gen" in signals else None
    rv = []
    for r in reserves or []:
        d = dict(key=r["key"], duration=float(r.get("duration", 0.0)),
                 price=np.asarray(r["price"], np.float64)[sel])
        if r.get("max") is not None:
            d["max"], d["min"] = np.asarray(r["max"], np.float64)[sel], np.asarray(r["min"], np.float64)[sel]
        rv.append(d)
    lfd = None
    if lf is not None:
        cut = lambda v: np.asarray(v, np.float64)[sel] if np.ndim(v) else float(v)
        lfd = {k: (cut(v) if v is not None and k != "combined" else v) for k, v in lf.items()}
    return market_group(n, dt, bat, blk("da_price"), frd, base=base, ene_min=blk("agg_emin"),
                        ene_max=blk("agg_emax"), binary_relax=relax and flag(sc.get("binary", 0)), name=name,
                        tags=[("day", int(r[0]) // n) for r in sel], reserves=rv, lf=lfd)

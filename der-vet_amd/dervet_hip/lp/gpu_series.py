"""Synthetic scenario sweeps generated on the GPU (BASELINE.json configs 4 / 5; csrc/dvh_series.hip).

``scenarios.sweep_parameters`` + ``scenarios._config4_series`` draw each scenario's perturbations with numpy
(``np.random.Generator(np.random.PCG64(SEED0 + s))``: lognormal load scale, 8,760 AR(1) innovations, six uniforms),
filter them with scipy and cut every window's series on the host: ~4 s per 10,000 scenarios, 7x the solve.
``DeviceSeries`` draws the same numbers on the device (``dvh_series_draws``: one thread per scenario running its PCG64
stream through numpy's ziggurat, csrc/dvh_rng.h) and cuts the device builder's inputs there (``dvh_series_windows``),
so a sweep ships 8 bytes per scenario to the GPU.  Every value is bit-identical to the host generator
(tests/test_gpu_series.py; tests/test_series.py checks the generator's arithmetic against numpy on the CPU), so the
batches -- and every certified result on them -- are unchanged.

``DeviceSeries(ids, solver).config4(ids_subset, n=..., dt=..., E=..., only=...)`` returns the same
``BatteryGroupSpec`` list as ``scenarios.config4(..., spec=True)``, with the per-window series and objective constants
as device tensors (``gpu_builder.pack_specs_device`` consumes either); ``.config5(...)`` the same for
``scenarios.config5(..., spec=True)`` (LP-relaxed ICE, the reliability SOE floor sliced from a device array).
"""
import ctypes
import math

import numpy as np

from .. import _lib
from . import scenarios
from . import tariff as _tariff
from .gpu_builder import BatteryGroupSpec

PHI = 0.9
STEPS = 8760
# the uniform draws after the series, in draw order (scenarios.sweep_parameters)
UNIFORMS = (("price_scale", 0.7, 1.3), ("demand", 5.0, 25.0), ("pv_rated", 0.0, 2000.0), ("E", 500.0, 10000.0),
            ("duration", 2.0, 6.0), ("rte", 0.80, 0.95))


class DeviceSeries:
    """The config-4 generator's draws for `scenario_ids`, held on `solver`'s device."""

    def __init__(self, scenario_ids, solver, device="cuda:0"):
        import torch
        self.ids = np.asarray(list(scenario_ids), np.int64)
        if len(self.ids) and (self.ids.min() < 0 or self.ids.max() >= 2 ** 63 - scenarios.SEED0):
            raise ValueError("scenario ids must be non-negative")
        self.row = {int(s): i for i, s in enumerate(self.ids)}
        self.solver = solver
        self.dev = torch.device(device)
        S = len(self.ids)
        f64 = dict(dtype=torch.float64, device=self.dev)
        self.z0 = torch.empty(S, **f64)
        self.ar = torch.empty((S, STEPS), **f64)
        unif = torch.empty((S, len(UNIFORMS)), **f64)
        seeds = np.ascontiguousarray(scenarios.SEED0 + self.ids, dtype=np.uint64)
        d = _lib.SweepDraws(count=S, steps=STEPS, n_uniform=len(UNIFORMS),
                            seeds=seeds.ctypes.data_as(ctypes.c_void_p), a1=-PHI,
                            innov=float(np.sqrt(1.0 - PHI * PHI)), z0=self.z0.data_ptr(), ar=self.ar.data_ptr(),
                            uniform=unif.data_ptr())
        torch.cuda.synchronize(self.dev)
        solver._check(solver._lib.dvh_series_draws(solver._h, ctypes.byref(d)), "dvh_series_draws")
        z0, u = self.z0.cpu().numpy(), unif.cpu().numpy()
        # Generator.lognormal(0, 0.15) = exp(0.0 + 0.15 z) with the host libm (numpy's random_lognormal); uniform(lo,
        # hi) = lo + (hi - lo) * u (random_uniform)
        P = {"load_scale": np.array([math.exp(0.0 + 0.15 * float(z)) for z in z0])}
        for j, (name, lo, hi) in enumerate(UNIFORMS):
            P[name] = lo + (hi - lo) * u[:, j]
        self.P = P
        per = lambda a: torch.as_tensor(np.ascontiguousarray(a, np.float64), device=self.dev)
        pdis = P["E"] / P["duration"]
        self._scen = dict(load_scale=per(P["load_scale"]), price_scale=per(P["price_scale"]),
                          pv_rated=per(P["pv_rated"]), hp=per(np.zeros(S)),
                          c0_add=per(np.broadcast_to(np.float64(10.0), (S,)) * pdis))
        ri = scenarios.reference_inputs()
        self._site = per(ri["multi_der_site_load"])
        self._prof = per(np.nan_to_num(ri["multi_der_pv_profile"]))
        self._plans = {}

    def parameters(self, ids=None):
        """sweep_parameters(ids) without the innovations (every array bit-identical)."""
        if ids is None:
            return {k: v.copy() for k, v in self.P.items()}
        rows = self.rows(ids)
        return {k: v[rows] for k, v in self.P.items()}

    def rows(self, ids):
        return np.array([self.row[int(s)] for s in ids], np.int64)

    def _plan(self, n, dt, year=2017):
        """Per window id: (t0, T, demand masks) and the per-step energy price on the device, as windows_by_period
        computes them for `year`'s calendar and data/tariff.csv."""
        key = (n, float(dt), int(year))
        if key not in self._plans:
            rep = int(round(1.0 / dt))
            Tall = STEPS * rep
            tar = scenarios.tariff()
            month, he, wd, yr = _tariff.calendar(year, Tall, dt)
            price = _tariff.energy_price(tar, month, he, wd)
            _, d_vals, d_masks = _tariff.demand_charges(tar, month, he, wd)
            if n == "month":
                wid = (yr - yr[0]) * 12 + month - 1
            elif n == "year":
                wid = yr - yr[0]
            else:
                wid = np.arange(Tall) // int(n)
            wins = []
            for w in np.unique(wid):
                sel = np.nonzero(wid == w)[0]
                if not np.array_equal(sel, np.arange(sel[0], sel[0] + len(sel))):
                    raise ValueError(f"window {w} is not a contiguous step range")
                masks = []
                for p in range(len(d_vals)):
                    for mo in np.unique(month[sel]):
                        mk = d_masks[p, sel] & (month[sel] == mo)
                        if mk.any():
                            masks.append(mk)
                wins.append((int(w), int(sel[0]), len(sel), np.array(masks, bool).reshape(-1, len(sel)), sel))
            import torch
            self._plans[key] = (rep, wins, torch.as_tensor(np.ascontiguousarray(price, np.float64), device=self.dev))
        return self._plans[key]

    def config4(self, ids, n="month", dt=1.0, E=None, only=None):
        """``scenarios.config4(ids, n, dt, E, only, spec=True)`` with the series cut on the device."""
        return self._groups(ids, 2017, n, dt, E, only)

    def config5(self, ids, years=20, start_year=2017, emin=None):
        """``scenarios.config5(ids, years, start_year, min_soe, cap_min_soe, spec=True)`` with the series cut on the
        device.  emin: the windows' SOE floor per scenario and hour, a device tensor [len(self.ids), 8760] in this
        series' scenario order (``min_soe_floor``), or None (no floor)."""
        import torch
        ids = np.asarray(list(ids), np.int64)
        P = self.parameters(ids)
        G = len(ids)
        col = lambda v: np.broadcast_to(np.asarray(v, np.float64), (G,)).astype(np.float64, copy=True)
        fuel = 2.5 + P["price_scale"]
        ice = dict(cap=col(750.0) * col(7.0), pmin=col(250.0) * col(7.0),
                   cost=(col(0.086618705) * col(fuel) + col(0.0)) * 1.0)
        floor = None
        if emin is not None:
            floor = emin[torch.as_tensor(self.rows(ids), device=self.dev)]
        out = []
        for y in range(years):
            gy = self._groups(ids, start_year + y, "month", 1.0, None, None, ice=ice, floor=floor)
            if y > 0:
                for g in gy:
                    g.tags = [(t[0], 12 * y + t[1]) for t in g.tags]
            out += gy
        return out

    def min_soe_floor(self, min_soe, cap=True):
        """The config-5 SOE floor on the device: the reliability requirement [len(self.ids), 8760] (host array, this
        series' scenario order), clipped at ulsoc x E (1.0 x E) as scenarios.config5(cap_min_soe=True) does."""
        import torch
        ms = np.asarray(min_soe, np.float64).reshape(len(self.ids), -1)
        if cap:
            ms = np.minimum(ms, (1.0 * self.P["E"])[:, None])
        return torch.as_tensor(np.ascontiguousarray(ms), device=self.dev)

    def _groups(self, ids, year, n, dt, E, only, ice=None, floor=None):
        import torch
        ids = np.asarray(list(ids), np.int64)
        rows = self.rows(ids)
        G = len(ids)
        P = self.parameters(ids)
        Eb = P["E"] if E is None else np.asarray(E, np.float64)
        rep, wins, price = self._plan(n, dt, year)
        rows_d = torch.as_tensor(rows.astype(np.int32), device=self.dev)
        id_list = ids.tolist()
        pdis = P["E"] / P["duration"]
        col = lambda v: np.broadcast_to(np.asarray(v, np.float64), (G,)).astype(np.float64, copy=True)
        scal = dict(E=col(Eb), pch=col(pdis), pdis=col(pdis), rte=col(P["rte"]), sdr=col(0.0) / 100.0,
                    soc_target=col(1.0), ulsoc=col(1.0), llsoc=col(0.0), om=col(0.0))
        specs = []
        for w, t0, T, masks, sel in wins:
            if only is not None and w not in only:
                continue
            J = masks.shape[0]
            rows_i = [np.nonzero(mk)[0] for mk in masks]
            dcm_t = np.concatenate(rows_i).astype(np.int32) if rows_i else np.zeros(0, np.int32)
            dcm_j = np.concatenate([np.full(len(r), j) for j, r in enumerate(rows_i)]).astype(np.int32) \
                if rows_i else np.zeros(0, np.int32)
            demand = np.ascontiguousarray(np.repeat(P["demand"][:, None], J, axis=1)) if J else np.zeros((G, 0))
            f64 = dict(dtype=torch.float64, device=self.dev)
            base, retail, c0 = torch.empty((G, T), **f64), torch.empty((G, T), **f64), torch.empty(G, **f64)
            a = _lib.WindowSeries(G=G, T=T, t0=t0, rep=rep, J=J, count=len(self.ids), hours=STEPS, dt=float(dt),
                                  rows=rows_d.data_ptr(), ar=self.ar.data_ptr(), site_load=self._site.data_ptr(),
                                  pv_profile=self._prof.data_ptr(), price=price.data_ptr(),
                                  load_scale=self._scen["load_scale"].data_ptr(),
                                  price_scale=self._scen["price_scale"].data_ptr(),
                                  pv_rated=self._scen["pv_rated"].data_ptr(), hp=self._scen["hp"].data_ptr(),
                                  c0_add=self._scen["c0_add"].data_ptr(), base=base.data_ptr(),
                                  retail=retail.data_ptr(), c0=c0.data_ptr())
            self.solver._check(self.solver._lib.dvh_series_windows(self.solver._h, ctypes.byref(a)),
                               "dvh_series_windows")
            em = None if floor is None else floor[:, t0 // rep:t0 // rep + T].contiguous() if rep == 1 else None
            if floor is not None and rep != 1:
                raise NotImplementedError("SOE floors are hourly (dt = 1)")
            g = BatteryGroupSpec(T=T, J=J, dt=float(dt), dcm_t=dcm_t, dcm_j=dcm_j, base=base, retail=retail, da=None,
                                 demand=demand, emin=em, emax=None, scal=scal, c0=c0,
                                 tags=[(s, w) for s in id_list], ice=ice)
            g.index = sel
            g.scen = ids
            specs.append(g)
        return specs

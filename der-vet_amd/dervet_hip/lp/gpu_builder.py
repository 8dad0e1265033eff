"""Device-side window builder (dvh_build_battery_group, csrc/dvh_build.hip): the battery + demand-charge +
retail / DA window of ``builder.battery_group`` expanded on the GPU from its compact inputs.

A sweep then ships, per window, the net-load and price series and a dozen battery scalars to HBM (~24 KB for a
T = 744 month) instead of the expanded LP (~170 KB: CSR, bounds, objective), and the expansion runs at HBM speed
instead of numpy's.  Values are bit-identical to the host builder (tests/test_gpu_builder.py), which stays the
parity reference (tests/test_builder.py pins it to the oracle).

``battery_group_spec`` takes battery_group's arguments (the supported subset: no curtailable PV, POI rows or
grid_charge = 0 -- those windows keep the host builder; the LP-relaxed ICE of config 5 is built on the device too) and returns a ``BatteryGroupSpec``; ``pack_specs_device``
lays a list of specs out as one device PackedBatch (group order, then window order, like ``pack_groups``) and
builds every window in place.
"""
import ctypes
from dataclasses import dataclass, field

import numpy as np

from .. import _lib
from ..packed import PackedBatch
from .builder import _col


@dataclass
class BatteryGroupSpec:
    T: int
    J: int
    dt: float
    dcm_t: np.ndarray        # int32 [mI]
    dcm_j: np.ndarray        # int32 [mI]
    base: np.ndarray         # [G, T] net load + hp
    retail: object           # [G, T] or None
    da: object               # [G, T] or None
    demand: np.ndarray       # [G, J]
    emin: object             # [G, T] or None
    emax: object             # [G, T] or None
    scal: dict               # name -> [G]
    c0: np.ndarray           # [G]
    tags: list = field(default_factory=list)
    ice: dict = None         # LP-relaxed ICE: cap, pmin, cost [G] (battery_group `ice`)

    @property
    def G(self):
        return self.base.shape[0]

    @property
    def n(self):
        return (5 if self.ice else 3) * self.T + self.J

    @property
    def m(self):
        return self.T + 1 + len(self.dcm_t) + (2 * self.T if self.ice else 0)

    @property
    def nnz(self):
        return 4 * self.T + (4 if self.ice else 3) * len(self.dcm_t) + (4 * self.T if self.ice else 0)


def battery_group_spec(T, dt, base_load, bat, retail_price=None, da_price=None, demand_masks=None, demand_prices=None,
                       ene_min=None, ene_max=None, name="es", tags=None, pv_curtail_max=None, ice=None, poi=None,
                       grid_charge=True, pv_gen=None):
    """The inputs of ``builder.battery_group(...)`` for the device builder (same arguments and meaning)."""
    if pv_curtail_max is not None or poi is not None or not grid_charge:
        raise NotImplementedError("device builder: curtailable PV, POI rows and grid_charge = 0 use the host builder")
    base_load = np.atleast_2d(np.asarray(base_load, np.float64))
    G = base_load.shape[0]
    masks = np.zeros((0, T), bool) if demand_masks is None else np.asarray(demand_masks, bool)
    masks = masks[masks.any(axis=1)] if len(masks) else masks
    J = masks.shape[0]
    E = _col(bat["E"], G)
    pch, pdis = _col(bat["Pch"], G), _col(bat["Pdis"], G)
    hp = _col(bat.get("hp", 0.0), G)
    base = base_load + hp[:, None]
    rows_i = [np.nonzero(mk)[0] for mk in masks]
    dcm_t = np.concatenate(rows_i).astype(np.int32) if rows_i else np.zeros(0, np.int32)
    dcm_j = np.concatenate([np.full(len(r), j) for j, r in enumerate(rows_i)]).astype(np.int32) if rows_i else \
        np.zeros(0, np.int32)
    retail = None if retail_price is None else _col(retail_price, G, T)
    da = None if da_price is None else _col(da_price, G, T)
    # the objective constant: the terms' constants summed in battery_group's order (DA, DCM, retailETS, fixed_om,
    # var_om), with the same numpy reductions on arrays of the same memory layout (a row sum over a Fortran-ordered
    # product accumulates in a different order than over a C-ordered one)
    c0 = np.zeros(G)
    if da is not None:
        c0 += (da * dt * base).sum(axis=1)
    if J:
        c0 += np.zeros(G)
    if retail is not None:
        c0 += (retail * dt * base).sum(axis=1)
    retail = None if retail is None else np.ascontiguousarray(retail)
    da = None if da is None else np.ascontiguousarray(da)
    c0 += _col(bat.get("fixedOM", 0.0), G) * pdis
    c0 += np.zeros(G)
    if ice is not None:  # the ICE fuel term's constant
        c0 += np.zeros(G)
    scal = dict(E=E, pch=pch, pdis=pdis, rte=_col(bat["rte"], G), sdr=_col(bat.get("sdr", 0.0), G) / 100.0,
                soc_target=_col(bat.get("soc_target", 1.0), G), ulsoc=_col(bat.get("ulsoc", 1.0), G),
                llsoc=_col(bat.get("llsoc", 0.0), G), om=_col(bat.get("OMexpenses", 0.0), G))
    demand = np.zeros((G, 0)) if not J else np.ascontiguousarray(np.asarray(demand_prices, np.float64).reshape(G, J))
    ice_d = None
    if ice is not None:  # battery_group's ICE rows / fuel term, the same products
        ice_d = dict(cap=_col(ice["rated_power"], G) * _col(ice.get("n", 1.0), G),
                     pmin=_col(ice.get("min_power", 0.0), G) * _col(ice.get("n", 1.0), G),
                     cost=(_col(ice["efficiency"], G) * _col(ice["fuel_cost"], G)
                           + _col(ice.get("variable_om_cost", 0.0), G)) * dt)
    return BatteryGroupSpec(T=T, J=J, dt=float(dt), dcm_t=dcm_t, dcm_j=dcm_j, base=np.ascontiguousarray(base),
                            retail=retail, da=da, demand=demand,
                            emin=None if ene_min is None else np.ascontiguousarray(_col(ene_min, G, T)),
                            emax=None if ene_max is None else np.ascontiguousarray(_col(ene_max, G, T)),
                            scal=scal, c0=c0, tags=list(tags) if tags is not None else [None] * G, ice=ice_d)


def desc_of(specs):
    """Descriptors of the packed layout (group order, then window order) and the array sizes."""
    count = sum(s.G for s in specs)
    desc = np.zeros((count, 8), np.int64)
    k = tr = tz = tn = tm = 0
    for s in specs:
        G, n, m, nnz = s.G, s.n, s.m, s.nnz
        kk = np.arange(G, dtype=np.int64)
        desc[k:k + G] = np.stack([np.full(G, n), np.full(G, m), np.full(G, s.T + 1), np.full(G, nnz),
                                  tr + kk * (m + 1), tz + kk * nnz, tn + kk * n, tm + kk * m], axis=1)
        k += G
        tr += G * (m + 1)
        tz += G * nnz
        tn += G * n
        tm += G * m
    return desc, dict(rows=tr, nnz=tz, n=tn, m=tm)


def pack_specs_device(specs, solver, device="cuda:0"):
    """One device PackedBatch (outputs allocated) holding every spec's windows, built on the GPU by the
    solver's handle (its stream; synchronised before returning)."""
    import torch
    desc, sz = desc_of(specs)
    dev = torch.device(device)
    f64 = dict(dtype=torch.float64, device=dev)
    pb = PackedBatch(desc=torch.as_tensor(desc).to(dev),
                     indptr=torch.empty(sz["rows"], dtype=torch.int32, device=dev),
                     indices=torch.empty(sz["nnz"], dtype=torch.int32, device=dev),
                     data=torch.empty(sz["nnz"], **f64), c=torch.empty(sz["n"], **f64),
                     c0=torch.empty(len(desc), **f64), q=torch.empty(sz["m"], **f64),
                     l=torch.empty(sz["n"], **f64), u=torch.empty(sz["n"], **f64)).alloc_outputs()
    torch.cuda.synchronize(dev)
    p = pb.as_ctypes()
    keep = []

    def up(a, t=torch.float64):
        if a is None:
            return None
        if isinstance(a, torch.Tensor):  # already on the device (lp/gpu_series.py)
            if a.device != dev or a.dtype != t or not a.is_contiguous():
                raise ValueError(f"device input must be a contiguous {t} tensor on {dev}")
            return a.data_ptr()
        x = torch.as_tensor(np.ascontiguousarray(a)).to(device=dev, dtype=t)
        keep.append(x)
        return x.data_ptr()

    first = 0
    for s in specs:
        g = _lib.BatteryGroup()
        g.T, g.J, g.G, g.mI, g.dt = s.T, s.J, s.G, len(s.dcm_t), s.dt
        g.has_retail, g.has_da = int(s.retail is not None), int(s.da is not None)
        g.has_emin, g.has_emax = int(s.emin is not None), int(s.emax is not None)
        g.dcm_t, g.dcm_j = up(s.dcm_t, torch.int32), up(s.dcm_j, torch.int32)
        g.base, g.retail, g.da, g.demand = up(s.base), up(s.retail), up(s.da), up(s.demand)
        g.emin, g.emax = up(s.emin), up(s.emax)
        for k, v in s.scal.items():
            setattr(g, k, up(v))
        g.c0 = up(s.c0)
        if s.ice:
            g.has_ice = 1
            g.ice_cap, g.ice_pmin, g.ice_cost = up(s.ice["cap"]), up(s.ice["pmin"]), up(s.ice["cost"])
        torch.cuda.synchronize(dev)
        rc = solver._lib.dvh_build_battery_group(solver._h, ctypes.byref(g), ctypes.byref(p), first)
        if rc != 0:
            raise RuntimeError("dvh_build_battery_group failed: " + solver._lib.dvh_last_error(solver._h).decode())
        first += s.G
    solver._check(solver._lib.dvh_synchronize(solver._h), "dvh_synchronize")
    del keep
    return pb

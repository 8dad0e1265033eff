"""Seeded two-phase schedule for scenario sweeps (BASELINE config 4 / 5; DER-VET's sensitivity loop,
``dervet/DERVET.py:75``, runs the same windows for many perturbed cases).

A sweep solves the same window (same month, same CSR pattern) for thousands of perturbed scenarios.  Instead
of starting every PDHG run from zero, the schedule

  1. solves a SEED subset of the scenarios cold (every ``stride``-th scenario in order of a similarity key,
     the battery energy rating by default), then
  2. solves every other scenario's window warm, from its nearest seed's solution of the same window
     (``dvh_options.warm_start``): bounded columns are scaled by the ratio of the two windows' upper bounds
     (charge / discharge power, energy), and, for the plain battery + DCM shape (x = [ch, dis, ene, tau]),
     the SOE-row duals by the ratio of the mean energy prices and the DCM-row duals by the ratio of the demand
     charges.

Every window is still solved to the same relative KKT tolerance and the same statuses; only the starting
point changes (``scripts/warm_study.py``: 3,351 -> 2,316 mean iterations on config-4 windows started from a
neighbour).  The two phases are two ``dvh_solve_packed_device`` calls on sub-ranges of ONE packed batch (seed
windows packed first), and the transfer between them is a device-side gather on the solver's stream.
"""
import os
from dataclasses import dataclass

import numpy as np

from .packed import PackedBatch


def seed_split(keys, stride, features=None, cover=False):
    """Scenario positions -> (seed positions, rest positions, partner) with `partner[i]` the index into the
    seed list of rest position `rest[i]`'s nearest seed in key order.  Seeds are every `stride`-th scenario
    in key order, starting at stride // 2 so that each seed sits in the middle of its neighbourhood.
    features [S, d] (optional): the partner is instead the nearest seed in these features (each standardised
    to unit variance); with cover=True the seeds themselves are chosen by greedy farthest-point sampling in
    those features."""
    keys = np.asarray(keys, np.float64)
    S = len(keys)
    stride = max(int(stride), 1)
    if stride == 1 or S < 2:
        return np.arange(S), np.zeros(0, np.int64), np.zeros(0, np.int64)
    order = np.argsort(keys, kind="stable")
    pos = np.arange(S)
    seed_pos = np.arange(min(stride // 2, S - 1), S, stride)           # positions in key order
    is_seed = np.zeros(S, bool)
    is_seed[seed_pos] = True
    rest_pos = pos[~is_seed]
    near = np.clip(np.searchsorted(seed_pos, rest_pos), 0, len(seed_pos) - 1)
    left = np.clip(near - 1, 0, len(seed_pos) - 1)
    pick = np.where(np.abs(seed_pos[left] - rest_pos) <= np.abs(seed_pos[near] - rest_pos), left, near)
    seeds, rest = order[seed_pos], order[rest_pos]
    if features is not None:
        f = standardise(features, S)
        if cover:  # greedy farthest-point seeds in feature space (same count), starting at the key-order seed
            ns = len(seeds)
            sel = [int(seeds[0])]
            dmin = ((f - f[sel[0]]) ** 2).sum(1)
            for _ in range(ns - 1):
                j = int(dmin.argmax())
                sel.append(j)
                dmin = np.minimum(dmin, ((f - f[j]) ** 2).sum(1))
            seeds = np.array(sel, np.int64)
            mask = np.ones(S, bool)
            mask[seeds] = False
            rest = np.nonzero(mask)[0]
        pick = _nearest(f[rest], f[seeds])
    return seeds, rest, pick


def standardise(features, S=None):
    """Features [S, d] scaled to zero mean and unit variance per column (constant columns left unscaled)."""
    f = np.asarray(features, np.float64)
    f = f.reshape(S if S is not None else f.shape[0], -1)
    return (f - f.mean(0)) / np.where(f.std(0) > 0, f.std(0), 1.0)


def affine_weights(fr, fs, idx, w0, lam):
    """Blend weights moved from w0 toward the affine combination of the partners' features that reproduces the row's own:
    per row, w = argmin |F'w - f|^2 + lam |w - w0|^2 subject to sum w = 1 (F: the q partners' features), in closed form
    (a regularised barycentric interpolation; weights may be negative).  fr [R, d], fs [S, d], idx / w0 [R, q]."""
    F = fs[idx]                                                  # [R, q, d]
    q = idx.shape[1]
    A = F @ np.swapaxes(F, 1, 2) + lam * np.eye(q)[None]         # [R, q, q]
    rhs = (F @ fr[:, :, None])[:, :, 0] + lam * w0               # [R, q]
    one = np.ones((len(idx), q))
    sol = np.linalg.solve(A, np.stack([rhs, one], axis=2))      # [R, q, 2]
    ai, a1 = sol[:, :, 0], sol[:, :, 1]
    mu = (ai.sum(1) - 1.0) / a1.sum(1)
    return ai - mu[:, None] * a1


def seed_partners(fr, fs, q, first=None, power=1.0, lam=None):
    """The q nearest seeds of every row of fr among the rows of fs (exact squared distances, nearest first; `first`:
    the nearest already known, e.g. from ``_nearest``) and inverse-distance weights 1 / d^power summing to 1 (a seed at
    distance 0 takes the whole weight); lam: the weights then moved toward the partners' affine combination that
    reproduces the row's features (``affine_weights``).  Returns (idx [R, q] int64, w [R, q] float64)."""
    fr = np.ascontiguousarray(fr, np.float64)
    fs = np.ascontiguousarray(fs, np.float64)
    q = max(1, min(int(q), len(fs)))
    R = len(fr)
    idx = np.zeros((R, q), np.int64)
    w = np.zeros((R, q), np.float64)
    bb = (fs * fs).sum(1)
    for a in range(0, R, 2048):
        # candidates by the expanded form (one GEMM), q + 2 of them to absorb its rounding, then exact distances
        fa = fr[a:a + 2048]
        g = fa @ fs.T
        g *= -2.0
        g += bb[None, :]
        qc = min(q + 2, len(fs))
        cand = np.argpartition(g, qc - 1, axis=1)[:, :qc] if qc < len(fs) else np.tile(np.arange(len(fs)), (len(fa), 1))
        cand.sort(axis=1)  # index order, so that equal distances keep the lower seed first
        dc = ((fa[:, None, :] - fs[cand]) ** 2).sum(-1)
        o = np.argsort(dc, axis=1, kind="stable")[:, :q]
        part = np.take_along_axis(cand, o, 1)
        d = np.zeros((len(fa), len(fs)))
        np.put_along_axis(d, part, np.take_along_axis(dc, o, 1), 1)
        if first is not None:  # keep the exact argmin of _nearest first (ties broken the same way)
            f0 = np.asarray(first[a:a + 2048], np.int64)
            has = (part == f0[:, None]).any(1)
            part[~has, -1] = f0[~has]  # (a tie at the boundary: the known nearest replaces the last one)
            rs = np.nonzero(~has)[0]    # ... with its exact distance (a 0 there was an infinite weight)
            d[rs, f0[rs]] = ((fa[rs] - fs[f0[rs]]) ** 2).sum(1)
            part = np.take_along_axis(part, np.argsort(part != f0[:, None], axis=1, kind="stable"), 1)
        dd = np.sqrt(np.take_along_axis(d, part, 1))
        inv = np.where(dd > 0, 1.0 / np.where(dd > 0, dd, 1.0) ** power, np.inf)
        ww = np.where(np.isinf(inv).any(1, keepdims=True), np.isinf(inv).astype(np.float64), inv)
        w[a:a + 2048] = ww / ww.sum(1, keepdims=True)
        idx[a:a + 2048] = part
    if lam is not None and q > 1:
        w = affine_weights(fr, fs, idx, w, float(lam))
    return idx, w


def _nearest(fr, fs):
    """Index of the nearest row of fs for every row of fr: np.argmin of the exact squared distances
    ((fr_i - fs_j) ** 2).sum() (the first of equal minima).  Ranked by the expanded form |b|^2 - 2 a.b (one small
    GEMM, in place) instead of an [rest, seeds, d] difference array (10,000 scenarios: ~20 ms instead of ~190 ms);
    rows whose best two candidates lie within the expanded form's rounding margin are re-ranked exactly."""
    fr = np.ascontiguousarray(fr, np.float64)
    fs = np.ascontiguousarray(fs, np.float64)
    if len(fr) == 0:
        return np.zeros(0, np.int64)
    bb = (fs * fs).sum(1)
    g = fr @ fs.T
    g *= -2.0
    g += bb[None, :]
    j0 = g.argmin(1)
    rows = np.arange(len(fr))
    tol = 1e-9 * ((fr * fr).sum(1) + bb.max() + 1.0)
    close = ((g <= (g[rows, j0] + tol)[:, None]).sum(1) > 1).nonzero()[0]
    for a in range(0, len(close), 1024):  # near ties: the exact distances, np.argmin's first-minimum rule
        i = close[a:a + 1024]
        j0[i] = ((fr[i, None, :] - fs[None, :, :]) ** 2).sum(-1).argmin(1)
    return j0


# dvh_options for the warm phase: restart checks every 64 iterations, KKT every 2nd check (the cold default is
# 32 / 4).  GPU sweep on 48,000 config-4 windows (profiles/r01h_warm_params*.log): warm phase 2,203 -> 2,152
# iterations, PDHG time of the schedule 376.6 -> 357.2 ms; every other restart / weight setting tried was slower.
# Round 2: KKT at every restart check, but a due check is skipped while its predicted outcome is > 4x eps
# (dvh_options.kkt_predict; a KKT check costs ~6 iterations): PDHG 550 -> 527 ms on the bench batch, 2,073 -> 2,038
# warm iterations (profiles/r02zy_kkt_predict.log).  Round 6: with the cheaper iteration the period was re-measured
# (profiles/r06u_check_period.log, r06w_check_period.log): 56 / 64 / 68 / 72 / 76 / 80 -> 298k / 306k / 309k / 308k /
# 305k / 297k windows/s on one box, but at 68 and at 72 one of the 120,000 bench windows stops 1.40e-6 from HiGHS's
# objective (the KKT test passes at a check that lands elsewhere; profiles/r06x_check_period_72.log): 64 stays.
WARM_OPTIONS = {"check_every": 64, "kkt_every": 1, "kkt_predict": 4}
# dvh_options for the cold seed phase: the defaults (checks every 32, KKT every 4th) with the same KKT gate: on the
# bench's 120,000 windows all cold, PDHG 864.6 -> 824.6 ms at unchanged iterations (profiles/r02zzb_cold_kkt_predict.log)
SEED_OPTIONS = {"kkt_predict": 4}


@dataclass
class _Transfer:
    """One rest group <- its seed group (same window id and CSR pattern)."""
    on_rest: int
    om_rest: int
    on_seed: int
    om_seed: int
    n: int
    m: int
    g_rest: int
    g_seed: int
    local: object        # [g_rest] index into the seed group, or [g_rest, q] for a blend of q partners
    battery_dcm: bool    # x = [ch, dis, ene, tau (1)]: scale the duals too
    T: int
    w_rest: int = 0      # window index of the rest group's first window (packing order)
    w_seed: int = 0      # and of the seed group's
    weights: object = None  # [g_rest, q] the partners' weights (blend), None: one partner


def _scenarios_of(g):
    """The group's scenario ids (tag[0] of each window), from the `scen` array the device series attach, else from
    the tags."""
    s = getattr(g, "scen", None)
    if s is not None:
        return np.asarray(s, np.int64)
    return np.fromiter((t[0] for t in g.tags), np.int64, len(g.tags))


def _window_id(tag):
    return tag[1] if isinstance(tag, tuple) and len(tag) > 1 else tag


def _same_pattern(a, b):
    """Same CSR pattern: host-built groups compare their CSR, device-builder specs the inputs that fix it."""
    if a.n != b.n or a.m != b.m:
        return False
    if hasattr(a, "indices"):
        return np.array_equal(a.indices, b.indices) and np.array_equal(a.indptr, b.indptr)
    return a.T == b.T and np.array_equal(a.dcm_t, b.dcm_t) and np.array_equal(a.dcm_j, b.dcm_j)


def plan(seed_groups, rest_groups, partner_of, blend=None):
    """Transfers from the packed seed windows (packed first) to the rest windows (packed after them).

    partner_of: dict rest scenario id -> seed scenario id (the nearest).  blend (optional): (rest scenario ids [R],
    their partners' seed scenario ids [R, q], weights [R, q]) -- the window starts from the weighted blend of those
    partners.  Groups are matched by window id (tag[1]) and must share the CSR pattern."""
    out = []
    on = om = wk = 0
    seed_at = {}
    for g in seed_groups:
        seed_at[_window_id(g.tags[0])] = (g, on, om, wk)
        on += g.G * g.n
        om += g.G * g.m
        wk += g.G
    # partner_of as sorted arrays: rest scenario -> seed scenario, looked up for a whole group at once
    pk = np.fromiter(partner_of.keys(), np.int64, len(partner_of))
    pv = np.fromiter(partner_of.values(), np.int64, len(partner_of))
    po = np.argsort(pk, kind="stable")
    pk, pv = pk[po], pv[po]
    cols = {}
    if blend is not None:
        b_ids = np.asarray(blend[0], np.int64)
        b_ord = np.argsort(b_ids, kind="stable")
        b_ids = b_ids[b_ord]
        b_seed = np.asarray(blend[1], np.int64)[b_ord]
        b_w = np.asarray(blend[2], np.float64)[b_ord]
    for g in rest_groups:
        wid = _window_id(g.tags[0])
        if wid not in seed_at:
            raise ValueError(f"no seed group for window {wid!r}")
        sg, son, som, swk = seed_at[wid]
        if not _same_pattern(sg, g):
            raise ValueError(f"seed and rest groups of window {wid!r} differ in pattern")
        rs = _scenarios_of(g)
        i = np.minimum(np.searchsorted(pk, rs), max(len(pk) - 1, 0))
        if len(rs) and (len(pk) == 0 or not np.array_equal(pk[i], rs)):
            raise KeyError("a rest scenario has no partner seed")
        key = id(sg)
        if key not in cols:  # the seed group's scenarios, sorted, and their positions in the group
            ss = _scenarios_of(sg)
            so = np.argsort(ss, kind="stable")
            cols[key] = (ss[so], so)
        ss, so = cols[key]
        want = pv[i]
        j = np.minimum(np.searchsorted(ss, want), max(len(ss) - 1, 0))
        if len(want) and (len(ss) == 0 or not np.array_equal(ss[j], want)):
            raise KeyError(f"a partner seed is not in the seed group of window {wid!r}")
        local = so[j].astype(np.int64)
        weights = None
        if blend is not None:  # every partner of the blend, looked up in the seed group as the nearest one is
            ib = np.minimum(np.searchsorted(b_ids, rs), max(len(b_ids) - 1, 0))
            if len(rs) and (len(b_ids) == 0 or not np.array_equal(b_ids[ib], rs)):
                raise KeyError("a rest scenario has no blend partners")
            want_q = b_seed[ib]
            jq = np.minimum(np.searchsorted(ss, want_q), max(len(ss) - 1, 0))
            if want_q.size and (len(ss) == 0 or not np.array_equal(ss[jq], want_q)):
                raise KeyError(f"a blend partner is not in the seed group of window {wid!r}")
            local = so[jq].astype(np.int64)
            weights = b_w[ib]
        out.append(_Transfer(on, om, son, som, g.n, g.m, g.G, sg.G, local,
                             g.n == 3 * g.T + 1 and g.J == 1, g.T, wk, swk, weights))
        on += g.G * g.n
        om += g.G * g.m
        wk += g.G
    return out


def transfer_rows(tr_list):
    """(int32 [windows][q + 2] {window, partner windows (q), T}, float64 [windows][q] weights) of blended transfers,
    for ``dvh_warm_transfer_blend``."""
    rows, wts = [], []
    for t in tr_list:
        loc = np.asarray(t.local, np.int64).reshape(t.g_rest, -1)
        q = loc.shape[1]
        r = np.empty((t.g_rest, q + 2), np.int32)
        r[:, 0] = t.w_rest + np.arange(t.g_rest)
        r[:, 1:q + 1] = t.w_seed + loc
        r[:, q + 1] = t.T if t.battery_dcm else 0
        rows.append(r)
        wts.append(np.ones((t.g_rest, 1)) if t.weights is None else np.asarray(t.weights, np.float64))
    if not rows:
        return np.zeros((0, 3), np.int32), np.zeros((0, 1))
    if len({r.shape[1] for r in rows}) != 1:
        raise ValueError("transfers with different partner counts")
    return np.ascontiguousarray(np.concatenate(rows)), np.ascontiguousarray(np.concatenate(wts))


def transfer_pairs(tr_list):
    """int32 [windows][3] {window, partner window, T (> 0: battery + DCM dual scaling)} of the transfers, for
    ``dvh_warm_transfer`` (the same warm starts as ``transfer``, in one launch on the solver's stream)."""
    parts = []
    for t in tr_list:
        if t.weights is not None:
            raise ValueError("blended transfers: use transfer_rows / dvh_warm_transfer_blend")
        p = np.empty((t.g_rest, 3), np.int32)
        p[:, 0] = t.w_rest + np.arange(t.g_rest)
        p[:, 1] = t.w_seed + np.asarray(t.local, np.int64)
        p[:, 2] = t.T if t.battery_dcm else 0
        parts.append(p)
    return np.ascontiguousarray(np.concatenate(parts)) if parts else np.zeros((0, 3), np.int32)


def transfer_device(solver, tr_list, pb, pairs=None, rows=None):
    """``transfer`` for a device-resident batch through the library (``dvh_warm_transfer``): one launch on the
    solver's stream, ordered after the seed solve and before the warm one; no host-side tensor work.
    rows: ``transfer_rows(tr_list)`` when the caller keeps it (blends)."""
    import ctypes
    if pairs is None and any(t.weights is not None for t in tr_list):  # blends of several partners
        rows, wts = transfer_rows(tr_list) if rows is None else rows
        p = pb.as_ctypes()
        solver._check(solver._lib.dvh_warm_transfer_blend(
            solver._h, ctypes.byref(p), rows.ctypes.data_as(ctypes.c_void_p), wts.ctypes.data_as(ctypes.c_void_p),
            len(rows), rows.shape[1] - 2), "dvh_warm_transfer_blend")
        return
    pairs = transfer_pairs(tr_list) if pairs is None else np.ascontiguousarray(pairs, np.int32)
    if pairs.ndim != 2 or pairs.shape[1] != 3:
        raise ValueError(f"pairs must be [count, 3] {{window, partner, T}}, got shape {pairs.shape}")
    p = pb.as_ctypes()
    solver._check(solver._lib.dvh_warm_transfer(solver._h, ctypes.byref(p), pairs.ctypes.data_as(ctypes.c_void_p),
                                                len(pairs)), "dvh_warm_transfer")


def transfer(tr_list, x, y, c, u):
    """Write warm starts for the rest windows into x / y (torch tensors, device or host) from the seeds'
    solutions already in x / y.  c, u: the packed objective and upper bounds."""
    import torch
    for t in tr_list:
        locs = np.asarray(t.local, np.int64).reshape(t.g_rest, -1)
        wts = None if t.weights is None else torch.as_tensor(np.asarray(t.weights, np.float64), device=x.device)
        Ur = u[t.on_rest:t.on_rest + t.g_rest * t.n].view(t.g_rest, t.n)
        Xb = Yb = None
        for k in range(locs.shape[1]):  # partners in row order (one: the plain transfer)
            loc = torch.as_tensor(locs[:, k], device=x.device)
            Xs = x[t.on_seed:t.on_seed + t.g_seed * t.n].view(t.g_seed, t.n)[loc]
            Us = u[t.on_seed:t.on_seed + t.g_seed * t.n].view(t.g_seed, t.n)[loc]
            ok = torch.isfinite(Ur) & torch.isfinite(Us) & (Us > 0)
            ratio = torch.where(ok, Ur / torch.where(ok, Us, torch.ones_like(Us)), torch.ones_like(Us))
            Xk = Xs * ratio
            Ys = y[t.om_seed:t.om_seed + t.g_seed * t.m].view(t.g_seed, t.m)[loc]
            if t.battery_dcm:
                T = t.T
                Cs = c[t.on_seed:t.on_seed + t.g_seed * t.n].view(t.g_seed, t.n)[loc]
                Cr = c[t.on_rest:t.on_rest + t.g_rest * t.n].view(t.g_rest, t.n)
                cd = Cr[:, 3 * T:3 * T + 1] / Cs[:, 3 * T:3 * T + 1].clamp(min=1e-12)
                cp = Cr[:, :T].abs().mean(1, keepdim=True) / Cs[:, :T].abs().mean(1, keepdim=True).clamp(min=1e-12)
                Ys = torch.cat([Ys[:, :T + 1] * cp, Ys[:, T + 1:] * cd], dim=1)
            if wts is None:
                Xb, Yb = Xk, Ys
            else:
                wk = wts[:, k:k + 1]
                Xb = wk * Xk if Xb is None else Xb + wk * Xk
                Yb = wk * Ys if Yb is None else Yb + wk * Ys
        x[t.on_rest:t.on_rest + t.g_rest * t.n].view(t.g_rest, t.n).copy_(Xb)
        y[t.om_rest:t.om_rest + t.g_rest * t.m].view(t.g_rest, t.m).copy_(Yb)


def sub_batch(pb, a, b):
    """Windows [a, b) of a device PackedBatch as a batch of its own (same flat arrays; the descriptors'
    offsets are absolute, per-window arrays are sliced)."""
    return PackedBatch(desc=pb.desc[a:b], indptr=pb.indptr, indices=pb.indices, data=pb.data, c=pb.c,
                       c0=pb.c0[a:b], q=pb.q, l=pb.l, u=pb.u, x=pb.x, y=pb.y, stats=pb.stats[a:b],
                       istats=pb.istats[a:b])


class SeededSweep:
    """Packs a scenario sweep seed-first and solves it in the two phases of the module docstring.

    make_groups(scenario_ids) -> list of WindowGroup (e.g. ``scenarios.config4``) or of device-builder specs
    (``functools.partial(scenarios.config4, spec=True)``: then ``packed`` is None and ``to_device`` expands the
    windows on the GPU, lp/gpu_builder.py); keys: similarity key per scenario (same order as `scenario_ids`)."""

    def __init__(self, make_groups, scenario_ids, keys, stride=8, features=None, cover=False, blend=1,
                 blend_power=1.0, blend_lam=None):
        from .lp import builder
        ids = np.asarray(list(scenario_ids), np.int64)
        seed_i, rest_i, pick = seed_split(keys, stride, features, cover)
        self.seed_ids, self.rest_ids = ids[seed_i], ids[rest_i]
        partner_of = {int(r): int(self.seed_ids[p]) for r, p in zip(self.rest_ids, pick)}
        # blend > 1 (with features): every rest window starts from the inverse-distance-weighted blend of its `blend`
        # nearest seeds' transferred solutions (algorithm lab, 2,048 scenarios: warm iterations 2,063 -> 1,978 with 3)
        bl = None
        self.blend = 1
        if blend > 1 and features is not None and len(seed_i) > 1 and len(rest_i):
            f = standardise(features, len(ids))
            idx, w = seed_partners(f[rest_i], f[seed_i], blend, first=pick, power=blend_power, lam=blend_lam)
            self.blend = idx.shape[1]
            bl = (self.rest_ids, self.seed_ids[idx], w)
        sg = make_groups(self.seed_ids)
        rg = make_groups(self.rest_ids) if len(self.rest_ids) else []
        self.transfers = plan(sg, rg, partner_of, bl)
        self.pairs = transfer_pairs(self.transfers) if bl is None else None
        self.rows = transfer_rows(self.transfers) if bl is not None else None
        self._order_dev = None
        self.n_seed = sum(g.G for g in sg)
        self.tags = [t for g in sg + rg for t in g.tags]
        self.specs = None
        if sg and not hasattr(sg[0], "indices"):
            from .lp import gpu_builder
            self.specs, self.packed = sg + rg, None
            self.desc = gpu_builder.desc_of(self.specs)[0]
        else:
            self.packed = builder.pack_groups(sg + rg)
            self.desc = np.asarray(self.packed.desc)

    def to_device(self, solver, device):
        """The sweep's packed batch on the device, outputs allocated (specs: built there by solver's handle)."""
        if self.specs is not None:
            from .lp import gpu_builder
            return gpu_builder.pack_specs_device(self.specs, solver, device)
        return self.packed.to_torch(device).alloc_outputs()

    def _order_warm(self, solver, dev):
        """Longest-expected-first launch order for the warm phase (dvh_set_launch_order): a rest window's expected
        cost is its blend's weighted mean of the partner seeds' iteration counts, just solved (the only predictor
        at hand: Spearman 0.18 with the warm count on the bench's 116,256 windows).  The band kernel's persistent
        form takes windows in this order, so only the launch's tail depends on it: PDHG 467.4 -> 463.3 ms per
        bench step (profiles/r04u_ab_band_queue.log; sorted by the windows' own counts, 441 ms, is the ceiling).  On
        the device (torch) apart from the permutation's copy to the host, which the library validates.
        DVH_SWEEP_ORDER=0: packing order (prev / prevasc / random: diagnostics of the r04r study)."""
        if self.rows is None or os.environ.get("DVH_SWEEP_ORDER", "1") == "0":
            return
        import torch
        rows, wts = self.rows
        n_rest = dev.count - self.n_seed
        if len(rows) != n_rest:
            return
        if self._order_dev is None or self._order_dev[0].device != dev.istats.device:
            self._order_dev = (torch.as_tensor(rows[:, 1:-1].astype(np.int64), device=dev.istats.device),
                               torch.as_tensor(wts, device=dev.istats.device),
                               torch.as_tensor(rows[:, 0].astype(np.int64) - self.n_seed, device=dev.istats.device))
        part, w, win = self._order_dev
        iters = dev.istats.view(-1, 2)[:, 1].to(torch.float64)
        if os.environ.get("DVH_SWEEP_ORDER") in ("prev", "prevasc"):  # diagnostic: the previous solve's own counts
            pred = iters[win + self.n_seed] * (-1.0 if os.environ["DVH_SWEEP_ORDER"] == "prevasc" else 1.0)
        elif os.environ.get("DVH_SWEEP_ORDER") == "random":  # diagnostic
            pred = torch.rand(len(win), generator=torch.Generator().manual_seed(7), dtype=torch.float64).to(win.device)
        else:
            pred = (w * iters[part]).sum(1)
        order = win[torch.argsort(pred, descending=True, stable=True)].to(torch.int32).cpu().numpy()
        solver.set_launch_order(order)

    def solve(self, solver, dev, warm_options=None, seed_options=None):
        """dev: this sweep's packed batch on the device (``self.packed.to_torch(..).alloc_outputs()``).
        warm_options: dvh_options fields for the warm phase only (restored afterwards; None: WARM_OPTIONS);
        seed_options: the same for the cold seed phase (None: SEED_OPTIONS).
        Returns the kernel timings {setup_ms, pdhg_ms, total_ms} and the windows per kernel path, summed over
        the two phases."""
        cnt = dev.count
        o0 = solver.options()
        warm_options = dict(WARM_OPTIONS if warm_options is None else warm_options)
        seed_options = dict(SEED_OPTIONS if seed_options is None else seed_options)
        restore = {k: getattr(o0, k) for k in list(warm_options) + list(seed_options)}
        restore["warm_start"] = o0.warm_start
        tm = {"total_ms": 0.0, "setup_ms": 0.0, "pdhg_ms": 0.0}
        paths = {}

        def account():
            for k, v in solver.timing().items():
                tm[k] += v
            for k, v in solver.kernel_stats().items():
                if k.endswith("_windows"):
                    paths[k] = paths.get(k, 0) + v

        solver.set_options(warm_start=0, **seed_options)
        try:
            solver.solve_packed(sub_batch(dev, 0, self.n_seed))
        finally:
            solver.set_options(**restore)
        account()
        if cnt > self.n_seed:
            if dev.x.is_cuda and not os.environ.get("DVH_SWEEP_TORCH_TRANSFER"):
                # one launch on the library's stream (the seed solve has completed on it)
                transfer_device(solver, self.transfers, dev, self.pairs, self.rows)
                self._order_warm(solver, dev)
            else:  # host tensors (tests), or the torch formulation for A/B timing
                transfer(self.transfers, dev.x, dev.y, dev.c, dev.u)
                if dev.x.is_cuda:
                    import torch
                    torch.cuda.synchronize(dev.x.device)  # before the library's stream reads the warm starts
            solver.set_options(warm_start=1, **warm_options)
            try:
                solver.solve_packed(sub_batch(dev, self.n_seed, cnt))
            finally:
                solver.set_options(**restore)
            account()
        return tm, paths

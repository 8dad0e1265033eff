"""Seeded two-phase sweep schedule (dervet_hip/sweep.py): host logic on CPU, the schedule itself on cuda:0.

CPU: seed selection / nearest-seed partners, the seed-first packing, and the warm-start transfer (bound-ratio
scaling of x, price-ratio scaling of the duals) on host tensors against a direct numpy restatement.
GPU: every window of a small config-4 sweep is optimal, objectives within 1e-5 of HiGHS on a sample and of
the all-cold solve, and the warm phase needs fewer iterations.
"""
import numpy as np
import pytest
import torch

from dervet_hip.lp import builder, scenarios
from dervet_hip.sweep import SeededSweep, seed_split, sub_batch, transfer, transfer_pairs


def test_seed_split_partners_are_nearest_in_key_order():
    rng = np.random.default_rng(3)
    keys = rng.uniform(0, 1, 101)
    seeds, rest, pick = seed_split(keys, 8)
    assert len(seeds) + len(rest) == 101 and len(set(seeds) | set(rest)) == 101
    order = np.argsort(keys, kind="stable")
    pos = np.empty(101, int)
    pos[order] = np.arange(101)
    for r, p in zip(rest, pick):
        d = abs(pos[seeds[p]] - pos[r])
        assert d == min(abs(pos[s] - pos[r]) for s in seeds)
    s1, r1, _ = seed_split(keys, 1)
    assert len(s1) == 101 and len(r1) == 0


def test_seeded_packing_and_transfer_on_host():
    ids = np.arange(12)
    keys = scenarios.sweep_parameters(ids)["E"]
    sw = SeededSweep(scenarios.config4, ids, keys, stride=4)
    assert sw.n_seed == 12 * len(sw.seed_ids) and sw.packed.count == 12 * 12
    # seeds packed first, every window once
    assert sorted(sw.tags) == sorted((int(s), w) for s in ids for w in range(12))
    assert {t[0] for t in sw.tags[:sw.n_seed]} == set(int(s) for s in sw.seed_ids)
    pb = sw.packed.to_torch("cpu").alloc_outputs()
    g = torch.Generator().manual_seed(0)
    pb.x.copy_(torch.randn(pb.x.shape, generator=g, dtype=torch.float64))
    pb.y.copy_(torch.randn(pb.y.shape, generator=g, dtype=torch.float64))
    x0, y0 = pb.x.clone(), pb.y.clone()
    transfer(sw.transfers, pb.x, pb.y, pb.c, pb.u)
    desc = np.asarray(sw.packed.desc)
    for tr in sw.transfers:
        for i in range(tr.g_rest):
            partner_local = int(tr.local[i])
            on_r, on_s = tr.on_rest + i * tr.n, tr.on_seed + partner_local * tr.n
            om_r, om_s = tr.om_rest + i * tr.m, tr.om_seed + partner_local * tr.m
            u_r, u_s = sw.packed.u[on_r:on_r + tr.n], sw.packed.u[on_s:on_s + tr.n]
            ok = np.isfinite(u_r) & np.isfinite(u_s) & (u_s > 0)
            ratio = np.where(ok, u_r / np.where(ok, u_s, 1.0), 1.0)
            np.testing.assert_allclose(pb.x[on_r:on_r + tr.n].numpy(), x0[on_s:on_s + tr.n].numpy() * ratio,
                                       rtol=1e-15, atol=0)
            assert tr.battery_dcm  # config-4 windows: x = [ch, dis, ene, tau]
            T = tr.T
            c_r, c_s = sw.packed.c[on_r:on_r + tr.n], sw.packed.c[on_s:on_s + tr.n]
            cd = c_r[3 * T] / max(c_s[3 * T], 1e-12)
            cp = np.abs(c_r[:T]).mean() / max(np.abs(c_s[:T]).mean(), 1e-12)
            ys = y0[om_s:om_s + tr.m].numpy()
            want = np.concatenate([ys[:T + 1] * cp, ys[T + 1:] * cd])
            np.testing.assert_allclose(pb.y[om_r:om_r + tr.m].numpy(), want, rtol=1e-14, atol=0)
    # seed windows untouched
    ns_n = int(desc[sw.n_seed, 6])
    assert torch.equal(pb.x[:ns_n], x0[:ns_n])
    # sub-batch views keep absolute offsets and slice the per-window arrays
    sb = sub_batch(pb, sw.n_seed, pb.count)
    assert sb.count == pb.count - sw.n_seed and int(sb.desc[0, 6]) == ns_n
    assert sb.c0.shape[0] == sb.count and sb.stats.shape[0] == sb.count


def test_transfer_pairs_name_each_rest_window_and_its_seed_partner():
    ids = np.arange(12)
    keys = scenarios.sweep_parameters(ids)["E"]
    sw = SeededSweep(scenarios.config4, ids, keys, stride=4)
    pairs = transfer_pairs(sw.transfers)
    assert pairs.dtype == np.int32 and pairs.shape == (sw.packed.count - sw.n_seed, 3)
    assert sorted(pairs[:, 0].tolist()) == list(range(sw.n_seed, sw.packed.count))
    seeds = set(int(s) for s in sw.seed_ids)
    for w, p, T in pairs:
        assert p < sw.n_seed and sw.tags[p][0] in seeds and sw.tags[p][1] == sw.tags[w][1]
        assert T == int(sw.desc[w, 2]) - 1  # battery + DCM windows: dual scaling with the window's T


@pytest.mark.gpu
def test_device_transfer_equals_host_transfer():
    """dvh_warm_transfer (one launch) gives the torch transfer's warm starts: x bit for bit, y to rounding (the
    mean |c| is summed in another order)."""
    from dervet_hip import BatchSolver
    from dervet_hip.sweep import transfer_device
    ids = np.arange(40)
    keys = scenarios.sweep_parameters(ids)["E"]
    sw = SeededSweep(scenarios.config4, ids, keys, stride=8)
    host = sw.packed.to_torch("cpu").alloc_outputs()
    g = torch.Generator().manual_seed(1)
    host.x.copy_(torch.randn(host.x.shape, generator=g, dtype=torch.float64))
    host.y.copy_(torch.randn(host.y.shape, generator=g, dtype=torch.float64))
    dev = sw.packed.to_torch("cuda:0").alloc_outputs()
    dev.x.copy_(host.x)
    dev.y.copy_(host.y)
    transfer(sw.transfers, host.x, host.y, host.c, host.u)
    with BatchSolver(0) as s:
        transfer_device(s, sw.transfers, dev)
        for bad in ([[0, 0, 0]],                 # a window paired with itself
                    [[5, 1, 0], [1, 2, 0]],      # a partner that is itself a listed window
                    [[5, 1, 0], [5, 2, 0]]):     # a window listed twice
            with pytest.raises(Exception):
                transfer_device(s, sw.transfers, dev, np.array(bad, np.int32))
    assert torch.equal(dev.x.cpu(), host.x)
    np.testing.assert_allclose(dev.y.cpu().numpy(), host.y.numpy(), rtol=1e-14, atol=0)


def test_multi_year_config5_sweep_pairs_windows_of_the_same_year_and_month():
    """Config 5 is solved several opt years per batch (bench_configs.py --c5-batch-years): window ids run 12 y +
    month over the horizon, so every warm window starts from its seed's window of the same year and month."""
    ids = np.arange(8)
    keys = scenarios.sweep_parameters(ids)["E"]
    sw = SeededSweep(lambda v: scenarios.config5(v, years=2), ids, keys, stride=4)
    assert sorted(sw.tags) == sorted((int(s), w) for s in ids for w in range(24))
    desc = np.asarray(sw.packed.desc)
    tag_at = {int(desc[k, 6]): sw.tags[k] for k in range(sw.packed.count)}
    checked = 0
    for tr in sw.transfers:
        for i in range(tr.g_rest):
            rest = tag_at[tr.on_rest + i * tr.n]
            seed = tag_at[tr.on_seed + int(tr.local[i]) * tr.n]
            assert rest[1] == seed[1] and seed[0] in set(int(s) for s in sw.seed_ids)
            checked += 1
    assert checked == sw.packed.count - sw.n_seed


@pytest.mark.gpu
def test_seeded_sweep_on_gpu_matches_cold_and_highs():
    from dervet_hip import BatchSolver
    from oracle import window_lp
    ids = np.arange(64)
    sw = SeededSweep(scenarios.config4, ids, scenarios.sweep_parameters(ids)["E"], stride=8)
    dev = sw.packed.to_torch("cuda:0").alloc_outputs()
    with BatchSolver(0) as s:
        _, paths = sw.solve(s, dev)
        assert s.options().warm_start == 0  # restored
        st, ist = dev.stats.cpu().numpy(), dev.istats.cpu().numpy()
        assert (ist[:, 0] == 0).all() and sum(paths.values()) == sw.packed.count
        cold = builder.pack_groups(scenarios.config4(ids)).to_torch("cuda:0").alloc_outputs()
        s.solve_packed(cold)
        cst, cist = cold.stats.cpu().numpy(), cold.istats.cpu().numpy()
    ctags = [t for g in scenarios.config4(ids) for t in g.tags]
    cobj = {t: cst[k, 0] for k, t in enumerate(ctags)}
    rel = [abs(st[k, 0] - cobj[t]) / max(abs(cobj[t]), 1.0) for k, t in enumerate(sw.tags)]
    assert max(rel) <= 1e-5  # both within the objective-error termination (eps_obj 1e-6) of the optimum
    assert ist[sw.n_seed:, 1].mean() < 0.85 * cist[:, 1].mean()
    # every window against HiGHS (the north_star gate: objective within 1e-5, primal residual <= 1e-6)
    from oracle import cpu_baseline
    lps = [window_lp.from_packed_window(sw.packed.window(k)) for k in range(sw.packed.count)]
    hobj, hst, _, _ = cpu_baseline.highs_batch(lps, 8)
    assert (hst == 0).all()
    err = np.abs(st[:, 0] - hobj) / np.maximum(np.abs(hobj), 1.0)
    assert err.max() <= 1e-5, (int(err.argmax()), float(err.max()))
    assert st[:, 1].max() <= 1e-6


def test_seed_split_feature_partners_are_nearest_in_standardised_features():
    rng = np.random.default_rng(5)
    keys = rng.uniform(0, 1, 300)
    feats = np.stack([rng.normal(0, 10, 300), rng.normal(0, 0.1, 300)], 1)
    seeds, rest, pick = seed_split(keys, 16, feats)
    f = (feats - feats.mean(0)) / feats.std(0)
    for r, p in zip(rest, pick):
        d = ((f[seeds] - f[r]) ** 2).sum(1)
        assert d[p] == d.min()


@pytest.mark.gpu
def test_config5_multi_year_seeded_sweep_on_gpu_matches_highs():
    """BASELINE config 5 as bench_configs.py runs it: the GPU min-SOE requirement (dvh_outage_min_soe, capped at E),
    several opt years in one seeded sweep batch (window ids 12 y + month), warm starts by dvh_warm_transfer, the
    LP-relaxed ICE band kernel; every window optimal and within 1e-5 of HiGHS with primal residual <= 1e-6."""
    from dervet_hip import BatchSolver
    from oracle import cpu_baseline, window_lp
    ids = np.arange(16)
    with BatchSolver(0) as s:
        ms = scenarios.config5_min_soe(ids, s)
        P = scenarios.sweep_parameters(ids)
        sw = SeededSweep(lambda v: scenarios.config5(v, years=2, min_soe=ms[np.asarray(list(v))], cap_min_soe=True),
                         ids, P["E"], stride=8, features=scenarios.sweep_features(P))
        dev = sw.packed.to_torch("cuda:0").alloc_outputs()
        _, paths = sw.solve(s, dev)
        st, ist = dev.stats.cpu().numpy(), dev.istats.cpu().numpy()
    assert sw.packed.count == 16 * 24 and paths.get("band_windows", 0) == sw.packed.count, paths
    assert (ist[:, 0] == 0).all()
    lps = [window_lp.from_packed_window(sw.packed.window(k)) for k in range(sw.packed.count)]
    hobj, hst, _, _ = cpu_baseline.highs_batch(lps, 8)
    assert (hst == 0).all()
    err = np.abs(st[:, 0] - hobj) / np.maximum(np.abs(hobj), 1.0)
    assert err.max() <= 1e-5, (int(err.argmax()), float(err.max()))
    assert st[:, 1].max() <= 1e-6


def test_nearest_seed_search_equals_the_exact_argmin_with_ties():
    """sweep._nearest ranks by the expanded |b|^2 - 2 a.b form and re-ranks near ties exactly: the partners are
    np.argmin of the exact squared distances (first of equal minima), including exact ties and duplicate seeds."""
    from dervet_hip.sweep import _nearest
    rng = np.random.default_rng(11)
    fs = rng.normal(0, 1, (300, 5))
    fs[7] = fs[3]                                  # duplicate seeds: the first index wins
    fr = np.concatenate([rng.normal(0, 1, (4000, 5)), fs[:50] + 1e-13, (fs[10] + fs[11])[None] / 2.0])
    ref = ((fr[:, None, :] - fs[None, :, :]) ** 2).sum(-1).argmin(1)
    assert np.array_equal(_nearest(fr, fs), ref)
    assert np.array_equal(_nearest(fr[:3], fs[:2]), ((fr[:3, None] - fs[None, :2]) ** 2).sum(-1).argmin(1))


def test_seed_partners_nearest_first_and_inverse_distance_weights():
    from dervet_hip.sweep import _nearest, seed_partners
    rng = np.random.default_rng(7)
    fs = rng.normal(0, 1, (40, 3))
    fr = np.concatenate([rng.normal(0, 1, (500, 3)), fs[5:6]])  # the last row sits on seed 5
    first = _nearest(fr, fs)
    idx, w = seed_partners(fr, fs, 3, first=first)
    assert idx.shape == (501, 3) and np.array_equal(idx[:, 0], first)
    d = np.sqrt(((fr[:, None, :] - fs[None, :, :]) ** 2).sum(-1))
    for i in range(500):
        assert set(idx[i]) == set(np.argsort(d[i], kind="stable")[:3])
        inv = 1.0 / d[i, idx[i]]
        np.testing.assert_allclose(w[i], inv / inv.sum(), rtol=1e-14)
    assert w[500, 0] == 1.0 and (w[500, 1:] == 0.0).all()  # a seed at distance 0 takes the whole weight


def test_seed_partners_substituted_nearest_gets_its_own_distance():
    """when the known nearest seed is not among the candidates (a tie at the boundary, here forced by
    passing a `first` that is not the nearest), it replaces the last partner WITH its exact distance -- not 0, which
    made its inverse-distance weight infinite and collapsed the blend onto it."""
    from dervet_hip.sweep import seed_partners
    rng = np.random.default_rng(3)
    fs = rng.normal(0, 1, (20, 2))
    fr = rng.normal(0, 1, (50, 2))
    d = np.sqrt(((fr[:, None, :] - fs[None, :, :]) ** 2).sum(-1))
    first = np.argsort(d, axis=1)[:, -1]          # the farthest seed, certainly not a candidate
    idx, w = seed_partners(fr, fs, 4, first=first)
    assert np.array_equal(idx[:, 0], first)
    for i in range(len(fr)):
        inv = 1.0 / d[i, idx[i]]
        np.testing.assert_allclose(w[i], inv / inv.sum(), rtol=1e-13)
        assert w[i, 0] < 0.5


def test_blended_transfer_on_host_is_the_weighted_sum_of_partner_transfers():
    """SeededSweep(blend=3): every rest window starts from the weighted sum of its three nearest seeds' transferred
    solutions (the single-partner transfer of each, weights summing to 1); transfer_rows names them for the device."""
    from dervet_hip.sweep import transfer_rows
    ids = np.arange(24)
    P = scenarios.sweep_parameters(ids)
    sw = SeededSweep(scenarios.config4, ids, P["E"], stride=4, features=scenarios.sweep_features(P), blend=3)
    assert sw.blend == 3 and sw.pairs is None
    pb = sw.packed.to_torch("cpu").alloc_outputs()
    g = torch.Generator().manual_seed(2)
    pb.x.copy_(torch.randn(pb.x.shape, generator=g, dtype=torch.float64))
    pb.y.copy_(torch.randn(pb.y.shape, generator=g, dtype=torch.float64))
    x0, y0 = pb.x.clone(), pb.y.clone()
    transfer(sw.transfers, pb.x, pb.y, pb.c, pb.u)
    rows, wts = transfer_rows(sw.transfers)
    assert rows.shape == (sw.packed.count - sw.n_seed, 5) and wts.shape == (rows.shape[0], 3)
    np.testing.assert_allclose(wts.sum(1), 1.0, rtol=1e-14)
    desc = np.asarray(sw.packed.desc)
    u, c = sw.packed.u, sw.packed.c
    for r in rows[::7]:
        w, T = int(r[0]), int(r[4])
        on_r, om_r, n, m = int(desc[w, 6]), int(desc[w, 7]), int(desc[w, 0]), int(desc[w, 1])
        wx, wy = np.zeros(n), np.zeros(m)
        for k, p in enumerate(r[1:4]):
            on_s, om_s = int(desc[p, 6]), int(desc[p, 7])
            ok = np.isfinite(u[on_r:on_r + n]) & np.isfinite(u[on_s:on_s + n]) & (u[on_s:on_s + n] > 0)
            ratio = np.where(ok, u[on_r:on_r + n] / np.where(ok, u[on_s:on_s + n], 1.0), 1.0)
            cd = c[on_r + 3 * T] / max(c[on_s + 3 * T], 1e-12)
            cp = np.abs(c[on_r:on_r + T]).mean() / max(np.abs(c[on_s:on_s + T]).mean(), 1e-12)
            ys = y0[om_s:om_s + m].numpy()
            wk = wts[list(rows[:, 0]).index(w), k]
            wx += wk * (x0[on_s:on_s + n].numpy() * ratio)
            wy += wk * np.concatenate([ys[:T + 1] * cp, ys[T + 1:] * cd])
        np.testing.assert_allclose(pb.x[on_r:on_r + n].numpy(), wx, rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(pb.y[om_r:om_r + m].numpy(), wy, rtol=1e-13, atol=1e-13)
    with pytest.raises(ValueError):
        transfer_pairs(sw.transfers)


@pytest.mark.gpu
def test_device_blend_transfer_equals_host_blend_transfer():
    """dvh_warm_transfer_blend (one launch) gives the torch blend's warm starts to rounding, and q = 1 with weight 1
    is dvh_warm_transfer bit for bit."""
    from dervet_hip import BatchSolver
    from dervet_hip.sweep import transfer_device, transfer_rows
    ids = np.arange(48)
    P = scenarios.sweep_parameters(ids)
    sw = SeededSweep(scenarios.config4, ids, P["E"], stride=8, features=scenarios.sweep_features(P), blend=3)
    host = sw.packed.to_torch("cpu").alloc_outputs()
    g = torch.Generator().manual_seed(4)
    host.x.copy_(torch.randn(host.x.shape, generator=g, dtype=torch.float64))
    host.y.copy_(torch.randn(host.y.shape, generator=g, dtype=torch.float64))
    dev = sw.packed.to_torch("cuda:0").alloc_outputs()
    dev.x.copy_(host.x)
    dev.y.copy_(host.y)
    x0, y0 = host.x.clone(), host.y.clone()
    transfer(sw.transfers, host.x, host.y, host.c, host.u)
    with BatchSolver(0) as s:
        transfer_device(s, sw.transfers, dev)
        np.testing.assert_allclose(dev.x.cpu().numpy(), host.x.numpy(), rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(dev.y.cpu().numpy(), host.y.numpy(), rtol=1e-13, atol=1e-13)
        # one partner, weight 1, through the blend entry == the plain transfer
        import ctypes
        sw1 = SeededSweep(scenarios.config4, ids, P["E"], stride=8, features=scenarios.sweep_features(P))
        d1 = sw1.packed.to_torch("cuda:0").alloc_outputs()
        d2 = sw1.packed.to_torch("cuda:0").alloc_outputs()
        for d in (d1, d2):
            d.x.copy_(x0.to("cuda:0"))
            d.y.copy_(y0.to("cuda:0"))
        transfer_device(s, sw1.transfers, d1)
        rows, wts = transfer_rows(sw1.transfers)
        p = d2.as_ctypes()
        s._check(s._lib.dvh_warm_transfer_blend(s._h, ctypes.byref(p), rows.ctypes.data_as(ctypes.c_void_p),
                                                wts.ctypes.data_as(ctypes.c_void_p), len(rows), 1), "blend")
        assert torch.equal(d1.x, d2.x) and torch.equal(d1.y, d2.y)
        bad = np.array([[5, 1, 2, 3, 0]], np.int32)
        with pytest.raises(Exception):  # a non-finite weight
            w_bad = np.array([[0.5, np.nan, 0.5]])
            s._check(s._lib.dvh_warm_transfer_blend(s._h, ctypes.byref(p), bad.ctypes.data_as(ctypes.c_void_p),
                                                    w_bad.ctypes.data_as(ctypes.c_void_p), 1, 3), "blend")


def test_affine_blend_weights_sum_to_one_and_approach_the_features():
    """sweep.affine_weights (bench.py --blend-lam): the weights sum to 1, large lam returns the inverse-distance
    weights, small lam reproduces the window's features from its partners' (when q > d)."""
    from dervet_hip.sweep import affine_weights, seed_partners
    rng = np.random.default_rng(3)
    fs, fr = rng.normal(size=(40, 3)), rng.normal(size=(25, 3))
    idx, w0 = seed_partners(fr, fs, 8)
    for lam in (1e-9, 1.0, 1e9):
        w = affine_weights(fr, fs, idx, w0, lam)
        np.testing.assert_allclose(w.sum(1), 1.0, rtol=0, atol=1e-9)
    np.testing.assert_allclose(affine_weights(fr, fs, idx, w0, 1e9), w0, atol=1e-7)
    w = affine_weights(fr, fs, idx, w0, 1e-9)
    np.testing.assert_allclose((w[:, :, None] * fs[idx]).sum(1), fr, atol=1e-6)
    i1, w1 = seed_partners(fr, fs, 8, lam=1.0)
    assert np.array_equal(i1, idx)
    np.testing.assert_allclose(w1, affine_weights(fr, fs, idx, w0, 1.0))

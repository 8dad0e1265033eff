"""GPU: the scenario series generated on the device (csrc/dvh_series.hip via lp/gpu_series.py) are bit-identical to
the host generator (scenarios.sweep_parameters / _config4_series / config4(spec=True)): every per-scenario draw, every
AR(1) series, every window's base / retail series and objective constant -- so the packed batches, and every result
certified on them, are unchanged."""
import numpy as np
import pytest
import torch

from dervet_hip.lp import gpu_builder, gpu_series, scenarios

pytestmark = pytest.mark.gpu


def _bits(a):
    a = a.cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    return np.ascontiguousarray(a, np.float64).view(np.int64)


def test_draws_equal_numpy_on_2000_scenarios(gpu_solver):
    ids = np.arange(2000) * 5 + 7          # ~17.5 M normals: ~4,500 ziggurat tail draws, ~200,000 wedge tests
    ds = gpu_series.DeviceSeries(ids, gpu_solver)
    P = scenarios.sweep_parameters(ids)
    for k, v in ds.P.items():
        assert np.array_equal(_bits(v), _bits(P[k])), k
    e = P["eps"]
    e[:, 1:] *= np.sqrt(1.0 - 0.9 * 0.9)
    from scipy.signal import lfilter
    a = lfilter([1.0], [1.0, -0.9], e, axis=1)
    assert np.array_equal(_bits(ds.ar), _bits(a))


@pytest.mark.parametrize("n,dt,ids", [("month", 1.0, [3, 11, 40, 41, 977]), ("month", 1.0, [977]),
                                     ("year", 1.0, [3, 11, 40]), ("year", 1.0, [41]), ("month", 0.25, [5, 6])])
def test_window_specs_equal_the_host_specs(gpu_solver, n, dt, ids):
    """G > 1: numpy sums the objective constant in step order; G = 1 (a lone window): pairwise."""
    ds = gpu_series.DeviceSeries(range(1000), gpu_solver)
    dev = ds.config4(ids, n=n, dt=dt, E=None if n == "month" else np.array([900.0] * len(ids)))
    host = scenarios.config4(ids, n=n, dt=dt, E=None if n == "month" else np.array([900.0] * len(ids)), spec=True)
    assert len(dev) == len(host)
    for d, h in zip(dev, host):
        assert (d.T, d.J, d.dt, d.tags) == (h.T, h.J, h.dt, h.tags)
        assert np.array_equal(d.dcm_t, h.dcm_t) and np.array_equal(d.dcm_j, h.dcm_j)
        for f in ("base", "retail", "c0", "demand"):
            assert np.array_equal(_bits(getattr(d, f)), _bits(getattr(h, f))), f
        assert d.da is None and h.da is None and d.emin is None and h.emin is None
        for k in h.scal:
            assert np.array_equal(_bits(d.scal[k]), _bits(h.scal[k])), k


def test_packed_batch_from_device_series_equals_host_spec_batch(gpu_solver):
    ids = list(range(0, 64))
    ds = gpu_series.DeviceSeries(ids, gpu_solver)
    a = gpu_builder.pack_specs_device(ds.config4(ids), gpu_solver)
    b = gpu_builder.pack_specs_device(scenarios.config4(ids, spec=True), gpu_solver)
    for f in ("desc", "indptr", "indices", "data", "c", "c0", "q", "l", "u"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f


def test_bad_rows_are_refused(gpu_solver):
    """dvh_series_windows range-checks every window's scenario row on the device (DVH_ERR_ARG, nothing read)."""
    import ctypes

    from dervet_hip import _lib
    ds = gpu_series.DeviceSeries([1, 2], gpu_solver)
    rep, wins, price = ds._plan("month", 1.0)
    _, t0, T, _, _ = wins[0]
    f64 = dict(dtype=torch.float64, device="cuda:0")
    rows = torch.tensor([0, 2], dtype=torch.int32, device="cuda:0")   # row 2 of a 2-scenario series
    out = [torch.empty((2, T), **f64), torch.empty((2, T), **f64), torch.empty(2, **f64)]
    sc = ds._scen
    a = _lib.WindowSeries(G=2, T=T, t0=t0, rep=1, J=1, count=2, hours=8760, dt=1.0, rows=rows.data_ptr(),
                          ar=ds.ar.data_ptr(), site_load=ds._site.data_ptr(), pv_profile=ds._prof.data_ptr(),
                          price=price.data_ptr(), load_scale=sc["load_scale"].data_ptr(),
                          price_scale=sc["price_scale"].data_ptr(), pv_rated=sc["pv_rated"].data_ptr(),
                          hp=sc["hp"].data_ptr(), c0_add=sc["c0_add"].data_ptr(), base=out[0].data_ptr(),
                          retail=out[1].data_ptr(), c0=out[2].data_ptr())
    assert gpu_solver._lib.dvh_series_windows(gpu_solver._h, ctypes.byref(a)) == _lib.DVH_ERR_ARG
    assert b"row" in gpu_solver._lib.dvh_last_error(gpu_solver._h)
    a.t0 = 8760 - T + 1                    # a window past the end of the series: refused on the host
    assert gpu_solver._lib.dvh_series_windows(gpu_solver._h, ctypes.byref(a)) == _lib.DVH_ERR_ARG


def test_config5_specs_equal_the_host_specs(gpu_solver):
    """Config 5 (LP-relaxed ICE, the reliability SOE floor clipped at E, two opt years incl. a leap year): the device
    series' specs and the packed batch equal scenarios.config5(spec=True)'s bit for bit."""
    pool = list(range(40))
    ids = [2, 9, 31]
    ds = gpu_series.DeviceSeries(pool, gpu_solver)
    rng = np.random.default_rng(5)
    ms = rng.uniform(0.0, 12000.0, (len(pool), 8760))     # some hours above E: clipped
    dev = ds.config5(ids, years=2, start_year=2019, emin=ds.min_soe_floor(ms))
    host = scenarios.config5(ids, years=2, start_year=2019, min_soe=ms[ids], cap_min_soe=True, spec=True)
    assert len(dev) == len(host) == 24
    for d, h in zip(dev, host):
        assert (d.T, d.J, d.tags) == (h.T, h.J, h.tags)
        for f in ("base", "retail", "c0", "demand", "emin"):
            assert np.array_equal(_bits(getattr(d, f)), _bits(getattr(h, f))), f
        for k in h.ice:
            assert np.array_equal(_bits(d.ice[k]), _bits(h.ice[k])), k
    a = gpu_builder.pack_specs_device(dev, gpu_solver)
    b = gpu_builder.pack_specs_device(host, gpu_solver)
    for f in ("desc", "indptr", "indices", "data", "c", "c0", "q", "l", "u"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f
    gpu_solver.solve_packed(a)
    assert gpu_solver.kernel_stats()["band_windows"] == a.count == 72  # the band-ICE kernel takes every window


def test_host_regenerated_rows_equal_the_host_generator(gpu_solver):
    """The fallback for scenarios whose wedge test the device reports as undecided (dvh_sweep_draws.ambiguous):
    their draws and series are regenerated on the host; the sweep stays bit-identical to the host generator."""
    ids = np.arange(40) * 3 + 1
    ds = gpu_series.DeviceSeries(ids, gpu_solver)
    assert len(ds.host_rows) == 0
    ds.ar[5].zero_()  # what the host path must overwrite
    ds.P["E"][[5, 17]] = 0.0
    ds.regenerate_on_host([5, 17])
    P = scenarios.sweep_parameters(ids)
    for k, v in ds.P.items():
        assert np.array_equal(_bits(v), _bits(P[k])), k
    e = P["eps"]
    e[:, 1:] *= np.sqrt(1.0 - 0.9 * 0.9)
    from scipy.signal import lfilter
    assert np.array_equal(_bits(ds.ar), _bits(lfilter([1.0], [1.0, -0.9], e, axis=1)))

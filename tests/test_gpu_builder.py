"""Device window builder (csrc/dvh_build.hip via lp/gpu_builder.py): the windows it expands in HBM are bit-identical
to the host builder's (builder.pack_groups, itself pinned to the oracle by tests/test_builder.py), and solving them
gives bit-identical results."""
import numpy as np
import pytest
import torch

from dervet_hip.lp import builder, gpu_builder, scenarios

pytestmark = pytest.mark.gpu

FIELDS = ("desc", "indptr", "indices", "data", "c", "c0", "q", "l", "u")


def _assert_same(dev, host):
    for f in FIELDS:
        a = getattr(dev, f).cpu().numpy()
        b = np.asarray(getattr(host, f))
        assert a.dtype == b.dtype and a.shape == b.shape, f
        assert np.array_equal(a, b), (f, np.flatnonzero(a != b)[:5])


def _mixed_case(spec):
    """DA + retail prices, demand charges, SOE floors and ceilings, self-discharge, quarter-hour steps, weekly
    windows with ragged sizes at the end of the series."""
    rng = np.random.default_rng(11)
    S, Tall, dt = 3, 96 * 17 + 40, 0.25
    load = rng.uniform(50, 400, (S, Tall))
    gen = rng.uniform(0, 120, (S, Tall))
    da = rng.normal(40, 15, Tall)
    emin = np.broadcast_to(rng.uniform(0, 200, Tall), (S, Tall))
    emax = np.broadcast_to(rng.uniform(700, 1000, Tall), (S, Tall))
    bat = dict(scenarios.template_battery(), sdr=0.5, soc_target=0.6, ulsoc=0.95, llsoc=0.05, OMexpenses=0.3,
               E=np.array([800.0, 1000.0, 1300.0]))
    return scenarios.windows_by_period(2017, dt, load, gen, bat, tariff_def=scenarios.tariff("data_tariff"),
                                       da_price=da, n=96 * 7, ene_min=emin, ene_max=emax, spec=spec)


@pytest.mark.parametrize("case", ["config4", "config1_da", "mixed", "config5_ice"])
def test_device_builder_is_bit_identical_to_the_host_builder(gpu_solver, case):
    if case == "config4":
        host, spec = scenarios.config4(range(12)), scenarios.config4(range(12), spec=True)
    elif case == "config1_da":
        host = scenarios.config1(with_retail=True)
        ri = scenarios.reference_inputs()
        spec = scenarios.windows_by_period(2017, 1.0, ri["hourly_site_load"][None, :], None,
                                           scenarios.template_battery(), tariff_def=scenarios.tariff("data_tariff"),
                                           da_price=ri["hourly_da_price"][None, :], spec=True)
    elif case == "config5_ice":  # LP-relaxed ICE + reliability SOE floors, a leap year's calendar
        host, spec = (scenarios.config5(range(5), years=1, start_year=2020, spec=f) for f in (False, True))
    else:
        host, spec = _mixed_case(False), _mixed_case(True)
    dev = gpu_builder.pack_specs_device(spec, gpu_solver)
    _assert_same(dev, builder.pack_groups(host))


def test_solving_device_built_windows_equals_host_built(gpu_solver):
    host = builder.pack_groups(scenarios.config4(range(8)))
    hd = host.to_torch("cuda:0").alloc_outputs()
    gpu_solver.solve_packed(hd)
    dd = gpu_builder.pack_specs_device(scenarios.config4(range(8), spec=True), gpu_solver)
    gpu_solver.solve_packed(dd)
    torch.cuda.synchronize()
    for f in ("x", "y", "stats", "istats"):
        assert torch.equal(getattr(hd, f), getattr(dd, f)), f
    assert (dd.istats[:, 0] == 0).all()


def test_seeded_sweep_on_device_built_windows_equals_host_built(gpu_solver):
    """bench.py's default: the seeded sweep over windows expanded on the GPU gives the host-built sweep's results
    bit for bit (same seeds, same warm-start transfers)."""
    import functools

    from dervet_hip.sweep import SeededSweep
    ids = range(40)
    P = scenarios.sweep_parameters(ids)
    out = []
    for make in (scenarios.config4, functools.partial(scenarios.config4, spec=True)):
        sw = SeededSweep(make, ids, P["E"], stride=8, features=scenarios.sweep_features(P))
        dev = sw.to_device(gpu_solver, "cuda:0")
        sw.solve(gpu_solver, dev)
        torch.cuda.synchronize()
        out.append((sw, dev))
    (sh, dh), (sd, dd) = out
    assert sd.packed is None and np.array_equal(sh.desc, sd.desc) and sh.n_seed == sd.n_seed
    for f in FIELDS[1:] + ("x", "y", "stats", "istats"):
        assert torch.equal(getattr(dh, f), getattr(dd, f)), f
    w = dd.window(5)
    assert np.array_equal(w["c"], sh.packed.window(5)["c"])


@pytest.mark.parametrize("field,value", [("dcm_t", "T"), ("dcm_t", -1), ("dcm_j", "J")])
def test_device_builder_rejects_demand_rows_outside_the_window(gpu_solver, field, value):
    """dvh_build_battery_group range-checks the demand-charge rows' steps (< T) and tau columns (< J)
    before the launch, instead of reading base[] and writing column indices outside the window."""
    spec = scenarios.config4(range(1), spec=True)[0]
    bad = np.array(getattr(spec, field), copy=True)
    bad[len(bad) // 2] = getattr(spec, value) if isinstance(value, str) else value
    setattr(spec, field, bad)
    with pytest.raises(RuntimeError, match="demand-charge row"):
        gpu_builder.pack_specs_device([spec], gpu_solver)

"""The device scenario generator's arithmetic on the CPU (csrc/dvh_rng.h compiled by g++ through
tests/native/series_host.cpp; the same header is compiled into dvh_series.hip): SeedSequence + PCG64 words, the
ziggurat normals, the AR(1) filter and the uniforms are bit-identical to numpy / scipy (the host generator,
dervet_hip/lp/scenarios.py), and the restated glibc log1p of the ziggurat tail equals the host libm everywhere the
generator can call it.  numpy's pairwise row summation, which dvh_series.hip restates for the windows' objective
constants, is pinned here too."""
import ctypes
import math
import os
import subprocess

import numpy as np
import pytest
from scipy.signal import lfilter

from dervet_hip.lp import scenarios

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "der-vet_amd", "csrc")


@pytest.fixture(scope="module")
def host(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("series") / "series_host.so")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", "-fPIC", "-shared", "-I", CSRC,
                    os.path.join(HERE, "native", "series_host.cpp"), "-o", so], check=True)
    lib = ctypes.CDLL(so)
    lib.log1p_mismatches.restype = ctypes.c_longlong
    lib.log1p_mismatches.argtypes = [ctypes.c_longlong, ctypes.c_longlong]
    return lib


def test_pcg64_words_equal_numpy(host):
    for seed in (0, 1, 2 ** 32 - 1, 2 ** 32, scenarios.SEED0, scenarios.SEED0 + 9999, 2 ** 63 + 12345):
        out = np.empty(16, np.uint64)
        host.raw_words(ctypes.c_uint64(seed), 16, out.ctypes.data_as(ctypes.c_void_p))
        assert np.array_equal(out, np.random.PCG64(seed).random_raw(16)), seed


def test_log1p_restatement_equals_host_libm(host):
    assert host.log1p_mismatches(2_000_000, 400_000) == 0


def draws(host, ids):
    ids = np.asarray(ids, np.int64)
    S = len(ids)
    seeds = np.ascontiguousarray(scenarios.SEED0 + ids, np.uint64)
    z0, ar, u = np.empty(S), np.empty((S, 8760)), np.empty((S, 6))
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    amb = host.series_draws_host(p(seeds), S, 8760, 6, ctypes.c_double(-0.9), ctypes.c_double(np.sqrt(1.0 - 0.81)),
                                 p(z0), p(ar), p(u))
    return amb, z0, ar, u


def test_scenario_draws_equal_the_host_generator(host):
    ids = list(range(0, 120, 3)) + [9999, 123456]
    amb, z0, ar, u = draws(host, ids)
    assert amb == 0
    P = scenarios.sweep_parameters(ids)
    # numpy's random_lognormal: exp(0.0 + 0.15 z) with the host libm (math.exp calls the same exp)
    assert np.array_equal(np.array([math.exp(0.0 + 0.15 * float(z)) for z in z0]), P["load_scale"])
    for j, (k, lo, hi) in enumerate((("price_scale", 0.7, 1.3), ("demand", 5.0, 25.0), ("pv_rated", 0.0, 2000.0),
                                     ("E", 500.0, 10000.0), ("duration", 2.0, 6.0), ("rte", 0.80, 0.95))):
        assert np.array_equal(lo + (hi - lo) * u[:, j], P[k]), k
    e = P["eps"].copy()
    e[:, 1:] *= np.sqrt(1.0 - 0.9 * 0.9)
    assert np.array_equal(ar, lfilter([1.0], [1.0, -0.9], e, axis=1))


def _pairwise(a):
    """numpy's DOUBLE_pairwise_sum as dvh_series.hip restates it."""
    n = len(a)
    if n < 8:
        r = 0.0
        for v in a:
            r = r + v
        return r
    if n <= 128:
        r = list(a[:8])
        i = 8
        while i < n - n % 8:
            for j in range(8):
                r[j] = r[j] + a[i + j]
            i += 8
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
        for v in a[i:]:
            res = res + v
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return _pairwise(a[:n2]) + _pairwise(a[n2:])


@pytest.mark.parametrize("T", [5, 8, 129, 672, 744, 2976, 8760, 8784])
def test_row_sums_are_pairwise_over_8192_element_buffers(T):
    rng = np.random.default_rng(T)
    A = rng.standard_normal((6, T)) * rng.uniform(0.01, 1000.0, (6, T))
    mine = []
    for r in A:
        acc = 0.0
        for off in range(0, T, 8192):
            acc = acc + _pairwise(list(r[off:off + 8192]))
        mine.append(acc)
    assert np.array_equal(np.array(mine), A.sum(axis=1))


def test_column_selected_window_products_sum_in_step_order():
    """The host windows' series are column selections of [S, steps] arrays (Fortran-ordered), so numpy reduces the
    [G, T] product with the window index innermost: an ordered running sum over t (dvh_series.hip, G > 1)."""
    rng = np.random.default_rng(3)
    A = rng.standard_normal((7, 8760)) * 100.0
    p = A[:, np.arange(744, 1488)] * A[:, np.arange(1488, 2232)]
    assert p.flags["F_CONTIGUOUS"] and not p.flags["C_CONTIGUOUS"]
    acc = np.zeros(7)
    for t in range(p.shape[1]):
        acc = acc + p[:, t]
    assert np.array_equal(acc, p.sum(axis=1))

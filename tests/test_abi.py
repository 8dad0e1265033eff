"""C-ABI contract (CPU only: no compute calls without a GPU).

libdervet_hip.so must load and export every function include/dervet_hip.h declares, the ctypes structs
must match the C layout, and the product path must fail loudly (no CPU fallback) when no GPU is present.
"""
import ctypes
import os
import re

import pytest

from dervet_hip import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dervet_hip.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(dvh_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    names = header_functions()
    assert len(names) >= 10
    for n in names:
        assert hasattr(lib, n), f"{n} declared in dervet_hip.h but not exported"
    assert set(names) == set(_lib.SYMBOLS), "ctypes binding out of sync with the header"


def test_version_and_defaults():
    lib = _lib.load()
    assert lib.dvh_version().decode().startswith("dervet_hip")
    o = _lib.default_options()
    assert o.eps == 1e-6 and o.check_every == 32 and o.kkt_every == 4 and o.max_iters == 100000 and o.kkt_predict == 0
    assert o.restart_artificial == 0.1 and o.primal_weight_theta == 1.0 and o.step_safety == 0.998


def test_struct_layout_matches_c():
    # sizes as laid out by the C compiler for x86-64 (include/dervet_hip.h)
    assert ctypes.sizeof(_lib.Options) == 8 + 4 * 4 + 8 * 6 + 4 * 8
    assert ctypes.sizeof(_lib.LP) == 16 + 8 * 4 + 8 + 8 * 3 + 8
    assert ctypes.sizeof(_lib.Result) == 8 * 2 + 8 * 4 + 8
    assert ctypes.sizeof(_lib.Packed) == 8 + 8 * 4 + 8 * 13


def test_null_handle_errors_are_codes_not_crashes():
    lib = _lib.load()
    assert lib.dvh_destroy(None) == _lib.DVH_ERR_ARG
    assert lib.dvh_solve_batch(None, None, 0, None) == _lib.DVH_ERR_ARG
    assert lib.dvh_last_error(None) == b"null handle"


def test_no_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from dervet_hip import BatchSolver, SolverError
    with pytest.raises(SolverError):
        BatchSolver(0)


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _lib.load(str(tmp_path / "libdervet_hip.so"))

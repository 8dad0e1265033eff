"""dervet_hip -- MI355X-native batched dispatch-LP solver beneath DER-VET's window loop.

Product path: window LPs (built by ``dervet_hip.lp`` or exported from CVXPY) -> ``libdervet_hip.so``
(C ABI in include/dervet_hip.h, HIP kernels for gfx950) -> per-window solutions written back through the
``BatchedMicrogridScenario`` drop-in (``dervet_hip.dropin``; ``dropin.install(batch_cases=True)`` also batches the
sensitivity cases behind ``DERVET.solve``).  A sharded run returns its results through the library's own RCCL
all-gather (``parallel.LibraryGather``).  There is no CPU fallback.
"""
from .solver import BatchSolver, SolverError, WindowLP, WindowResult, version  # noqa: F401
from .packed import PackedBatch, pack  # noqa: F401

__all__ = ["BatchSolver", "SolverError", "WindowLP", "WindowResult", "PackedBatch", "pack", "version"]

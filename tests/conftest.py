import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "der-vet_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libdervet_hip on cuda:0)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def gpu_solver():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected but no GPU is visible (run with -m 'not gpu' on CPU hosts)")
    from dervet_hip import BatchSolver
    s = BatchSolver(0)
    yield s
    s.close()

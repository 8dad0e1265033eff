"""Setup-kernel cost split (dev helper): setup_ms of a config-4 batch for several Ruiz pass counts.
Usage: python scripts/setup_probe.py <scenarios>"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "der-vet_amd"))
import numpy as np  # noqa: E402

from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
pb = builder.pack_groups(scenarios.config4(np.arange(S)))
dev = pb.to_torch("cuda:0").alloc_outputs()
s = BatchSolver(0, max_iters=32)
for ruiz in (10, 10, 5, 1, 0):
    s.set_options(ruiz_iters=ruiz)
    s.solve_packed(dev)
    print(f"ruiz {ruiz:2d}: setup {s.timing()['setup_ms']:.2f} ms for {pb.count} windows", flush=True)

"""Warm-phase parameter sweep (dev helper): the seeded config-4 schedule with different dvh_options for the warm
phase only.  Prints warm-phase iterations and kernel time per variant.

Usage: python scripts/warm_params.py <scenarios> ['<json list of warm-option dicts>']
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "der-vet_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import scenarios  # noqa: E402
from dervet_hip.sweep import SeededSweep  # noqa: E402

VARIANTS = [
    {"check_every": 64, "kkt_every": 2},
    {"check_every": 64, "kkt_every": 2, "power_iters": 48},
    {"check_every": 64, "kkt_every": 2, "power_iters": 32},
    {"check_every": 64, "kkt_every": 2, "power_iters": 16},
    {"check_every": 64, "kkt_every": 2, "ruiz_iters": 5},
    {"check_every": 64, "kkt_every": 2, "restart_sufficient": 0.15},
]


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    variants = json.loads(sys.argv[2]) if len(sys.argv) > 2 else VARIANTS
    ids = np.arange(S)
    P = scenarios.sweep_parameters(ids)
    sw = SeededSweep(scenarios.config4, ids, P["E"], stride=32, features=scenarios.sweep_features(P))
    dev = sw.packed.to_torch("cuda:0").alloc_outputs()
    s = BatchSolver(0)
    ns = sw.n_seed
    base = None
    for v in variants:
        tms = []
        for rep in range(2):
            tm, _ = sw.solve(s, dev, warm_options=v)
            tms.append(tm["pdhg_ms"])
        ist = dev.istats.cpu().numpy()
        obj = dev.stats.cpu().numpy()[:, 0]
        if base is None:
            base = obj.copy()
        rel = np.abs(obj - base) / np.maximum(np.abs(base), 1.0)
        print(f"{str(v):40s} pdhg {min(tms):7.1f} ms  warm iters mean {ist[ns:, 1].mean():7.1f}  p99 "
              f"{np.percentile(ist[ns:, 1], 99):.0f}  optimal {(ist[:, 0] == 0).sum()}/{len(ist)}  "
              f"max obj diff vs default {rel.max():.1e}", flush=True)


if __name__ == "__main__":
    main()

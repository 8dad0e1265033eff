"""Converged solves of a config-4 sample under several restart-check / KKT-check periods (dev helper): PDHG
kernel time, iteration statistics and objective agreement with the first setting.

Usage: python scripts/sweep_checks.py <scenarios> <check:kkt> [<check:kkt> ...]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "der-vet_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402


def main():
    S = int(sys.argv[1])
    pb = builder.pack_groups(scenarios.config4(range(S)))
    dev = pb.to_torch("cuda:0").alloc_outputs()
    s = BatchSolver(0)
    base = None
    for spec in sys.argv[2:]:
        ce, ke = (int(v) for v in spec.split(":"))
        s.set_options(check_every=ce, kkt_every=ke)
        best = None
        for _ in range(2):
            s.solve_packed(dev)
            torch.cuda.synchronize()
            t = s.timing()["pdhg_ms"]
            best = t if best is None else min(best, t)
        ist = dev.istats.cpu().numpy()
        obj = dev.stats.cpu().numpy()[:, 0].copy()
        if base is None:
            base = obj
        rel = np.abs(obj - base) / np.maximum(np.abs(base), 1e-12)
        it = ist[:, 1]
        print(f"check {ce:3d} kkt {ke:2d}: pdhg {best:7.1f} ms  {pb.count / best * 1e3:8.0f} windows/s  iters mean "
              f"{it.mean():7.1f} p99 {np.percentile(it, 99):6.0f} max {it.max():6d}  optimal {(ist[:, 0] == 0).sum()}/"
              f"{pb.count}  max rel obj diff vs first {rel.max():.1e}", flush=True)


if __name__ == "__main__":
    main()

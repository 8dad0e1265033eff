"""A/B of the kernel cascade paths on a config-4 sample (dev helper): fixed-iteration cost per window-iteration
per CU, and converged solves (time, iterations, objective agreement between paths).

Usage: python scripts/ab_paths.py <scenarios> [fixed_iters]
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "der-vet_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    fixed = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    pb = builder.pack_groups(scenarios.config4(range(S)))
    dev = pb.to_torch("cuda:0").alloc_outputs()
    s = BatchSolver(0)
    units = pb.count / 256.0
    objs = {}
    for path in ("default", "ell"):
        s.set_kernel_path(path)
        for label, kw in (("plain", dict(check_every=1000000, kkt_every=1)), ("checks", dict(check_every=32, kkt_every=4))):
            s.set_options(eps=1e-30, max_iters=fixed, **kw)
            best = min((s.solve_packed(dev), torch.cuda.synchronize(), s.timing()["pdhg_ms"])[2] for _ in range(3))
            print(f"{path:8s} fixed {fixed} {label:6s}: {best * 1e3 / units / fixed:.3f} us/iter/CU  {s.kernel_stats()}",
                  flush=True)
        s.set_options(eps=1e-6, max_iters=100000, check_every=32, kkt_every=4)
        best = None
        for _ in range(2):
            s.solve_packed(dev)
            torch.cuda.synchronize()
            t = s.timing()["pdhg_ms"]
            best = t if best is None else min(best, t)
        ist = dev.istats.cpu().numpy()
        objs[path] = dev.stats.cpu().numpy()[:, 0].copy()
        it = ist[:, 1]
        print(f"{path:8s} converged: pdhg {best:.1f} ms  {pb.count / best * 1e3:.0f} windows/s  iters mean {it.mean():.1f} "
              f"max {it.max()}  optimal {(ist[:, 0] == 0).sum()}/{pb.count}  {best * 1e3 / (it.sum() / 256.0):.3f} "
              f"us/iter/CU", flush=True)
    rel = np.abs(objs["default"] - objs["ell"]) / np.maximum(np.abs(objs["ell"]), 1e-12)
    print(f"max rel objective difference band vs ell: {rel.max():.2e}")


if __name__ == "__main__":
    main()

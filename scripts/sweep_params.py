"""Converged solves of a config-4 sample under several solver option sets (dev helper for tuning the restart /
step / scaling parameters on the GPU): PDHG time, iteration statistics and objective agreement with the first
option set.

Usage: python scripts/sweep_params.py <scenarios> '<json dict>' ['<json dict>' ...]
"""
import json
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
    base = None
    for spec in sys.argv[2:]:
        kw = json.loads(spec)
        s = BatchSolver(0)
        s.set_options(**kw)
        s.solve_packed(dev)
        torch.cuda.synchronize()
        tm = s.timing()
        ist = dev.istats.cpu().numpy()
        st = dev.stats.cpu().numpy()
        obj = st[:, 0].copy()
        if base is None:
            base = obj
        rel = np.abs(obj - base) / np.maximum(np.abs(base), 1e-12)
        it = ist[:, 1]
        print(f"{spec:70s} pdhg {tm['pdhg_ms']:7.1f} ms setup {tm['setup_ms']:5.1f}  iters mean {it.mean():7.1f} p99 "
              f"{np.percentile(it, 99):6.0f} max {it.max():6d}  opt {(ist[:, 0] == 0).sum()}/{pb.count}  "
              f"pres max {np.nanmax(st[:, 1]):.1e}  obj diff vs first {rel.max():.1e}", flush=True)
        s.close()


if __name__ == "__main__":
    main()

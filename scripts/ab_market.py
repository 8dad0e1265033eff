"""A/B of kernels on daily market-service windows (dev helper): the three Usecase 3 golden cases (365 days each,
DA + frequency regulation, LP relaxation of binary = 1), replicated R times.  Kernel variant from the
environment (DVH_SMALL=-1 off, 0..2 a small-window variant; see dvh_kernels.hip small_dispatch).

Usage: DVH_SMALL=<v> python scripts/ab_market.py [R] [path]
"""
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "der-vet_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402
from oracle import cases  # noqa: E402


def groups(R):
    arr, meta = cases.load_market()
    out = []
    for name in ("es", "es+pv", "es+pv+dg"):
        sig = {k.split("__", 1)[1]: v for k, v in arr.items() if k.startswith(name + "__")}
        out += [scenarios.market_days(sig, meta[name]["params"])] * R
    return out


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    path = sys.argv[2] if len(sys.argv) > 2 else "default"
    t0 = time.time()
    pb = builder.pack_groups(groups(R))
    dev = pb.to_torch("cuda:0").alloc_outputs()
    s = BatchSolver(0)
    s.set_kernel_path(path)
    best = None
    for _ in range(3):
        s.solve_packed(dev)
        torch.cuda.synchronize()
        t = s.timing()
        best = t if best is None or t["total_ms"] < best["total_ms"] else best
    ist = dev.istats.cpu().numpy()
    obj = dev.stats.cpu().numpy()[:, 0]
    it = ist[:, 1]
    print(f"DVH_SMALL={os.environ.get('DVH_SMALL', '')} path={path} windows={pb.count} total {best['total_ms']:.2f} ms "
          f"(setup {best['setup_ms']:.2f}, pdhg {best['pdhg_ms']:.2f}) -> {pb.count / best['total_ms'] * 1e3:.0f} windows/s; "
          f"iters mean {it.mean():.0f} max {it.max()}; optimal {(ist[:, 0] == 0).sum()}/{pb.count}; "
          f"{s.kernel_stats()}; obj checksum {np.sum(obj[:1095]):.6f} (build {time.time() - t0:.1f}s)", flush=True)


if __name__ == "__main__":
    main()

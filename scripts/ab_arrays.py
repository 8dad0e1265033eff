#!/usr/bin/env python3
"""Dev A/B: solve one config-4 batch (cold, library defaults + kkt_predict) with the library DVH_LIB points at and save
x / y / stats / istats to gpurun_out/ab_<name>.npz; `compare a b` prints per-array equality and the largest
differences.  Usage (GPU box): [DVH_LIB=...] python scripts/ab_arrays.py run NAME [scenarios] | compare A B"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "der-vet_amd")]
import numpy as np  # noqa: E402

if sys.argv[1] == "run":
    import torch  # noqa: F401
    from dervet_hip import BatchSolver
    from dervet_hip.lp import builder, scenarios
    name, S = sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 500
    mode = sys.argv[4] if len(sys.argv) > 4 else "cold"
    pb = builder.pack_groups(scenarios.config4(range(S)))
    dev = pb.to_torch("cuda:0").alloc_outputs()
    opts = dict(kkt_predict=4) if mode == "cold" else dict(check_every=64, kkt_every=1, kkt_predict=4)
    if os.environ.get("AB_MAX_ITERS"):
        opts["max_iters"] = int(os.environ["AB_MAX_ITERS"])
    with BatchSolver(0, **opts) as s:
        s.solve_packed(dev)
        if mode == "warm":  # a second solve warm from the first's solution with the per-window x scaled by 0.9
            dev.x.mul_(0.9)
            s.set_options(warm_start=1, max_iters=int(os.environ.get("AB_WARM_ITERS", "100000")))
            s.solve_packed(dev)
    np.savez(os.path.join(ROOT, "gpurun_out", f"ab_{name}.npz"), x=dev.x.cpu().numpy(), y=dev.y.cpu().numpy(),
             stats=dev.stats.cpu().numpy(), istats=dev.istats.cpu().numpy())
else:
    a = np.load(os.path.join(ROOT, "gpurun_out", f"ab_{sys.argv[2]}.npz"))
    b = np.load(os.path.join(ROOT, "gpurun_out", f"ab_{sys.argv[3]}.npz"))
    for k in ("x", "y", "stats", "istats"):
        eq = np.array_equal(a[k], b[k])
        d = np.abs(a[k].astype(np.float64) - b[k].astype(np.float64))
        print(k, "equal" if eq else f"DIFFER: {int((d > 0).sum())} entries, max abs {d.max():.3e}, "
              f"first rows {np.unique(np.nonzero(d)[0])[:8]}")

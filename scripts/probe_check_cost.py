#!/usr/bin/env python3
"""Dev probe: the cost of the band kernel's checks, from the per-iteration time at a fixed iteration count (eps 1e-14:
no window converges) under different check schedules (check_every C, kkt_every K; DVH_LIB picks a build).
Usage (GPU box): python scripts/probe_check_cost.py [scenarios] [iters]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "der-vet_amd")]
import torch  # noqa: E402
from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
N = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
pb = builder.pack_groups(scenarios.config4(range(S)))
dev = pb.to_torch("cuda:0").alloc_outputs()
for C, K, P in [(1024, 1, 0), (256, 1000, 0), (128, 1000, 0), (64, 1000, 0), (32, 1000, 0), (64, 1, 0), (32, 4, 0),
                (32, 1, 0), (64, 1, 4), (32, 4, 4)]:
    s = BatchSolver(0, eps=1e-14, eps_obj=0.0, max_iters=N, check_every=C, kkt_every=K, kkt_predict=P)
    best = None
    for r in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        s.solve_packed(dev)
        torch.cuda.synchronize()
        el = time.perf_counter() - t
        if r > 0:
            best = el if best is None else min(best, el)
    it = float(dev.istats[:, 1].double().mean())
    print(f"check_every {C:5d} kkt_every {K:5d} kkt_predict {P}: {best * 1e3:7.2f} ms = "
          f"{best / (pb.count * it) * 512 * 1e6:.4f} us per window-iteration per slot (iters {it:.0f})", flush=True)
    s.close()

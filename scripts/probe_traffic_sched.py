#!/usr/bin/env python3
"""Dev probe for rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE: the bench's band kernel at a fixed iteration count (eps 1e-14,
no window converges) under one check schedule, so the HBM bytes of the iteration, the restart checks and the KKT checks
can be told apart by difference.  One solve after a warm-up (both dispatches are counted; average them).
Usage: rocprofv3 --pmc FETCH_SIZE -- python3 scripts/probe_traffic_sched.py <check_every> <kkt_every> [scenarios] [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "der-vet_amd")]
import torch  # noqa: E402
from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402

C, K = int(sys.argv[1]), int(sys.argv[2])
S = int(sys.argv[3]) if len(sys.argv) > 3 else 5000
N = int(sys.argv[4]) if len(sys.argv) > 4 else 1024
pb = builder.pack_groups(scenarios.config4(range(S)))
dev = pb.to_torch("cuda:0").alloc_outputs()
s = BatchSolver(0, eps=1e-14, eps_obj=0.0, max_iters=N, check_every=C, kkt_every=K, kkt_predict=0)
for r in range(2):
    s.solve_packed(dev)
torch.cuda.synchronize()
print(f"windows {pb.count} iters {float(dev.istats[:, 1].double().mean()):.0f} check_every {C} kkt_every {K}", flush=True)
s.close()

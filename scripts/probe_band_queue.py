#!/usr/bin/env python3
"""Dev probe: per-iteration speed of the band kernel's one-workgroup-per-window and persistent forms with every window
running the same fixed number of iterations (eps 1e-14, max_iters N: no dispatch-order or tail effects).
Usage (GPU box): DVH_BAND_QUEUE=0|1 python scripts/probe_band_queue.py [scenarios] [iters] [config4 | config5]
(the per-slot figure assumes 512 slots: the ICE form has 256, one per CU)"""
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
CFG = sys.argv[3] if len(sys.argv) > 3 else "config4"
pb = builder.pack_groups(scenarios.config4(range(S)) if CFG == "config4" else scenarios.config5(range(S), years=1))
dev = pb.to_torch("cuda:0").alloc_outputs()
s = BatchSolver(0, eps=1e-14, eps_obj=0.0, max_iters=N)
best = None
for r in range(3):
    torch.cuda.synchronize()
    t = time.perf_counter()
    s.solve_packed(dev)
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    if r > 0:
        best = el if best is None else min(best, el)
it = dev.istats[:, 1].double()
print(f"{CFG} queue={os.environ.get('DVH_BAND_QUEUE', '1')} windows {pb.count} iters mean {float(it.mean()):.0f} "
      f"min {int(it.min())}: {best * 1e3:.1f} ms = {best / (pb.count * float(it.mean())) * 512 * 1e6:.3f} us per "
      f"window-iteration per slot ({s.timing()})", flush=True)

#!/usr/bin/env python3
"""Cold solves of BASELINE config 5's windows (battery + PV + LP-relaxed ICE + DCM, 744-step monthly windows) on the
band kernel's ICE form, for rocprofv3 kernel-trace / PMC passes (scripts/profile_kernels.sh): one warm-up solve, then
one measured solve of the same batch.  Usage: prof_config5.py [scenarios]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "der-vet_amd")]
import torch  # noqa: E402
from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 100
pb = builder.pack_groups(scenarios.config5(range(S), years=1))
dev = pb.to_torch("cuda:0").alloc_outputs()
s = BatchSolver(0)
for _ in range(2):
    s.solve_packed(dev)
    torch.cuda.synchronize()
it = dev.istats[:, 1].double()
print(json.dumps({"config": "config5", "windows": pb.count, "timing": s.timing(), "paths": s.kernel_stats(),
                  "iters_mean": float(it.mean()), "iters_max": int(it.max()),
                  "optimal": int((dev.istats[:, 0] == 0).sum())}), flush=True)
del dev
s.close()

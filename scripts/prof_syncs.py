#!/usr/bin/env python3
"""Host waits of the cascade under a HIP API trace (scripts/prof_r03.sh): one band-only batch (1,200 config-4
windows) through dvh_solve_packed_device, three times; the library's own count (dvh_last_host_syncs) is printed to
compare with the trace's hipStreamSynchronize calls."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "der-vet_amd")]
import torch
from dervet_hip import BatchSolver
from dervet_hip.lp import builder, scenarios
pb = builder.pack_groups(scenarios.config4(range(100)))
dev = pb.to_torch("cuda:0").alloc_outputs()
s = BatchSolver(0)
torch.cuda.synchronize()
counts = []
for _ in range(3):
    s.solve_packed(dev)
    counts.append(s.host_syncs())
torch.cuda.synchronize()
print(json.dumps({"windows": pb.count, "host_syncs_per_solve": counts, "paths": s.kernel_stats()}), flush=True)
del dev
s.close()

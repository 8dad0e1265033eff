#!/usr/bin/env python3
"""One cold solve of BASELINE config 3's DCM + PV variant (the 5-minute annual window, 12 monthly demand columns) on
the long team, after a warm-up solve; for rocprofv3 kernel-trace / PMC passes (scripts/prof_r03.sh)."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "der-vet_amd")]
import torch
from dervet_hip import BatchSolver
from dervet_hip.lp import builder, scenarios
import numpy as np
variant = sys.argv[1] if len(sys.argv) > 1 else "dcm"
if variant == "dcm_nopv":  # bench_configs.py's "config3+dcm" row: site load + DA + retail + 12 monthly DCM, no PV
    ri = scenarios.reference_inputs()
    groups = scenarios.windows_by_period(2019, 1.0 / 12, ri["fivemin_site_load"][None, :], None,
                                         scenarios.template_battery(), da_price=ri["fivemin_da_price"][None, :],
                                         tariff_def=scenarios.tariff(), n="year")
else:
    groups = scenarios.config3(variant)
pb = builder.pack_groups(groups)
dev = pb.to_torch("cuda:0").alloc_outputs()
s = BatchSolver(0)
s.solve_packed(dev)
torch.cuda.synchronize()
s.solve_packed(dev)
torch.cuda.synchronize()
print(json.dumps({"variant": variant, "timing": s.timing(), "paths": s.kernel_stats(),
                  "iters": int(dev.istats[0, 1]), "status": int(dev.istats[0, 0]), "n": int(pb.desc[0, 0]),
                  "m": int(pb.desc[0, 1]), "nnz": int(pb.desc[0, 3])}), flush=True)
del dev
s.close()
torch.cuda.synchronize()
maps = os.environ.get("DVH_DUMP_MAPS")
if maps:  # the process's mappings, to resolve the PCs of a teardown crash under the profiler
    with open("/proc/self/maps") as f, open(maps, "w") as g:
        g.write(f.read())

"""A/B of warm-phase options of bench.py's seeded sweep (device-built config-4 batch): per setting, the warm
windows' mean iterations, the schedule's PDHG time (best of 2) and the objective spread against the first
setting.  Usage: python scripts/ab_warm.py [scenarios] (settings below).

Round-2 result (profiles/r02t_ab_warm_weight.log): carrying each seed's final primal weight over to its warm
partners (an experimental dvh_packed.weight field, full or square-root ratio) gave 2,075-2,093 warm iterations
against 2,073 without it, so the field was not kept; primal_weight_theta = 0.5 in the warm phase: 2,016 iterations
but a longer tail (iters_max 16,640), PDHG time within the box-to-box noise."""
import functools
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "der-vet_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import scenarios  # noqa: E402
from dervet_hip.sweep import SeededSweep, WARM_OPTIONS  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
SETTINGS = [dict(WARM_OPTIONS), dict(WARM_OPTIONS, primal_weight_theta=0.5)]
ids = range(S)
P = scenarios.sweep_parameters(ids)
s = BatchSolver(0)
sw = SeededSweep(functools.partial(scenarios.config4, spec=True), ids, P["E"], stride=32,
                 features=scenarios.sweep_features(P))
dev = sw.to_device(s, "cuda:0")
ref = None
for opt in SETTINGS:
    best = None
    for _ in range(2):
        tm, _ = sw.solve(s, dev, warm_options=opt)
        torch.cuda.synchronize()
        if best is None or tm["pdhg_ms"] < best["pdhg_ms"]:
            best = tm
    ist = dev.istats.cpu().numpy()
    obj = dev.stats.cpu().numpy()[:, 0].copy()
    if ref is None:
        ref = obj
    ns = sw.n_seed
    print(json.dumps({"warm_options": opt, "pdhg_ms": round(best["pdhg_ms"], 1),
                      "iters_seed": round(float(ist[:ns, 1].mean()), 1),
                      "iters_warm": round(float(ist[ns:, 1].mean()), 1), "iters_max": int(ist[:, 1].max()),
                      "optimal": int((ist[:, 0] == 0).sum()),
                      "max_obj_rel_diff_vs_first": float(np.max(np.abs(obj - ref) / np.maximum(np.abs(ref), 1.0)))}), flush=True)

#!/usr/bin/env python3
"""Dev probe: the degenerate T = 2 windows of tests/test_gpu_configs.py::test_band_kernel_forms_agree on each band form
(status, iterations, objective per window).  Usage (GPU box): [DVH_LIB=...] python scripts/probe_t2.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "der-vet_amd")]
import numpy as np  # noqa: E402
from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import builder  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 2
rng = np.random.default_rng(T)
G = 3
load = 400 + 200 * rng.random((G, T))
masks = np.zeros((2, T), bool)
masks[0, : (T + 1) // 2] = True
masks[1, (T + 1) // 2:] = True
bat = dict(E=rng.uniform(500, 2000, G), Pch=rng.uniform(100, 400, G), Pdis=rng.uniform(100, 400, G),
           rte=rng.uniform(0.8, 0.95, G), sdr=rng.uniform(0, 1, G), soc_target=rng.uniform(0.3, 0.9, G),
           ulsoc=0.95, llsoc=0.05, fixedOM=10.0, OMexpenses=rng.uniform(0, 5, G))
groups = [builder.battery_group(T, 1.0, load, bat, retail_price=rng.uniform(0.03, 0.2, (G, T)),
                                demand_masks=masks[:1], demand_prices=rng.uniform(5, 20, (G, 1))),
          builder.battery_group(T, 1.0, load, bat, retail_price=rng.uniform(0.03, 0.2, (G, T)),
                                demand_masks=masks, demand_prices=rng.uniform(5, 20, (G, 2)))]
lps = [lp for g in groups for lp in builder.group_window_lps(g)]
with BatchSolver(0, max_iters=20000) as s:
    for path in ("band3", "band1"):
        s.set_kernel_path(path)
        res = s.solve(lps)
        print(os.environ.get("DVH_LIB", "cur"), path, os.environ.get("DVH_BAND_QUEUE", "1"),
              [(r.status, r.iters, round(r.obj, 6)) for r in res], flush=True)

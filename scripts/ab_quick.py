#!/usr/bin/env python3
"""Dev A/B harness (DVH_LIB picks a build): per-iteration speed of the band forms at a fixed iteration count
(config 4 battery, config 5 ICE), the 1,095 Usecase-3 market days (market options and defaults, median of 5) and the
config-3 DCM + PV window (long team).  Usage (GPU box): DVH_LIB=... python scripts/ab_quick.py [tag]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "der-vet_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402
from oracle import cases  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else os.environ.get("DVH_LIB", "default")
out = {"tag": tag}


def timed(s, dev, reps=3):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        s.solve_packed(dev)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    return float(np.median(ts))


for name, groups, slots in (("config4", scenarios.config4(range(5000)), 512),
                            ("config5", scenarios.config5(range(1000), years=1), 256)):
    dev = builder.pack_groups(groups).to_torch("cuda:0").alloc_outputs()
    with BatchSolver(0, eps=1e-14, eps_obj=0.0, max_iters=1024) as s:
        s.solve_packed(dev)
        el = timed(s, dev)
    out[name + "_us_per_window_iter_per_slot"] = round(el / (dev.count * 1024) * slots * 1e6, 4)
arr, meta = cases.load_market()
sig = lambda nm: {k.split("__", 1)[1]: v for k, v in arr.items() if k.startswith(nm + "__")}
days = builder.pack_groups([scenarios.market_days(sig(nm), meta[nm]["params"], name=nm)
                            for nm in ("es", "es+pv", "es+pv+dg")]).to_torch("cuda:0").alloc_outputs()
for label, opts in (("market_options_ms", scenarios.MARKET_OPTIONS), ("market_default_ms", {})):
    with BatchSolver(0, **opts) as s:
        s.solve_packed(days)
        out[label] = round(1e3 * timed(s, days, 5), 2)
        out[label.replace("_ms", "_iters_max")] = int(days.istats[:, 1].max())
lps = builder.group_window_lps(scenarios.config3("dcm")[0])
with BatchSolver(0) as s:
    s.solve(lps)
    t = time.perf_counter()
    r = s.solve(lps)[0]
    out["config3_dcm_pv_ms"] = round(1e3 * (time.perf_counter() - t), 1)
    out["config3_iters"] = int(r.iters)
print(json.dumps(out), flush=True)

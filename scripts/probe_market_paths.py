#!/usr/bin/env python3
"""Market days (Usecase 3 es) on the ELL vs the generic kernel at several batch sizes: wall per solve (median of 5)."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "der-vet_amd")]
import numpy as np, torch
from dervet_hip import BatchSolver
from dervet_hip.lp import builder, scenarios
from oracle import cases
arr, meta = cases.load_market()
sig = {k.split("__", 1)[1]: v for k, v in arr.items() if k.startswith("es__")}
s = BatchSolver(0)
def sig_of(name):
    return {k.split("__", 1)[1]: v for k, v in arr.items() if k.startswith(name + "__")}
all3 = [scenarios.market_days(sig_of(nm), meta[nm]["params"], name=nm) for nm in ("es", "es+pv", "es+pv+dg")]
for step in (30, 9, 3, 1, "x3", "x12"):
    if isinstance(step, int):
        gs = [scenarios.market_days(sig, meta["es"]["params"], days=list(range(0, 365, step)))]
    else:
        gs = all3 * (int(step[1:]) // 3)
    dev = builder.pack_groups(gs).to_torch("cuda:0").alloc_outputs()
    out = {"days": sum(g.G for g in gs)}
    for path in ("default", "generic"):
        s.set_kernel_path(path)
        s.solve_packed(dev)
        ts = []
        for _ in range(5):
            torch.cuda.synchronize(); t = time.perf_counter(); s.solve_packed(dev); torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
        out[path] = {"ms": round(1e3 * float(np.median(ts)), 2), "pdhg_ms": round(s.timing()["pdhg_ms"], 2),
                     "iters": float(dev.istats[:, 1].float().mean()), "paths": {k: v for k, v in s.kernel_stats().items() if k.endswith("windows") and v}}
    print(json.dumps(out), flush=True)

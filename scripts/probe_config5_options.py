#!/usr/bin/env python3
"""Config-5 windows (ICE band form; 1,000 scenarios x one opt year, scripts/certify_config5.py's batch) under seeded
schedules with different warm / seed option sets: best-of-3 wall, iterations, optimal count.

Usage: python scripts/probe_config5_options.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "der-vet_amd"), os.path.join(ROOT, "scripts")]
import torch  # noqa: E402
from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.sweep import SEED_OPTIONS, WARM_OPTIONS  # noqa: E402
from certify_config5 import _sweep  # noqa: E402

sw = _sweep(1000)
dev = sw.packed.to_torch("cuda:0").alloc_outputs()
s = BatchSolver(0)
W, S = dict(WARM_OPTIONS), dict(SEED_OPTIONS)
variants = [("default", W, S),
            ("warm check 32", {**W, "check_every": 32}, S),
            ("warm check 128", {**W, "check_every": 128}, S),
            ("warm kkt_every 2", {**W, "kkt_every": 2}, S),
            ("warm predict 0", {**W, "kkt_predict": 0}, S),
            ("warm predict 8", {**W, "kkt_predict": 8}, S),
            ("seed check 64", W, {**S, "check_every": 64}),
            ("seed kkt_every 1", W, {**S, "kkt_every": 1}),
            ("default", W, S)]
for name, w, sd in variants:
    best = None
    for rep in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        sw.solve(s, dev, warm_options=w, seed_options=sd)
        torch.cuda.synchronize()
        el = time.perf_counter() - t
        best = el if best is None else min(best, el)
    ist = dev.istats.cpu().numpy()
    print(json.dumps({"variant": name, "ms": round(1e3 * best, 2), "windows_per_s": round(dev.count / best, 1),
                      "iters_mean": float(ist[:, 1].mean()), "iters_max": int(ist[:, 1].max()),
                      "optimal": int((ist[:, 0] == 0).sum())}), flush=True)

#!/usr/bin/env python3
"""Config 3 as stated (DCM + PV, T = 105,120) started from stitched sub-window solutions: daily sub-windows (365, the
bench_configs row) vs the 12 monthly windows (each with its own month's demand charge), with and without the monthly
DCM duals carried over (dervet_hip/stitch.py), and with the sub-windows solved to a looser tolerance first.  Prints the
sub-window batch time, the long window's iterations and time.

Usage: python scripts/probe_config3_stitch.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "der-vet_amd")]
import torch  # noqa: E402
from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402
from dervet_hip.stitch import stitched_start  # noqa: E402

long = scenarios.config3("dcm")[0]
long_lp = builder.group_window_lps(long)[0]
s = BatchSolver(0)
o0 = s.options()
base = {"eps": o0.eps, "eps_obj": o0.eps_obj}
monthly = scenarios.config3("dcm", n="month")
daily = scenarios.config3("dcm", n=288)
runs = [("cold", None, False, None), ("daily", daily, False, None), ("monthly", monthly, False, None),
        ("monthly+dcm_duals", monthly, True, None)]
runs += [(f"monthly+dcm_duals eps_sub={e:g}", monthly, True, e) for e in (1e-2, 1e-3, 1e-4, 1e-5)]
for name, subs, duals, eps_sub in runs:
    for rep in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        sub_ms, sres = 0.0, []
        if subs is not None:
            if eps_sub:
                s.set_options(eps=eps_sub, eps_obj=eps_sub)
            sres = s.solve([builder.group_window_lps(g)[0] for g in subs])
            sub_ms = s.timing()["total_ms"]
            s.set_options(**base)
            x0, y0 = stitched_start(long, subs, [r.x for r in sres], [r.y for r in sres], duals)
            s.set_options(warm_start=1)
            res = s.solve([long_lp], start=[(x0, y0)])[0]
            s.set_options(warm_start=0)
        else:
            res = s.solve([long_lp])[0]
        long_ms = s.timing()["total_ms"]
        wall = time.perf_counter() - t
    print(json.dumps({"start": name, "subs": len(subs) if subs else 0,
                      "subs_iters_max": int(max(r.iters for r in sres)) if sres else 0,
                      "subs_ms": round(sub_ms, 2), "long_ms": round(long_ms, 2), "long_iters": res.iters,
                      "gpu_ms": round(sub_ms + long_ms, 2), "status": res.status_name, "obj": res.obj,
                      "wall_ms": round(1e3 * wall, 1)}), flush=True)

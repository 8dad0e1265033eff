"""Config 3 (one 5-minute annual window, T = 105,120) started from stitched sub-window solutions (dervet_hip/stitch.py):
sub-window length vs sub-window solve time, the long window's iterations and solve time, whole-call wall time.
Monthly 5-minute windows (T ~ 8,928) run on the medium tier.  Usage: python scripts/probe_stitch.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "der-vet_amd"))
import numpy as np  # noqa: E402

from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import scenarios  # noqa: E402
from dervet_hip.stitch import solve_stitched  # noqa: E402


def main():
    ri = scenarios.reference_inputs()
    T = len(ri["fivemin_da_price"])
    s = BatchSolver(0)
    variants = {
        "config3": dict(load=np.zeros((1, T)), extra={}),
        "config3+dcm": dict(load=ri["fivemin_site_load"][None, :], extra=dict(tariff_def=scenarios.tariff())),
    }
    for name, v in variants.items():
        mk = lambda n: scenarios.windows_by_period(2019, 1.0 / 12, v["load"], None, scenarios.template_battery(),  # noqa
                                                   da_price=ri["fivemin_da_price"][None, :], n=n, **v["extra"])
        long = mk("year")[0]
        for sub in (288, 2016, "month"):
            subs = mk(sub)
            best = None
            for rep in range(2):
                t = time.perf_counter()
                res, sres, tm = solve_stitched(s, long, subs)
                el = time.perf_counter() - t
                if best is None or el < best[0]:
                    best = (el, res, tm, sres)
            el, res, tm, sres = best
            print(json.dumps({"config": name, "sub": sub, "subs": len(subs), "wall_ms": round(el * 1e3, 1),
                              "subs_ms": round(tm["subs_ms"], 1), "long_ms": round(tm["long_ms"], 1),
                              "long_iters": int(res.iters), "long_status": res.status_name,
                              "subs_iters_max": int(max(r.iters for r in sres)), "obj": res.obj,
                              "paths": s.kernel_stats()}), flush=True)


if __name__ == "__main__":
    main()

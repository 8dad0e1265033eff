"""Market-day windows (bench_configs.py --only 6 workloads) with and without the objective-error termination test
(dvh_options.eps_obj): wall time of a resident-batch solve, iterations (mean / p99 / max), statuses.
Usage: python scripts/probe_market_gate.py"""
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "der-vet_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402


def workloads():
    gold = os.path.join(ROOT, "tests", "golden")
    arr = dict(np.load(os.path.join(gold, "uc3_market.npz")))
    with open(os.path.join(gold, "uc3_market.json")) as f:
        meta = json.load(f)
    names = ("es", "es+pv", "es+pv+dg")
    sigs = {nm: {k.split("__", 1)[1]: v for k, v in arr.items() if k.startswith(nm + "__")} for nm in names}
    yield "market-uc3", [scenarios.market_days(sigs[nm], meta[nm]["params"]) for nm in names]
    groups = []
    for nm in names:
        sg, pdis = sigs[nm], float(meta[nm]["params"]["Battery"]["dis_max_rated"])
        N = len(sg["da_price"])
        h = np.arange(N)
        res = [dict(key="SR", price=0.6 * sg["regu_price"], duration=0.5, max=np.full(N, 0.5 * pdis),
                    min=np.zeros(N)), dict(key="NSR", price=0.3 * sg["regu_price"], duration=1.0)]
        lf = dict(eou=0.2 + 0.05 * np.sin(h / 7.0), eod=0.2 + 0.05 * np.cos(h / 5.0),
                  up_price=0.8 * sg["regu_price"], down_price=0.8 * sg["regd_price"], energy_price=sg["da_price"],
                  up_max=np.full(N, 0.25 * pdis), up_min=np.zeros(N), down_max=np.full(N, 0.25 * pdis),
                  down_min=np.zeros(N), combined=False)
        groups.append(scenarios.market_days(sg, meta[nm]["params"], reserves=res, lf=lf))
    yield "market-uc3+lf+sr+nsr", groups


def main():
    s = BatchSolver(0)
    for name, groups in workloads():
        dev = builder.pack_groups(groups).to_torch("cuda:0").alloc_outputs()
        for opts in ({"eps_obj": 1e-6}, {"eps_obj": 0.0}, {"kkt_predict": 4}):
            s.set_options(**opts)
            best = None
            for _ in range(3):
                torch.cuda.synchronize()
                t = time.perf_counter()
                s.solve_packed(dev)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t
                best = dt if best is None else min(best, dt)
            ist = dev.istats.cpu().numpy()
            it = ist[:, 1]
            print(json.dumps({"workload": name, "options": opts, "wall_ms": round(best * 1e3, 2),
                              "iters_mean": float(it.mean()), "iters_p99": float(np.percentile(it, 99)),
                              "iters_max": int(it.max()), "optimal": int((ist[:, 0] == 0).sum()),
                              "windows": int(len(ist)), "paths": s.kernel_stats()}), flush=True)
            s.set_options(eps_obj=1e-6, kkt_predict=0)


if __name__ == "__main__":
    main()

"""Seed stride / seed choice of the seeded schedule on the bench workload (GPU; dev helper): 10,000 config-4
scenarios (device series + builder) packed for several strides (and farthest-point seeds), each solved twice;
PDHG time, seed / warm iterations.  Usage: python scripts/probe_seed_stride.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "der-vet_amd"))

import torch  # noqa: E402

from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import gpu_series, scenarios  # noqa: E402
from dervet_hip.sweep import SeededSweep  # noqa: E402


def main():
    scen = range(10000)
    solver = BatchSolver(0)
    series = gpu_series.DeviceSeries(scen, solver, "cuda:0")
    P = series.parameters()
    for stride, cover in ((32, False), (24, False), (48, False), (16, False), (32, True), (64, False)):
        sweep = SeededSweep(series.config4, scen, P["E"], stride=stride, features=scenarios.sweep_features(P),
                            cover=cover)
        dev = sweep.to_device(solver, "cuda:0")
        sweep.solve(solver, dev)
        best = None
        for _ in range(2):
            torch.cuda.synchronize()
            t = time.perf_counter()
            tm, _ = sweep.solve(solver, dev)
            torch.cuda.synchronize()
            el = time.perf_counter() - t
            best = el if best is None else min(best, el)
        ist = dev.istats.cpu().numpy()
        ns = sweep.n_seed
        print(json.dumps(dict(stride=stride, cover=cover, seeds=int(ns), wall_ms=round(1e3 * best, 2),
                              pdhg_ms=round(tm["pdhg_ms"], 2), iters_seed=round(float(ist[:ns, 1].mean()), 1),
                              iters_warm=round(float(ist[ns:, 1].mean()), 1), optimal=float((ist[:, 0] == 0).mean()))),
              flush=True)
        del dev
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

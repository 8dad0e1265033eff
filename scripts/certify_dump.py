#!/usr/bin/env python3
"""GPU half of the full-population objective certification.

Builds exactly the bench workload (config 4, 10,000 scenarios x 12 monthly windows, seeded schedule as
bench.py runs it), solves it once seeded and once all-cold, and writes every window's
{obj, primal_res_rel, dual_res_rel, gap_rel, status, iters} plus the (scenario, month) tags to
gpurun_out/certify/<label>.npz.  scripts/certify_highs.py solves the same 120,000 LPs with HiGHS on the
host and compares.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "der-vet_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenarios", type=int, default=10000)
    ap.add_argument("--label", default="r02")
    ap.add_argument("--eps", type=float, default=0.0)
    ap.add_argument("--opt", action="append", default=[], help="dvh_options field=value (repeatable)")
    ap.add_argument("--no-cold", action="store_true")
    ap.add_argument("--lib", default=None, help="alternative libdervet_hip.so (A/B builds)")
    ap.add_argument("--blend", type=int, default=1, help="warm starts blended from this many nearest seeds")
    args = ap.parse_args()
    if args.lib:
        from dervet_hip import _lib
        _lib.LIB_PATH = os.path.abspath(args.lib)
    from dervet_hip import BatchSolver
    from dervet_hip.lp import scenarios
    from dervet_hip.sweep import SeededSweep

    scen = range(args.scenarios)
    t0 = time.time()
    P = scenarios.sweep_parameters(scen)
    sweep = SeededSweep(scenarios.config4, scen, P["E"], stride=32, features=scenarios.sweep_features(P),
                        blend=args.blend)
    dev = sweep.packed.to_torch("cuda:0").alloc_outputs()
    print(f"built {dev.count} windows in {time.time() - t0:.1f} s", flush=True)
    solver = BatchSolver(0)
    opts = {}
    if args.eps > 0:
        opts["eps"] = args.eps
    for kv in args.opt:
        k, v = kv.split("=")
        opts[k] = float(v) if "." in v or "e" in v else int(v)
    if opts:
        solver.set_options(**opts)
    out = {"tags": np.array(sweep.tags, np.int64), "n_seed": sweep.n_seed}
    for rep in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        tm, paths = sweep.solve(solver, dev)
        torch.cuda.synchronize()
        el = time.perf_counter() - t
    print(f"seeded: {el * 1e3:.1f} ms ({dev.count / el:.0f} windows/s) {tm} {paths}", flush=True)
    out["seeded_stats"] = dev.stats.cpu().numpy()
    out["seeded_istats"] = dev.istats.cpu().numpy()
    out["seeded_ms"] = el * 1e3
    if not args.no_cold:
        solver.set_options(warm_start=0)
        for rep in range(2):
            torch.cuda.synchronize()
            t = time.perf_counter()
            solver.solve_packed(dev)
            torch.cuda.synchronize()
            el = time.perf_counter() - t
        print(f"cold: {el * 1e3:.1f} ms ({dev.count / el:.0f} windows/s) {solver.timing()}", flush=True)
        out["cold_stats"] = dev.stats.cpu().numpy()
        out["cold_istats"] = dev.istats.cpu().numpy()
        out["cold_ms"] = el * 1e3
    os.makedirs(os.path.join(ROOT, "gpurun_out", "certify"), exist_ok=True)
    path = os.path.join(ROOT, "gpurun_out", "certify", f"{args.label}.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, flush=True)


if __name__ == "__main__":
    main()

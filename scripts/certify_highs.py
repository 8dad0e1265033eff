#!/usr/bin/env python3
"""Host half of the full-population objective certification.

Solves every window of the bench workload (config 4, 10,000 scenarios x 12 monthly windows, packed in the
seeded schedule's order exactly as bench.py / scripts/certify_dump.py pack it) with HiGHS (restated LP,
oracle/window_lp.py) on a process pool, and compares with the GPU objectives of certify_dump.py.

  python scripts/certify_highs.py solve  --out gpurun_out/certify/highs.npz [--procs 8]
  python scripts/certify_highs.py compare --highs gpurun_out/certify/highs.npz --gpu gpurun_out/certify/r02.npz
"""
import argparse
import json
import os
import sys
import time
from multiprocessing import get_context

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "der-vet_amd"))

import numpy as np  # noqa: E402

_PB = None


def _solve(k):
    from oracle import window_lp
    r = window_lp.solve_highs(window_lp.from_packed_window(_PB.window(int(k))))
    return r.get("obj", np.nan), r["status"]


def solve(args):
    global _PB
    from dervet_hip.lp import scenarios
    from dervet_hip.sweep import SeededSweep
    scen = range(args.scenarios)
    P = scenarios.sweep_parameters(scen)
    t = time.time()
    sweep = SeededSweep(scenarios.config4, scen, P["E"], stride=32, features=scenarios.sweep_features(P))
    _PB = sweep.packed
    print(f"built {_PB.count} windows in {time.time() - t:.1f} s", flush=True)
    idx = np.arange(_PB.count)
    if args.every > 1:
        idx = idx[::args.every]
    t = time.time()
    pool = get_context("fork").Pool(args.procs)
    objs = np.full(_PB.count, np.nan)
    sts = np.full(_PB.count, -1, np.int32)
    done = 0
    for i, (o, s) in zip(idx, pool.imap(_solve, idx, chunksize=64)):
        objs[i], sts[i] = o, s
        done += 1
        if done % 5000 == 0:
            print(f"{done}/{len(idx)} in {time.time() - t:.0f} s", flush=True)
    pool.close()
    pool.join()
    wall = time.time() - t
    np.savez_compressed(args.out, obj=objs, status=sts, tags=np.array(sweep.tags, np.int64), wall_s=wall,
                        procs=args.procs, solved=idx)
    print(f"HiGHS: {len(idx)} windows in {wall:.0f} s on {args.procs} processes -> {args.out}", flush=True)


def no_battery(scenarios_):
    """obj_no_battery per window of the bench packing (battery idle, tau at the largest DCM rhs; oracle/cba.py
    no_battery_objective, vectorised for the config-4 windows' single tau column)."""
    from dervet_hip.lp import scenarios
    from dervet_hip.sweep import SeededSweep
    scen = range(scenarios_)
    P = scenarios.sweep_parameters(scen)
    pb = SeededSweep(scenarios.config4, scen, P["E"], stride=32, features=scenarios.sweep_features(P)).packed
    d = pb.desc
    nb = np.empty(pb.count)
    for k in range(pb.count):
        n, m, me, _, _, _, on, om = (int(v) for v in d[k])
        assert n == 3 * (me - 1) + 1
        nb[k] = pb.c0[k] + pb.c[on + n - 1] * pb.q[om + me:om + m].max()
    return nb


def compare(args):
    h = np.load(args.highs)
    nb = no_battery(args.scenarios) if args.benefit else None
    out = {}
    for path in args.gpu:
        g = np.load(path)
        assert np.array_equal(g["tags"], h["tags"]), "window order differs"
        ok = h["status"] == 0
        for ph in ("seeded", "cold"):
            if f"{ph}_stats" not in g:
                continue
            st, ist = g[f"{ph}_stats"], g[f"{ph}_istats"]
            rel = np.abs(st[:, 0] - h["obj"]) / np.abs(h["obj"])
            r = rel[ok]
            worst = np.argsort(-np.where(ok, rel, -1))[:20]
            ben = {}
            if nb is not None:
                br = (np.abs(st[:, 0] - h["obj"]) / np.abs(nb - h["obj"]))[ok]
                ben = dict(max_benefit_rel=float(br.max()), p99_benefit_rel=float(np.quantile(br, 0.99)),
                           median_benefit_usd=float(np.median((nb - h["obj"])[ok])),
                           min_benefit_usd=float(np.min((nb - h["obj"])[ok])))
            out[f"{os.path.basename(path)}:{ph}"] = dict(**ben,
                windows=int(ok.sum()), gpu_optimal=int((ist[:, 0] == 0).sum()), max_rel=float(r.max()),
                p99_rel=float(np.quantile(r, 0.99)), p999_rel=float(np.quantile(r, 0.999)), mean_rel=float(r.mean()),
                n_gt_1e5=int((r > 1e-5).sum()), n_gt_5e6=int((r > 5e-6).sum()), n_gt_2e6=int((r > 2e-6).sum()),
                max_primal_res_rel=float(st[:, 1].max()), iters_mean=float(ist[:, 1].mean()),
                ms=float(g[f"{ph}_ms"]), worst=[(int(k), [int(v) for v in g["tags"][k]], float(rel[k]),
                                                 int(ist[k, 1])) for k in worst[:8]])
    print(json.dumps(out, indent=1))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    a = sub.add_parser("solve")
    a.add_argument("--scenarios", type=int, default=10000)
    a.add_argument("--procs", type=int, default=os.cpu_count() or 1)
    a.add_argument("--every", type=int, default=1)
    a.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "certify", "highs.npz"))
    b = sub.add_parser("compare")
    b.add_argument("--highs", default=os.path.join(ROOT, "gpurun_out", "certify", "highs.npz"))
    b.add_argument("--gpu", nargs="+", required=True)
    b.add_argument("--json", default=None)
    b.add_argument("--benefit", action="store_true", help="also the battery-benefit error (obj_no_battery - obj)")
    b.add_argument("--scenarios", type=int, default=10000)
    args = ap.parse_args()
    solve(args) if args.cmd == "solve" else compare(args)


if __name__ == "__main__":
    main()

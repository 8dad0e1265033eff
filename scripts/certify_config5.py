#!/usr/bin/env python3
"""Certification of the ICE band form's windows (the ICE form's objective gate leaves out the
sum_j |r_d,j| |x_j| term that the battery forms and the CPU restatements apply -- is the exemption harmless?).

  dump    (GPU) config-5 windows of --scenarios scenarios x one opt year (battery + PV + LP-relaxed ICE + DCM + retail,
          the synthetic 4-h requirement of scenarios.config5(min_soe=None)), solved with bench_configs' seeded schedule
          and all cold; objectives, statuses and iterations -> gpurun_out/certify/<label>.npz
  compare (host) the same windows rebuilt (deterministic) and solved by HiGHS on the restated LP, process pool;
          max / p99 relative objective error, optimal counts -> JSON

Usage: python scripts/certify_config5.py dump --scenarios 1000 --label c5_r05
       python scripts/certify_config5.py compare --label c5_r05 --json profiles/r05ze_certify_config5.json
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


def _sweep(S):
    from dervet_hip.lp import scenarios
    from dervet_hip.sweep import SeededSweep
    ids = list(range(S))
    P = scenarios.sweep_parameters(ids)
    return SeededSweep(lambda v: scenarios.config5(v, years=1), ids, P["E"], stride=32,
                       features=scenarios.sweep_features(P), blend=4)


def dump(args):
    import torch
    from dervet_hip import BatchSolver
    sw = _sweep(args.scenarios)
    dev = sw.packed.to_torch("cuda:0").alloc_outputs()
    s = BatchSolver(0)
    out = {"tags": np.array(sw.tags, np.int64), "scenarios": args.scenarios}
    for rep in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        tm, paths = sw.solve(s, dev)
        torch.cuda.synchronize()
        el = time.perf_counter() - t
    print(f"seeded: {el * 1e3:.1f} ms ({dev.count / el:.0f} windows/s) {paths}", flush=True)
    out["seeded_stats"], out["seeded_istats"] = dev.stats.cpu().numpy(), dev.istats.cpu().numpy()
    s.set_options(warm_start=0)
    for rep in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        s.solve_packed(dev)
        torch.cuda.synchronize()
        el = time.perf_counter() - t
    print(f"cold: {el * 1e3:.1f} ms ({dev.count / el:.0f} windows/s) {s.kernel_stats()}", flush=True)
    out["cold_stats"], out["cold_istats"] = dev.stats.cpu().numpy(), dev.istats.cpu().numpy()
    os.makedirs(os.path.join(ROOT, "gpurun_out", "certify"), exist_ok=True)
    path = os.path.join(ROOT, "gpurun_out", "certify", f"{args.label}.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, flush=True)


def _init(S):
    global _PB
    _PB = _sweep(S).packed


def _solve(k):
    from oracle import window_lp
    r = window_lp.solve_highs(window_lp.from_packed_window(_PB.window(int(k))))
    return r.get("obj", np.nan), r["status"]


def compare(args):
    g = np.load(os.path.join(ROOT, "gpurun_out", "certify", f"{args.label}.npz"))
    S = int(g["scenarios"])
    n = len(g["tags"])
    t = time.time()
    with get_context("fork").Pool(args.procs, initializer=_init, initargs=(S,)) as pool:
        res = pool.map(_solve, range(n), chunksize=16)
    hobj = np.array([r[0] for r in res])
    hst = np.array([r[1] for r in res])
    out = {"workload": f"config 5, {S} scenarios x 1 opt year x 12 monthly windows (ICE band form; synthetic 4-h "
                       f"requirement), HiGHS on the restated LP ({args.procs} processes, {time.time() - t:.0f} s)",
           "windows": n, "highs_optimal": int((hst == 0).sum())}
    for sched in ("seeded", "cold"):
        st, ist = g[f"{sched}_stats"], g[f"{sched}_istats"]
        ok = (hst == 0) & (ist[:, 0] == 0)
        rel = np.abs(st[ok, 0] - hobj[ok]) / np.maximum(np.abs(hobj[ok]), 1.0)
        out[sched] = {"gpu_optimal": int((ist[:, 0] == 0).sum()), "compared": int(ok.sum()),
                      "max_rel": float(rel.max()), "p99_rel": float(np.quantile(rel, 0.99)),
                      "mean_rel": float(rel.mean()), "n_gt_1e6": int((rel > 1e-6).sum()),
                      "n_gt_1e5": int((rel > 1e-5).sum()), "iters_mean": float(ist[:, 1].mean()),
                      "max_primal_res_rel": float(st[:, 1].max())}
    print(json.dumps(out, indent=1))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    a = sub.add_parser("dump")
    a.add_argument("--scenarios", type=int, default=1000)
    a.add_argument("--label", default="c5")
    b = sub.add_parser("compare")
    b.add_argument("--label", default="c5")
    b.add_argument("--procs", type=int, default=os.cpu_count() or 1)
    b.add_argument("--json", default=None)
    args = ap.parse_args()
    dump(args) if args.cmd == "dump" else compare(args)


if __name__ == "__main__":
    main()

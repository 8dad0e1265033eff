"""Secondary benchmark: the post-facto reliability sweep on one MI355X.

Workload: S synthetic scenarios of the config-2/4 site (critical load of data/multi_der_hourly_timeseries.csv
x LogNormal(0, 0.15), battery E ~ U[500, 10000] kWh, P = E / U[2, 6], rte ~ U[0.80, 0.95], PV rated
U[0, 2000] kW with nu = 20 %, gamma = 43 %, SOE at each start ~ U[0, E]), 8760 hourly outage starts each,
max outage 80 h: S x 8760 outage simulations per step.  Prints one JSON line: simulations/s (kernel time
from HIP events and wall time of the whole call), and the reference restatement (oracle/outage.py, the
serial per-start recursion of Reliability.py:489-570) timed on a bounded sample on one host core.

Usage: python bench_reliability.py [--scenarios S] [--steps K] [--warmup W]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "der-vet_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)


def make_cases(S, seed=20250217):
    from dervet_hip import reliability
    from dervet_hip.lp import scenarios
    ri = scenarios.reference_inputs()
    cl0 = ri["multi_der_critical_load"]
    pv0 = np.nan_to_num(ri["multi_der_pv_profile"])
    cases = []
    for s in range(S):
        rng = np.random.default_rng(seed + s)
        E = rng.uniform(500, 10000)
        P = E / rng.uniform(2, 6)
        cases.append(reliability.OutageCase(
            critical_load=cl0 * rng.lognormal(0.0, 0.15), dt=1.0, max_outage_duration=80,
            ess=dict(E=E, P_ch=P, P_dis=P, rte=rng.uniform(0.80, 0.95), llsoc=0.0, ulsoc=1.0),
            init_soe=rng.uniform(0, E, len(cl0)), pv_max=[rng.uniform(0, 2000) * pv0], pv_nu=[0.2],
            pv_gamma=[0.43]))
    return cases


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenarios", type=int, default=2000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-starts", type=int, default=8760 * 12)
    args = ap.parse_args()
    import torch
    if not torch.cuda.is_available():
        raise SystemExit("bench_reliability.py needs a GPU")
    from dervet_hip import BatchSolver, reliability
    cases = make_cases(args.scenarios)
    sims = sum(len(c.critical_load) for c in cases)
    s = BatchSolver(0)
    for _ in range(args.warmup):
        reliability.outage_coverage(cases, s)
    kms, walls = [], []
    for _ in range(args.steps):
        t = time.perf_counter()
        lengths, _ = reliability.outage_coverage(cases, s)
        walls.append(time.perf_counter() - t)
        kms.append(reliability.last_kernel_ms(s))
    steps_sim = int(sum(int(L.sum()) for L in lengths))
    # CPU: the serial restatement of the reference recursion on a bounded sample of scenario 0's starts
    from oracle import outage
    n = 0
    t = time.perf_counter()
    for c in cases:
        dg, pmax, props, pvar, gamma = reliability.der_mix_properties(c)
        cl = np.asarray(c.critical_load)
        for st in range(len(cl)):
            if n >= args.cpu_starts:
                break
            outage.simulate_outage(st, cl, np.zeros(len(pmax)), pmax, pvar, gamma, props, c.init_soe[st], 80, 80,
                                   1.0)
            n += 1
        if n >= args.cpu_starts:
            break
    cpu_s = time.perf_counter() - t
    k = float(np.mean(kms))
    line = {
        "metric": "reliability outage simulations/sec (load coverage probability sweep, 1 GPU)",
        "value": round(sims / (k * 1e-3), 1), "unit": "outage simulations/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(k, 3), "higher_is_better": True, "dtype": "f64",
        "data": "synthetic: config-4-style perturbations of data/multi_der_hourly_timeseries.csv critical load",
        "config": {"workload": f"{args.scenarios} scenarios x 8760 hourly outage starts, max outage 80 h",
                   "simulations": sims, "covered_steps_simulated": steps_sim},
        "wall_ms_per_call": round(1e3 * float(np.mean(walls)), 2),
        "cpu_baseline": {"value": round(n / cpu_s, 1), "unit": "outage simulations/s", "cores": 1, "kind": "port",
                         "sample": f"{n} outage starts (first scenarios), oracle/outage.py (serial restatement of "
                                   f"Reliability.py:489-570), {cpu_s:.1f} s"},
    }
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()

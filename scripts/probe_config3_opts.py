#!/usr/bin/env python3
"""Dev probe: BASELINE config 3 (the 5-minute annual battery + PV + DCM window, the long team of dvh_chain.hip) under
option sets -- iterations, solve time, objective error against the committed HiGHS golden.
Usage (GPU box): python scripts/probe_config3_opts.py [case: dcm | da] ['{"primal_weight_theta": 0.5}' ...]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "der-vet_amd")]
from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "dcm"
variants = [json.loads(v) for v in sys.argv[2:]] or [{}]
gold = json.load(open(os.path.join(ROOT, "tests", "golden", "config3_highs.json")))[case]["obj"]
lps = builder.group_window_lps(scenarios.config3(case)[0])
for v in variants:
    with BatchSolver(0, **v) as s:
        s.solve(lps)  # warm-up (first launch)
        t0 = time.perf_counter()
        r = s.solve(lps)[0]
        el = time.perf_counter() - t0
        tm = s.timing()
    print(f"{case} {json.dumps(v):70s} {r.status_name:10s} iters {r.iters:6d} wall {el * 1e3:7.1f} ms "
          f"(pdhg {tm['pdhg_ms']:6.1f}) rel err {abs(r.obj - gold) / abs(gold):.2e}", flush=True)

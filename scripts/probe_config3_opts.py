#!/usr/bin/env python3
"""Config 3 (5-minute annual window + 12 monthly DCM columns + fixed PV, the long team) under alternative restart /
check options: wall ms, iterations and the objective's error against the HiGHS golden (tests/golden/config3_highs.json).
Usage (GPU box): python scripts/probe_config3_opts.py"""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "der-vet_amd")]
import torch  # noqa: E402
from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402

gold = json.load(open(os.path.join(ROOT, "tests", "golden", "config3_highs.json")))["dcm"]
pb = builder.pack_groups(scenarios.config3("dcm"))
s = BatchSolver(0)
base = s.options()
SETS = [("default", {}),
        ("check64", {"check_every": 64}), ("check16", {"check_every": 16}),
        ("kkt2", {"kkt_every": 2}), ("kkt8", {"kkt_every": 8}),
        ("theta05", {"primal_weight_theta": 0.5}),
        ("art02", {"restart_artificial": 0.2}), ("art005", {"restart_artificial": 0.05}),
        ("suff01", {"restart_sufficient": 0.1}), ("suff03", {"restart_sufficient": 0.3}),
        ("nec09", {"restart_necessary": 0.9}), ("nec07", {"restart_necessary": 0.7})]
for name, opts in SETS:
    s.set_options(**{k: getattr(base, k) for k in ("check_every", "kkt_every", "primal_weight_theta", "restart_artificial",
                                                   "restart_sufficient", "restart_necessary")})
    s.set_options(**opts)
    dev = pb.to_torch("cuda:0").alloc_outputs()
    best = None
    for r in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        s.solve_packed(dev)
        torch.cuda.synchronize()
        el = time.perf_counter() - t
        best = el if best is None else min(best, el)
    st = dev.stats.cpu().numpy()[0]
    ist = dev.istats.cpu().numpy()[0]
    obj = float(st[0])
    print(json.dumps({"set": name, "options": opts, "ms": round(best * 1e3, 2), "status": int(ist[0]), "iters": int(ist[1]),
                      "obj_rel_err": abs(obj - gold["obj"]) / max(abs(gold["obj"]), 1.0)}), flush=True)
    del dev

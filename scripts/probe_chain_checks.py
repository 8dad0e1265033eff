#!/usr/bin/env python3
"""Team kernel: what the restart and KKT checks cost per iteration, at a fixed iteration count (eps 1e-14: no window
converges), on config 3 DCM + PV and 64 annual windows (the medium tier).
Usage (GPU box): python scripts/probe_chain_checks.py [iters]"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "der-vet_amd")]
import torch  # noqa: E402
from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
s = BatchSolver(0)
for v in ("dcm", "year64"):
    groups = scenarios.config4(range(64), n="year") if v == "year64" else scenarios.config3(v)
    pb = builder.pack_groups(groups)
    dev = pb.to_torch("cuda:0").alloc_outputs()
    for ce, ke in ((32, 4), (32, 1000), (1024, 1000), (64, 2)):
        s.set_options(max_iters=N, eps=1e-14, eps_obj=1e-14, check_every=ce, kkt_every=ke)
        best = None
        for r in range(3):
            s.solve_packed(dev)
            torch.cuda.synchronize()
            t = s.timing()["pdhg_ms"]
            best = t if best is None else min(best, t)
        it = int(dev.istats[:, 1].max())
        print(json.dumps({"variant": v, "check_every": ce, "kkt_every": ke, "iters": it, "pdhg_ms": round(best, 2),
                          "us_per_iter": round(1e3 * best / it, 3)}), flush=True)

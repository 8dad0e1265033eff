#!/usr/bin/env python3
"""Per-iteration time of the team kernel on BASELINE config 3's variants at a fixed iteration count (eps 1e-14: no
window converges, so every variant runs exactly --iters iterations): which part of a team iteration costs what.
Usage: python scripts/probe_chain.py [--iters 8192] [variants ...]   (DVH_LIB picks a library build)"""
import argparse, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "der-vet_amd")]
import torch  # noqa: E402
from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=8192)
ap.add_argument("variants", nargs="*", default=["da", "dcm_nopv", "dcm"])
a = ap.parse_args()
s = BatchSolver(0)
for v in a.variants:
    if v == "dcm_nopv":
        ri = scenarios.reference_inputs()
        groups = scenarios.windows_by_period(2019, 1.0 / 12, ri["fivemin_site_load"][None, :], None,
                                             scenarios.template_battery(), da_price=ri["fivemin_da_price"][None, :],
                                             tariff_def=scenarios.tariff(), n="year")
    elif v.startswith("year"):  # annual hourly windows of config-4 scenarios (the medium tier), e.g. year64
        groups = scenarios.config4(range(int(v[4:] or 64)), n="year")
    else:
        groups = scenarios.config3(v)
    pb = builder.pack_groups(groups)
    dev = pb.to_torch("cuda:0").alloc_outputs()
    s.set_options(max_iters=a.iters, eps=1e-14, eps_obj=1e-14)
    best = None
    for r in range(3):
        s.solve_packed(dev)
        torch.cuda.synchronize()
        t = s.timing()["pdhg_ms"]
        best = t if best is None else min(best, t)
    it = int(dev.istats[:, 1].max())
    print(json.dumps({"variant": v, "windows": pb.count, "iters": it, "pdhg_ms": round(best, 2),
                      "us_per_iter": round(1e3 * best / it, 3), "paths": s.kernel_stats()}), flush=True)

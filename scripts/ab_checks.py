"""Cost of the restart / KKT checks in the battery-banded kernel: per window-iteration time at a fixed iteration
count (no convergence) for several (check_every, kkt_every) settings, on config-4 windows.

Usage: python scripts/ab_checks.py <scenarios> <fixed_iters> [config4|config1]
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "der-vet_amd"))

import torch  # noqa: E402

from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402


def main():
    S, iters = int(sys.argv[1]), int(sys.argv[2])
    which = sys.argv[3] if len(sys.argv) > 3 else "config4"
    groups = scenarios.config4(range(S)) if which == "config4" else scenarios.config1() * S
    pb = builder.pack_groups(groups)
    dev = pb.to_torch("cuda:0").alloc_outputs()
    s = BatchSolver(0)
    out = {}
    for ce, ke in ((1000000, 1), (32, 4), (64, 2), (64, 4), (128, 1)):
        s.set_options(eps=1e-30, eps_obj=0.0, max_iters=iters, check_every=ce, kkt_every=ke)
        best = None
        for _ in range(3):
            s.solve_packed(dev)
            torch.cuda.synchronize()
            t = s.timing()["pdhg_ms"]
            best = t if best is None else min(best, t)
        out[f"{ce}/{ke}"] = round(best * 1e3 / (pb.count / 256.0) / iters, 4)
        print(f"check {ce:>7} kkt {ke}: {out[f'{ce}/{ke}']:.4f} us per window-iteration per CU", flush=True)
    print("RESULT " + json.dumps(out))


if __name__ == "__main__":
    main()

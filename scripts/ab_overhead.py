"""Per-window fixed cost of the battery-banded kernel (structure check, coefficient loads, power iteration,
output) vs its per-iteration cost: kernel time per window at several fixed iteration counts and power-iteration
counts, config-4 windows.

Usage: python scripts/ab_overhead.py <scenarios>
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
    S = int(sys.argv[1])
    pb = builder.pack_groups(scenarios.config4(range(S)))
    dev = pb.to_torch("cuda:0").alloc_outputs()
    s = BatchSolver(0)
    out = {}
    for pw in (1, 64):
        for iters in (32, 1024, 4096):
            s.set_options(eps=1e-30, eps_obj=0.0, max_iters=iters, check_every=64, kkt_every=2, power_iters=pw)
            best = None
            for _ in range(3):
                s.solve_packed(dev)
                torch.cuda.synchronize()
                t = s.timing()
                best = t if best is None or t["pdhg_ms"] < best["pdhg_ms"] else best
            key = f"power{pw}_iters{iters}"
            out[key] = {"us_per_window_per_cu": round(best["pdhg_ms"] * 1e3 / (pb.count / 256.0), 2),
                        "setup_ms": round(best["setup_ms"], 3)}
            print(key, out[key], flush=True)
    print("RESULT " + json.dumps(out))


if __name__ == "__main__":
    main()

"""Setup-kernel cost on the bench batch (dev helper): setup ms per solve for several Ruiz pass counts, and the
pass count the early exit stops at.  Usage: python scripts/probe_setup.py [scenarios]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "der-vet_amd"))
import torch  # noqa: E402

from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import scenarios  # noqa: E402


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    from dervet_hip.lp import gpu_builder
    s = BatchSolver(0)
    specs = scenarios.config4(range(S), spec=True)
    dev = gpu_builder.pack_specs_device(specs, s, "cuda:0")
    out = {}
    for ri in (0, 1, 5, 10):
        s.set_options(max_iters=1, ruiz_iters=ri, power_iters=1)
        best = None
        for _ in range(3):
            s.solve_packed(dev)
            torch.cuda.synchronize()
            t = s.timing()["setup_ms"]
            best = t if best is None else min(best, t)
        out[f"ruiz{ri}"] = round(best, 2)
    print("RESULT " + json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

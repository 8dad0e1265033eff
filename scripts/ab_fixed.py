"""Per-iteration cost of library builds at a FIXED iteration count (no convergence; dev helper for A/B of
kernel variants built with scripts/build_variants.sh, including deliberately incomplete ablations).

Usage: python scripts/ab_fixed.py <scenarios> <iters> <lib.so> [<lib.so> ...]
       DVH_AB_OPTS='{"label": {"check_every": 16, "kkt_every": 4}, ...}' overrides the option sets.
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_SETS = {"plain": dict(check_every=1000000, kkt_every=1), "default": dict(check_every=32, kkt_every=4)}
CHILD = r'''
import sys, os, json
sys.path.insert(0, os.path.join(%r, "..", "der-vet_amd"))
import torch
from dervet_hip import BatchSolver, _lib
_lib.LIB_PATH = %r
from dervet_hip.lp import scenarios, builder
pb = builder.pack_groups(scenarios.config4(range(%d)))
dev = pb.to_torch("cuda:0").alloc_outputs()
s = BatchSolver(0)
out = {}
for label, kw in json.loads(%r).items():
    s.set_options(eps=1e-30, max_iters=%d, **kw)
    best = None
    for rep in range(3):
        s.solve_packed(dev); torch.cuda.synchronize()
        t = s.timing()["pdhg_ms"]
        best = t if best is None else min(best, t)
    out[label] = best * 1e3 / (pb.count / 256.0) / %d
print("RESULT " + json.dumps(out))
'''


def main():
    S, iters = int(sys.argv[1]), int(sys.argv[2])
    sets = os.environ.get("DVH_AB_OPTS") or json.dumps(DEFAULT_SETS)
    for lib in sys.argv[3:]:
        code = CHILD % (HERE, os.path.abspath(lib), S, sets, iters, iters)
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600)
        line = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
        if r.returncode != 0 or not line:
            print(f"{lib}: FAILED rc={r.returncode}\n{r.stderr[-1500:]}", flush=True)
            continue
        res = json.loads(line[0][7:])
        print(f"{os.path.basename(lib):24s} " + "  ".join(f"{k} {v:.3f}" for k, v in res.items()) + "  us/iter/CU",
              flush=True)


if __name__ == "__main__":
    main()

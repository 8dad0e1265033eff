"""A/B of library builds on a config-4 sample (dev helper; variants from scripts/build_variants.sh).

Usage: python scripts/ab_variants.py <scenarios> <lib.so> [<lib.so> ...]
Each library runs in its own subprocess (one ctypes load per process); prints PDHG kernel time, iteration
totals, time per window-iteration and the max objective difference against the first library.
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))

CHILD = r'''
import sys, os, json
sys.path.insert(0, os.path.join(%r, "..", "der-vet_amd"))
import numpy as np, torch
from dervet_hip import BatchSolver, _lib
_lib.LIB_PATH = %r
from dervet_hip.lp import scenarios, builder
gs = scenarios.config4(range(%d)); pb = builder.pack_groups(gs)
dev = pb.to_torch("cuda:0").alloc_outputs()
s = BatchSolver(0)
s.solve_packed(dev); torch.cuda.synchronize()
best = None
for rep in range(2):
    s.solve_packed(dev); torch.cuda.synchronize()
    tm = s.timing()
    best = tm if best is None or tm["pdhg_ms"] < best["pdhg_ms"] else best
ist = dev.istats.cpu().numpy(); st = dev.stats.cpu().numpy()
np.save(%r, st[:, 0])
print("RESULT " + json.dumps({"pdhg_ms": best["pdhg_ms"], "setup_ms": best["setup_ms"], "iters": int(ist[:, 1].sum()),
      "iters_max": int(ist[:, 1].max()), "optimal": int((ist[:, 0] == 0).sum()), "n": int(pb.count),
      "paths": s.kernel_stats()}))
'''


def main():
    S = int(sys.argv[1])
    libs = sys.argv[2:]
    out = os.path.join(HERE, "..", "gpurun_out")
    os.makedirs(out, exist_ok=True)
    base = None
    for i, lib in enumerate(libs):
        npy = os.path.join(out, f"ab_obj_{i}.npy")
        code = CHILD % (HERE, os.path.abspath(lib), S, npy)
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600)
        line = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
        if r.returncode != 0 or not line:
            print(f"{lib}: FAILED rc={r.returncode}\n{r.stderr[-2000:]}", flush=True)
            return 1
        res = json.loads(line[0][7:])
        import numpy as np
        obj = np.load(npy)
        if base is None:
            base = obj
        rel = float(np.max(np.abs(obj - base) / np.maximum(np.abs(base), 1e-12)))
        per_us = res["pdhg_ms"] * 1e3 / (res["iters"] / 256.0)
        print(f"{os.path.basename(lib):28s} pdhg {res['pdhg_ms']:8.1f} ms  setup {res['setup_ms']:6.1f}  iters {res['iters']} "
              f"(max {res['iters_max']})  opt {res['optimal']}/{res['n']}  {per_us:.3f} us/iter/CU  "
              f"max rel obj diff vs first {rel:.2e}  {res['paths']}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""A/B of libdervet_hip builds (scripts/build_variants.sh) on config-4 windows: per-iteration cost at a fixed
iteration count (no convergence) and a converged cold solve (time, mean iterations, objectives vs the first build).

Usage: python scripts/ab_band.py <scenarios> <fixed_iters> <lib.so> [<lib.so> ...]
"""
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
CHILD = r'''
import sys, os, json
sys.path.insert(0, os.path.join(%r, "..", "der-vet_amd"))
import numpy as np, torch
from dervet_hip import BatchSolver, _lib
_lib.LIB_PATH = %r
from dervet_hip.lp import scenarios, builder
pb = builder.pack_groups(scenarios.config4(range(%d)))
dev = pb.to_torch("cuda:0").alloc_outputs()
s = BatchSolver(0)
out = {}
for label, kw in (("plain", dict(check_every=1000000, kkt_every=1)), ("checks", dict(check_every=32, kkt_every=4)),
                  ("warm64_2", dict(check_every=64, kkt_every=2)), ("kkt32_1", dict(check_every=32, kkt_every=1))):
    s.set_options(eps=1e-30, eps_obj=0.0, max_iters=%d, **kw)
    best = None
    for rep in range(3):
        s.solve_packed(dev); torch.cuda.synchronize()
        t = s.timing()["pdhg_ms"]
        best = t if best is None else min(best, t)
    out[label] = best * 1e3 / (pb.count / 256.0) / %d
s.set_options(eps=1e-6, eps_obj=1e-6, max_iters=100000, check_every=32, kkt_every=4)
best = None
for rep in range(2):
    s.solve_packed(dev); torch.cuda.synchronize()
    t = s.timing()["pdhg_ms"]
    best = t if best is None else min(best, t)
ist = dev.istats.cpu().numpy()
out["solve_ms"] = best
out["iters"] = float(ist[:, 1].mean())
out["optimal"] = float((ist[:, 0] == 0).mean())
out["paths"] = s.kernel_stats()
np.save(%r, dev.stats.cpu().numpy()[:, 0])
print("RESULT " + json.dumps(out))
'''


def main():
    S, iters = int(sys.argv[1]), int(sys.argv[2])
    ref = None
    for k, lib in enumerate(sys.argv[3:]):
        obj_path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"ab_band_{k}.npy")
        code = CHILD % (HERE, os.path.abspath(lib), S, iters, iters, obj_path)
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=900)
        line = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
        if r.returncode != 0 or not line:
            print(f"{lib}: FAILED rc={r.returncode}\n{r.stderr[-2000:]}", flush=True)
            continue
        res = json.loads(line[0][7:])
        obj = np.load(obj_path)
        if ref is None:
            ref = obj
        d = float(np.max(np.abs(obj - ref) / np.maximum(np.abs(ref), 1.0)))
        print(f"{os.path.basename(lib):22s} plain {res['plain']:.3f} checks {res['checks']:.3f} 64/2 {res['warm64_2']:.3f} "
              f"32/1 {res['kkt32_1']:.3f} us/iter/CU | solve "
              f"{res['solve_ms']:.1f} ms, iters {res['iters']:.1f}, optimal {res['optimal']:.4f}, max obj diff vs "
              f"first {d:.2e}, band {res['paths']['band_windows']}", flush=True)


if __name__ == "__main__":
    main()

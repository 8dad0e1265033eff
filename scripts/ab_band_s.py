"""A/B of the battery band kernel's steps-per-lane forms (DVH_BAND_S=1: 768 threads, one window per CU; DVH_BAND_S=2:
384 threads, two steps per lane, two windows per CU) on config-4 windows: per window-iteration cost at a fixed
iteration count (no convergence, with and without checks) and a converged cold solve (time, iterations, statuses,
objective agreement between the forms).

Usage: python scripts/ab_band_s.py <scenarios> <fixed_iters> [S ...]
"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CHILD = r'''
import sys, os, json
import numpy as np
sys.path.insert(0, os.path.join(%r, "..", "der-vet_amd"))
import torch
from dervet_hip import BatchSolver
from dervet_hip.lp import scenarios, builder
pb = builder.pack_groups(scenarios.config4(range(%d)))
dev = pb.to_torch("cuda:0").alloc_outputs()
s = BatchSolver(0)
out = {}
iters = %d
for label, kw in (("plain", dict(check_every=1000000, kkt_every=1)), ("checks", dict(check_every=64, kkt_every=2))):
    s.set_options(eps=1e-30, eps_obj=0.0, max_iters=iters, **kw)
    best = None
    for rep in range(3):
        s.solve_packed(dev); torch.cuda.synchronize()
        t = s.timing()["pdhg_ms"]
        best = t if best is None else min(best, t)
    out[label] = round(best * 1e3 / (pb.count / 256.0) / iters, 4)
s.set_options()
best = None
for rep in range(2):
    s.solve_packed(dev); torch.cuda.synchronize()
    t = s.timing()["pdhg_ms"]
    best = t if best is None else min(best, t)
st = dev.istats.cpu().numpy()
obj = dev.stats.cpu().numpy()[:, 0]
np.save(%r, obj)
out.update(solve_ms=round(best, 2), iters_mean=float(st[:, 1].mean()), iters_max=int(st[:, 1].max()),
           optimal=float((st[:, 0] == 0).mean()), kernel=s.kernel_stats())
print("RESULT " + json.dumps(out))
'''


def main():
    S, iters = int(sys.argv[1]), int(sys.argv[2])
    forms = [int(a) for a in sys.argv[3:]] or [1, 2]
    objs = {}
    for f in forms:
        fn = f"/tmp/ab_band_s_obj{f}.npy"
        env = dict(os.environ, DVH_BAND_S=str(f))
        r = subprocess.run([sys.executable, "-c", CHILD % (HERE, S, iters, fn)], capture_output=True, text=True,
                           timeout=600, env=env)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
        if r.returncode != 0 or not line:
            print(f"S={f}: FAILED rc={r.returncode}\n{r.stderr[-2000:]}", flush=True)
            continue
        res = json.loads(line[0][7:])
        import numpy as np
        objs[f] = np.load(fn)
        if len(objs) > 1:
            a, b = objs[forms[0]], objs[f]
            res["max_obj_rel_diff_vs_first"] = float(np.max(np.abs(a - b) / np.maximum(1.0, np.abs(a))))
        print(f"S={f}: " + json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

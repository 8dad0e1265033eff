"""Lab: iterations to re-converge from a start of the SAME window at accuracy eps0 (cold solve stopped at eps0, then
a fresh warm solve to 1e-6) vs the uninterrupted cold solve.  Usage: python scripts/lab/restart_penalty.py S eps0..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np  # noqa: E402
from lab import Lab, builder, scenarios  # noqa: E402

S = int(sys.argv[1])
lps = [lp for g in scenarios.config4(range(S)) for lp in builder.group_window_lps(g)]
lab = Lab()
full = lab.solve(lps, check_every=32, kkt_every=1)
print(f"cold to 1e-6: mean {full['iters'].mean():.1f}")
for e0 in [float(v) for v in sys.argv[2:]]:
    a = lab.solve(lps, check_every=32, kkt_every=1, eps=e0, eps_obj=e0)
    b = lab.solve(lps, list(zip(a["x"], a["y"])), check_every=64, kkt_every=1, warm_start=1)
    print(f"eps0 {e0:.0e}: phase 1 {a['iters'].mean():.1f} + phase 2 {b['iters'].mean():.1f} = "
          f"{a['iters'].mean() + b['iters'].mean():.1f}  (p2 p99 {np.percentile(b['iters'], 99):.0f}) "
          f"max rel obj {np.max(np.abs(b['obj'] - full['obj']) / np.abs(full['obj'])):.1e}", flush=True)

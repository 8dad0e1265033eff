"""Config 3 on the large-LP path: timing, iterations, objective vs HiGHS (dev helper; GPU box)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "der-vet_amd"))
import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402

from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402
from oracle import window_lp  # noqa: E402

variant = sys.argv[1] if len(sys.argv) > 1 else "da"
ri = scenarios.reference_inputs()
T = len(ri["fivemin_da_price"])
if variant == "da":
    g = scenarios.windows_by_period(2019, 1.0 / 12, np.zeros((1, T)), None, scenarios.template_battery(),
                                    da_price=ri["fivemin_da_price"][None, :], n="year")
else:
    g = scenarios.windows_by_period(2019, 1.0 / 12, ri["fivemin_site_load"][None, :], None,
                                    scenarios.template_battery(), da_price=ri["fivemin_da_price"][None, :],
                                    tariff_def=scenarios.tariff(), n="year")
lp = builder.group_window_lps(g[0])[0]
print("n", lp.n, "m", lp.m, "nnz", len(lp.data), flush=True)
with BatchSolver(0) as s:
    for rep in range(int(sys.argv[2]) if len(sys.argv) > 2 else 2):
        t = time.time()
        r = s.solve([lp])[0]
        wall = time.time() - t
        print(f"rep {rep}: status {r.status_name} iters {r.iters} obj {r.obj:.10g} wall {wall:.3f}s timing {s.timing()} "
              f"paths {s.kernel_stats()} pres {r.primal_res_rel:.2e} dres {r.dual_res_rel:.2e} gap {r.gap_rel:.2e}",
              flush=True)
if variant == "da":
    K = sp.csr_matrix((lp.data, lp.indices, lp.indptr), shape=(lp.m, lp.n))
    t = time.time()
    h = window_lp.solve_highs(dict(K=K, q=lp.q, c=lp.c, c0=lp.c0, l=lp.l, u=lp.u, m_eq=lp.m_eq))
    print(f"highs obj {h['obj']:.10g} rel err {abs(r.obj - h['obj']) / abs(h['obj']):.2e}  ({time.time() - t:.1f}s)")

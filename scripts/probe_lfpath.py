import sys, os
sys.path.insert(0, "der-vet_amd"); sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from test_market_reserves import _signals, _lf, reserve_series
from dervet_hip.lp import scenarios, builder
from dervet_hip import BatchSolver
sig, meta = _signals("es")
pdis = float(meta["params"]["Battery"]["dis_max_rated"])
for lfon, rs in ((False, True), (True, False), (True, True)):
    g = scenarios.market_days(sig, meta["params"], days=list(range(0, 40)), reserves=reserve_series(sig, pdis) if rs else None,
                              lf=_lf(sig, pdis) if lfon else None)
    s = BatchSolver(0)
    r = s.solve(builder.group_window_lps(g))
    print("lf", lfon, "res", rs, "n", g.n, "m", g.m, s.kernel_stats(), [x.status for x in r[:3]], flush=True)

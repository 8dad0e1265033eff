#!/usr/bin/env python3
"""Market days with reserves / load following: ELL (default) vs generic kernel wall per solve (median of 5)."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "der-vet_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
from dervet_hip import BatchSolver
from dervet_hip.lp import builder, scenarios
from oracle import cases
from test_market_reserves import reserve_series, _lf
arr, meta = cases.load_market()
sig = {k.split("__", 1)[1]: v for k, v in arr.items() if k.startswith("es__")}
pdis = float(meta["es"]["params"]["Battery"]["dis_max_rated"])
s = BatchSolver(0)
for kind in ("fr", "reserves", "lf", "lf_combined"):
    for days in (list(range(3, 365, 20)), list(range(0, 365, 3)), list(range(365))):
        kw = dict(reserves=reserve_series(sig, pdis)) if kind != "fr" else {}
        if kind.startswith("lf"):
            kw["lf"] = _lf(sig, pdis, combined=kind == "lf_combined")
        g = scenarios.market_days(sig, meta["es"]["params"], days=days, **kw)
        dev = builder.pack_groups([g]).to_torch("cuda:0").alloc_outputs()
        out = {"kind": kind, "days": g.G, "n": g.n, "m": g.m, "small": os.environ.get("DVH_SMALL", "on")}
        for path in ("ell", "generic"):
            s.set_kernel_path(path)
            s.solve_packed(dev)
            ts = []
            for _ in range(5):
                torch.cuda.synchronize(); t = time.perf_counter(); s.solve_packed(dev); torch.cuda.synchronize()
                ts.append(time.perf_counter() - t)
            out[path] = round(1e3 * float(np.median(ts)), 2)
            out[path + "_variant"] = s.kernel_stats()["variant"]
        print(json.dumps(out), flush=True)

#!/usr/bin/env python3
"""Market-day routing A/B: the 3 x 365 Usecase 3 days of bench_configs.py --only 6 (DA + FR), the same days with
SR + NSR, with LF + SR + NSR, and with CombinedMarket LF, timed on the default route and on the generic kernel
(best of 5 after a warm-up).  The small-window variant is chosen by the DVH_SMALL environment variable of the
process (dvh_kernels.hip small_dispatch: unset = the routing table, -1 = off, k = force variant k).

Usage: DVH_SMALL=<v> [MARKET_DAYS=d (days per case, default 365)] python scripts/probe_market_variants.py [kinds]   (kinds: fr,fr_default,reserves,lf,lf_combined)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "der-vet_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402


def workloads(kinds):
    gold = os.path.join(ROOT, "tests", "golden")
    arr = dict(np.load(os.path.join(gold, "uc3_market.npz")))
    with open(os.path.join(gold, "uc3_market.json")) as f:
        meta = json.load(f)
    names = ("es", "es+pv", "es+pv+dg")
    for kind in kinds:
        groups = []
        for nm in names:
            sg = {k.split("__", 1)[1]: v for k, v in arr.items() if k.startswith(nm + "__")}
            pdis = float(meta[nm]["params"]["Battery"]["dis_max_rated"])
            N = len(sg["da_price"])
            h = np.arange(N)
            kw = {}
            if kind in ("reserves", "lf", "lf_combined"):
                kw["reserves"] = [dict(key="SR", price=0.6 * sg["regu_price"], duration=0.5, max=np.full(N, 0.5 * pdis),
                                       min=np.zeros(N)), dict(key="NSR", price=0.3 * sg["regu_price"], duration=1.0)]
            if kind.startswith("lf"):
                kw["lf"] = dict(eou=0.2 + 0.05 * np.sin(h / 7.0), eod=0.2 + 0.05 * np.cos(h / 5.0),
                                up_price=0.8 * sg["regu_price"], down_price=0.8 * sg["regd_price"],
                                energy_price=sg["da_price"], up_max=np.full(N, 0.25 * pdis), up_min=np.zeros(N),
                                down_max=np.full(N, 0.25 * pdis), down_min=np.zeros(N), combined=kind == "lf_combined")
            nd = int(os.environ.get("MARKET_DAYS", "365"))
            days = list(range(0, 365, max(1, 365 // nd)))[:nd]
            groups.append(scenarios.market_days(sg, meta[nm]["params"], days=days, **kw))
        yield kind, builder.pack_groups(groups)


def main(argv):
    kinds = argv[0].split(",") if argv else ["fr", "fr_default", "reserves", "lf", "lf_combined"]
    s = BatchSolver(0)
    o0 = s.options()
    base = {k: getattr(o0, k) for k in scenarios.MARKET_OPTIONS}
    for kind, pb in workloads(kinds):
        dev = pb.to_torch("cuda:0").alloc_outputs()
        s.set_options(**(base if kind == "fr_default" else scenarios.MARKET_OPTIONS))
        d = np.asarray(pb.desc)
        out = {"kind": kind, "windows": pb.count, "n": int(d[:, 0].max()), "m": int(d[:, 1].max()),
               "small": os.environ.get("DVH_SMALL", "table")}
        for path in ("default", "generic"):
            s.set_kernel_path(path)
            s.solve_packed(dev)
            ts = []
            for _ in range(5):
                torch.cuda.synchronize()
                t = time.perf_counter()
                s.solve_packed(dev)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t)
            ist = dev.istats.cpu().numpy()
            out[path] = {"ms": round(1e3 * min(ts), 2), "variant": s.kernel_stats()["variant"],
                         "optimal": int((ist[:, 0] == 0).sum()), "iters_max": int(ist[:, 1].max()),
                         "paths": {k: v for k, v in s.kernel_stats().items() if k.endswith("_windows") and v}}
        s.set_kernel_path("default")
        print(json.dumps(out), flush=True)
        del dev


if __name__ == "__main__":
    main(sys.argv[1:])

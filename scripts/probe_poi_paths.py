#!/usr/bin/env python3
"""POI / PV-curtailment windows (tests/test_gpu_poi.py's rows: MicrogridPOI.py:215-258 import/export limits, charge
from PV with curtailable PV) at several window lengths, S scenarios each (load scaled per scenario): wall of the
default route vs the generic CSR kernel (best of 5 after a warm-up), variant and optimal count.

Usage: python scripts/probe_poi_paths.py [S] [lengths, e.g. 240,480,month]
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
from oracle import cases  # noqa: E402


def groups(kind, S, n):
    wins, arr, meta, _ = cases.case_windows("es+pv+dg")
    p = meta["params"]
    gen = float(p["PV"]["rated_capacity"]) * np.nan_to_num(arr["pv_profile"])
    bat = cases.battery_from_params(p)
    scale = np.linspace(0.8, 1.2, S)[:, None]
    load = arr["site_load"][None] * scale
    kw = dict(pv_curtail_max=np.repeat((12.0 * gen)[None], S, 0))
    if kind == "poi_no_export":
        kw["poi"] = dict(max_import=-12000.0, max_export=0.0)
    else:
        kw["grid_charge"] = False
    return scenarios.windows_by_period(2017, 1.0, load, np.zeros((S, gen.size)), bat, tariff_def=meta["tariff"],
                                       ene_min=np.repeat(arr["agg_emin"][None], S, 0),
                                       ene_max=np.repeat(arr["agg_emax"][None], S, 0), n=n, **kw)


def main(argv):
    S = int(argv[0]) if argv else 64
    lengths = argv[1].split(",") if len(argv) > 1 else ["240", "480", "month"]
    s = BatchSolver(0)
    for n in lengths:
        for kind in ("poi_no_export", "grid_charge_curtailable"):
            pb = builder.pack_groups(groups(kind, S, n if n == "month" else int(n)))
            dev = pb.to_torch("cuda:0").alloc_outputs()
            d = np.asarray(pb.desc)
            out = {"kind": kind, "length": n, "windows": pb.count, "n": int(d[:, 0].max()), "m": int(d[:, 1].max())}
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
                ks = s.kernel_stats()
                out[path] = {"ms": round(1e3 * min(ts), 2), "variant": ks["variant"],
                             "optimal": int((ist[:, 0] == 0).sum()), "iters_max": int(ist[:, 1].max()),
                             "paths": {k: v for k, v in ks.items() if k.endswith("_windows") and v}}
            s.set_kernel_path("default")
            print(json.dumps(out), flush=True)
            del dev


if __name__ == "__main__":
    main(sys.argv[1:])

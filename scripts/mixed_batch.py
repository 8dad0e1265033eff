#!/usr/bin/env python3
"""A mixed batch through one dvh_solve_packed_device call -- every kernel tier at once: Usecase 3 market days (ELL),
config-4 monthly windows (battery band), config-5 windows (band ICE), POI + curtailable-PV windows (generic CSR),
annual hourly windows (medium tier) and the 5-minute annual window (long team) -- printing one SHA-256 of every
window's (x, y, stats, istats) per group, the kernel paths, the host syncs and the wall time.  DVH_LIB selects the
library, so two builds can be compared bit for bit (scripts/ab_cascade.sh).  Usage: mixed_batch.py [out.json]"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "der-vet_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from dervet_hip import _lib  # noqa: E402

if os.environ.get("DVH_LIB"):  # an earlier build (A/B) may predate dvh_last_host_syncs
    import ctypes
    if not hasattr(ctypes.CDLL(os.environ["DVH_LIB"]), "dvh_last_host_syncs"):
        _lib.SYMBOLS.pop("dvh_last_host_syncs")
from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402
from oracle import cases  # noqa: E402


def groups():
    arr, meta = cases.load_market()
    sig = {k.split("__", 1)[1]: v for k, v in arr.items() if k.startswith("es__")}
    out = [("market", [scenarios.market_days(sig, meta["es"]["params"], days=list(range(0, 365, 3)))])]
    out.append(("config4", scenarios.config4(range(24))))
    out.append(("config5", scenarios.config5(range(4), years=1)))
    wins, a, m, _ = cases.case_windows("es+pv+dg")
    gen = float(m["params"]["PV"]["rated_capacity"]) * np.nan_to_num(a["pv_profile"])
    out.append(("poi", scenarios.windows_by_period(2017, 1.0, a["site_load"][None], np.zeros_like(gen)[None],
                                                   cases.battery_from_params(m["params"]), tariff_def=m["tariff"],
                                                   ene_min=a["agg_emin"][None], ene_max=a["agg_emax"][None],
                                                   grid_charge=False, pv_curtail_max=(12.0 * gen)[None])))
    out.append(("annual", scenarios.config4([0, 1], n="year")))
    out.append(("config3", scenarios.config3("da")))
    return out


def main():
    gs = groups()
    flat = [g for _, gl in gs for g in gl]
    pb = builder.pack_groups(flat)
    sizes = [sum(g.G for g in gl) for _, gl in gs]
    dev = pb.to_torch("cuda:0").alloc_outputs()
    s = BatchSolver(0)
    s.solve_packed(dev)  # warm-up: workspace sizing, code objects
    dev.x.zero_()
    dev.y.zero_()
    walls = []
    for _ in range(5):
        torch.cuda.synchronize()
        t = time.perf_counter()
        s.solve_packed(dev)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t)
    wall = float(np.median(walls))
    desc = np.asarray(pb.desc)
    x, y = dev.x.cpu().numpy(), dev.y.cpu().numpy()
    st, ist = dev.stats.cpu().numpy(), dev.istats.cpu().numpy()
    out = {"groups": {}, "paths": s.kernel_stats(), "host_syncs": s.host_syncs() if "dvh_last_host_syncs" in _lib.SYMBOLS else None, "wall_ms": round(1e3 * wall, 2), "wall_ms_all": [round(1e3 * v, 2) for v in walls],
           "lib": os.environ.get("DVH_LIB", "default")}
    k = 0
    for (name, _), n in zip(gs, sizes):
        h = hashlib.sha256()
        for w in range(k, k + n):
            d = desc[w]
            h.update(x[d[6]:d[6] + d[0]].tobytes())
            h.update(y[d[7]:d[7] + d[1]].tobytes())
            h.update(st[w].tobytes())
            h.update(ist[w].tobytes())
        out["groups"][name] = {"windows": n, "sha256": h.hexdigest()[:32],
                               "optimal": int((ist[k:k + n, 0] == 0).sum())}
        k += n
    del dev
    s.close()  # release the handle before interpreter teardown (the profiler's exit hooks run after it)
    line = json.dumps(out)
    print(line, flush=True)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()

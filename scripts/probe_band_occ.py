"""Residency probe of the band kernel forms: PDHG time at a fixed iteration count for batches of about 1, 2 and 3
windows per CU (252 / 504 / 756 config-4 windows on 256 CUs).  If two windows share a CU, the 504-window time stays
close to the 252-window time.  Usage: DVH_BAND_S=<1|2> python scripts/probe_band_occ.py [iters]
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "der-vet_amd"))

import torch  # noqa: E402

from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    s = BatchSolver(0)
    s.set_options(eps=1e-30, eps_obj=0.0, max_iters=iters, check_every=1000000, kkt_every=1)
    out = {"S": os.environ.get("DVH_BAND_S", "2")}
    for nsc in (21, 42, 63):
        pb = builder.pack_groups(scenarios.config4(range(nsc)))
        dev = pb.to_torch("cuda:0").alloc_outputs()
        best = None
        for _ in range(3):
            s.solve_packed(dev)
            torch.cuda.synchronize()
            t = s.timing()["pdhg_ms"]
            best = t if best is None else min(best, t)
        out[str(pb.count)] = round(best, 3)
    print("RESULT " + json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

"""Cold-solve parameter sweep (dev helper): the bench's 120,000 config-4 windows (device-built) solved cold with
different dvh_options.  Prints PDHG time, iterations and the objective difference to the first variant.

Usage: python scripts/cold_params.py <scenarios> '<json list of option dicts>'
"""
import functools
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "der-vet_amd"))
import numpy as np  # noqa: E402

from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import gpu_builder, scenarios  # noqa: E402


def main():
    S = int(sys.argv[1])
    variants = json.loads(sys.argv[2])
    s = BatchSolver(0)
    specs = functools.partial(scenarios.config4, spec=True)(range(S))
    dev = gpu_builder.pack_specs_device(specs, s, "cuda:0")
    o0 = s.options()
    base = None
    for v in variants:
        s.set_options(**v)
        tms = []
        for rep in range(2):
            s.solve_packed(dev)
            tms.append(s.timing()["pdhg_ms"])
        s.set_options(**{k: getattr(o0, k) for k in v})
        ist = dev.istats.cpu().numpy()
        obj = dev.stats.cpu().numpy()[:, 0]
        if base is None:
            base = obj.copy()
        rel = np.abs(obj - base) / np.maximum(np.abs(base), 1.0)
        print(f"{str(v):60s} pdhg {min(tms):7.1f} ms  iters mean {ist[:, 1].mean():7.1f}  optimal "
              f"{(ist[:, 0] == 0).sum()}/{len(ist)}  max obj diff vs first {rel.max():.1e}", flush=True)


if __name__ == "__main__":
    main()

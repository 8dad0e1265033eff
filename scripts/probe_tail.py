"""Launch tails of the bench's seeded sweep (dev helper): per phase (seed / warm) the PDHG time, the window-iterations
and the throughput; then the warm phase again with its windows reordered longest-first by the seed partner's
iteration count (LPT order; stats scattered back).  Usage: python scripts/probe_tail.py [scenarios]"""
import functools
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "der-vet_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import scenarios  # noqa: E402
from dervet_hip.sweep import SeededSweep, WARM_OPTIONS, sub_batch, transfer_device  # noqa: E402


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    scen = range(S)
    solver = BatchSolver(0)
    P = scenarios.sweep_parameters(scen)
    sw = SeededSweep(functools.partial(scenarios.config4, spec=True), scen, P["E"], stride=32,
                     features=scenarios.sweep_features(P))
    dev = sw.to_device(solver, "cuda:0")
    ns, cnt = sw.n_seed, dev.count
    o0 = solver.options()
    out = {}
    for rep in range(2):
        solver.set_options(warm_start=0)
        solver.solve_packed(sub_batch(dev, 0, ns))
        seed_ms = solver.timing()["pdhg_ms"]
        transfer_device(solver, sw.transfers, dev, sw.pairs)
        solver.set_options(warm_start=1, **WARM_OPTIONS)
        solver.solve_packed(sub_batch(dev, ns, cnt))
        warm_ms = solver.timing()["pdhg_ms"]
        solver.set_options(**{k: getattr(o0, k) for k in WARM_OPTIONS}, warm_start=o0.warm_start)
        it = dev.istats[:, 1].cpu().numpy().astype(np.int64)
        out[f"rep{rep}"] = dict(seed_ms=round(seed_ms, 2), warm_ms=round(warm_ms, 2),
                                seed_witer=int(it[:ns].sum()), warm_witer=int(it[ns:].sum()),
                                seed_ns_per_witer=round(seed_ms * 1e6 / it[:ns].sum(), 4),
                                warm_ns_per_witer=round(warm_ms * 1e6 / it[ns:].sum(), 4),
                                seed_iters_max=int(it[:ns].max()), warm_iters_max=int(it[ns:].max()))
    np.save("gpurun_out/tail_iters.npy", it)
    np.save("gpurun_out/tail_pairs.npy", sw.pairs)
    print("RESULT " + json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

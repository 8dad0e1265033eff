"""Seeded-sweep study (dev helper): config-4 windows solved cold vs with the two-phase seeded schedule
(dervet_hip/sweep.py) for several seed strides.  Prints kernel times, mean iterations per phase and the
largest objective difference against the cold solve.

Usage: python scripts/seeded_study.py <scenarios> <stride> [<stride> ...]
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "der-vet_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402
from dervet_hip.sweep import SeededSweep  # noqa: E402


def main():
    S = int(sys.argv[1])
    strides = [int(v) for v in sys.argv[2:]] or [8]
    ids = np.arange(S)
    keys = scenarios.sweep_parameters(ids)["E"]
    s = BatchSolver(0)
    groups = scenarios.config4(ids)
    cold_tags = [t for g in groups for t in g.tags]
    pb = builder.pack_groups(groups)
    del groups
    dev = pb.to_torch("cuda:0").alloc_outputs()
    s.solve_packed(dev)
    t = time.perf_counter()
    s.solve_packed(dev)
    cold_wall = time.perf_counter() - t
    tm = s.timing()
    ist = dev.istats.cpu().numpy()
    st = dev.stats.cpu().numpy()
    cold = {tg: (st[k, 0], ist[k, 1], ist[k, 0]) for k, tg in enumerate(cold_tags)}
    print(f"cold: wall {cold_wall * 1e3:.1f} ms  setup {tm['setup_ms']:.1f}  pdhg {tm['pdhg_ms']:.1f}  "
          f"iters mean {ist[:, 1].mean():.1f}", flush=True)
    del dev
    P = scenarios.sweep_parameters(ids)
    feats = {
        "E": None,
        "E/load,dur,rte,pv/load,dem/price": np.stack([np.log(P["E"] / P["load_scale"]), P["duration"], P["rte"],
                                                      P["pv_rated"] / P["load_scale"],
                                                      P["demand"] / P["price_scale"]], 1),
        "E/load,dur,pv/load": np.stack([np.log(P["E"] / P["load_scale"]), P["duration"],
                                        P["pv_rated"] / P["load_scale"]], 1),
        "E/load,dur,pv/load,rte": np.stack([np.log(P["E"] / P["load_scale"]), P["duration"],
                                            P["pv_rated"] / P["load_scale"], P["rte"]], 1),
        "E/load,pv/load": np.stack([np.log(P["E"] / P["load_scale"]), P["pv_rated"] / P["load_scale"]], 1),
    }
    if os.environ.get("FEATS"):
        feats = {k: v for k, v in feats.items() if k in os.environ["FEATS"].split(";")}
    for stride, (fname, fv) in [(st, kv) for st in strides for kv in feats.items()]:
        print(f"features: {fname}", flush=True)
        sw = SeededSweep(scenarios.config4, ids, keys, stride=stride, features=fv,
                         cover=bool(int(os.environ.get("COVER", "0"))))
        d2 = sw.packed.to_torch("cuda:0").alloc_outputs()
        sw.solve(s, d2)
        torch.cuda.synchronize()
        t = time.perf_counter()
        tm2, paths = sw.solve(s, d2)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t
        ist2 = d2.istats.cpu().numpy()
        st2 = d2.stats.cpu().numpy()
        rel = np.array([abs(st2[k, 0] - cold[tg][0]) / max(abs(cold[tg][0]), 1.0) for k, tg in enumerate(sw.tags)])
        ns = sw.n_seed
        print(f"stride {stride:3d}: wall {wall * 1e3:.1f} ms  setup {tm2['setup_ms']:.1f}  pdhg {tm2['pdhg_ms']:.1f}"
              f"  iters seeds {ist2[:ns, 1].mean():.1f} rest {ist2[ns:, 1].mean():.1f} all {ist2[:, 1].mean():.1f}"
              f"  optimal {(ist2[:, 0] == 0).sum()}/{len(ist2)}  max obj rel diff vs cold {rel.max():.1e}  "
              f"paths {paths}", flush=True)
        del d2


if __name__ == "__main__":
    main()

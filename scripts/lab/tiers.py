"""Lab (dev study): seeded schedules with more than one seed tier, total window-iterations on host cores.

Two tiers (bench.py's schedule): 1 in s1 scenarios (battery-energy order) solved cold, the rest warm from the
inverse-distance blend of their 4 nearest seeds.  Three tiers: 1 in s1 cold; then 1 in s2 (s2 < s1, the tier-1
scenarios excluded) warm from the tier-1 seeds; then the rest warm from the 4 nearest of tier 1 and tier 2 together.
Usage: python scripts/lab/tiers.py <scenarios> <s1>:<s2> ...   (s2 = 0: two tiers)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np  # noqa: E402
from lab import Lab, builder, scenarios, transfer  # noqa: E402

from dervet_hip.sweep import seed_partners, standardise  # noqa: E402

S = int(sys.argv[1])
groups = scenarios.config4(range(S))
wins = [[lp for lp in builder.group_window_lps(g)] for g in groups]  # [window id][scenario]
P = scenarios.sweep_parameters(range(S))
f = standardise(scenarios.sweep_features(P), S)
order = np.argsort(P["E"], kind="stable")
lab = Lab()
cold_cache = {}


def pick_every(cands, stride):
    """every stride-th of the candidate scenarios in battery-energy order (starting at stride // 2)"""
    c = [s for s in order if s in cands]
    return np.array(c[stride // 2::stride], np.int64)


def solve_cold(ids):
    lps = [w[s] for w in wins for s in ids]
    r = lab.solve(lps, check_every=32, kkt_every=1)
    sol = {(wi, s): (r["x"][wi * len(ids) + i], r["y"][wi * len(ids) + i]) for wi in range(len(wins))
           for i, s in enumerate(ids)}
    return int(r["iters"].sum()), sol


def solve_warm(ids, known):
    ks = np.array(sorted({s for (_, s) in known}), np.int64)
    idx, wgt = seed_partners(f[ids], f[ks], 4)
    lps, starts = [], []
    for wi, w in enumerate(wins):
        for i, s in enumerate(ids):
            a = [transfer(w[s], w[ks[p]], *known[(wi, int(ks[p]))]) for p in idx[i]]
            starts.append((sum(q * aa[0] for q, aa in zip(wgt[i], a)), sum(q * aa[1] for q, aa in zip(wgt[i], a))))
            lps.append(w[s])
    r = lab.solve(lps, starts, check_every=64, kkt_every=1, warm_start=1)
    sol = {(wi, s): (r["x"][wi * len(ids) + i], r["y"][wi * len(ids) + i]) for wi in range(len(wins))
           for i, s in enumerate(ids)}
    return int(r["iters"].sum()), sol, r["iters"]


allids = set(range(S))
nwin = S * len(wins)
for spec in sys.argv[2:]:
    s1, s2 = (int(v) for v in spec.split(":"))
    t1 = pick_every(allids, s1)
    it1, sol = solve_cold(t1)
    rest = allids - set(t1.tolist())
    line = f"s1 {s1:3d} s2 {s2:3d}: tier1 {len(t1):4d} cold {it1 / (len(t1) * len(wins)):7.1f}"
    total = it1
    if s2 > 0:
        t2 = pick_every(rest, s2)
        it2, sol2, _ = solve_warm(t2, sol)
        sol.update(sol2)
        rest = rest - set(t2.tolist())
        total += it2
        line += f" | tier2 {len(t2):4d} warm {it2 / (len(t2) * len(wins)):7.1f}"
    t3 = np.array(sorted(rest), np.int64)
    it3, _, its = solve_warm(t3, sol)
    total += it3
    line += (f" | rest {len(t3):4d} warm {it3 / (len(t3) * len(wins)):7.1f} (p99 {np.percentile(its, 99):.0f}) | "
             f"all {total / nwin:7.1f} iterations per window")
    print(line, flush=True)

"""Per-window iteration counts of bench.py's seeded config-4 sweep (device-built), for scheduling studies:
gpurun_out/iters.npz with iters / status per window (packed order), n_seed, and each warm window's seed index."""
import functools
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "der-vet_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import scenarios  # noqa: E402
from dervet_hip.sweep import SeededSweep  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
ids = range(S)
P = scenarios.sweep_parameters(ids)
s = BatchSolver(0)
sw = SeededSweep(functools.partial(scenarios.config4, spec=True), ids, P["E"], stride=32,
                 features=scenarios.sweep_features(P))
dev = sw.to_device(s, "cuda:0")
tm, _ = sw.solve(s, dev)
torch.cuda.synchronize()
tm2, _ = sw.solve(s, dev)
ist = dev.istats.cpu().numpy()
# warm window -> packed index of its seed window
seed_of = np.full(len(ist), -1, np.int64)
for t in sw.transfers:
    rows = np.arange(t.g_rest)
    base_r = t.on_rest
    # windows of this rest group are contiguous in packed order; find the first via desc offsets
    k0 = int(np.searchsorted(sw.desc[:, 6], t.on_rest))
    s0 = int(np.searchsorted(sw.desc[:, 6], t.on_seed))
    seed_of[k0:k0 + t.g_rest] = s0 + t.local
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "iters.npz"), iters=ist[:, 1], status=ist[:, 0], n_seed=sw.n_seed,
         seed_of=seed_of, T=sw.desc[:, 2] - 1)
print("timing", tm2)

#!/usr/bin/env python3
"""Dev probe: where one band-kernel iteration's time goes, per wave.  Needs the probe build
(python -c "from dervet_hip.build import build_variant; build_variant('scripts/_variants/lib_probe.so', ['-DDVH_BAND_PROBE=1'])")
loaded with DVH_LIB=scripts/_variants/lib_probe.so.  Every window runs the same fixed number of iterations (eps 1e-14,
max_iters N); each wave's shader-clock cycles per iteration are split into the primal half-step, the wait at the first
barrier, the dual half-step, the wait at the second barrier, and the checks (csrc/dvh_band.hip DVH_BAND_PROBE).
Usage (GPU box): DVH_LIB=... python scripts/probe_band_latency.py [scenarios] [iters] [config4 | config5]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "der-vet_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
N = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
CFG = sys.argv[3] if len(sys.argv) > 3 else "config4"
groups = scenarios.config4(range(S)) if CFG == "config4" else scenarios.config5(range(S), years=1)
pb = builder.pack_groups(groups)
dev = pb.to_torch("cuda:0").alloc_outputs()
s = BatchSolver(0, eps=1e-14, eps_obj=0.0, max_iters=N)
for r in range(2):
    torch.cuda.synchronize()
    t = time.perf_counter()
    s.solve_packed(dev)
    torch.cuda.synchronize()
    el = time.perf_counter() - t
it = dev.istats[:, 1].double().cpu().numpy()
x = dev.x.cpu().numpy()
desc = np.asarray(pb.desc)
NWV = 4 if CFG == "config4" else 12
P = np.stack([x[int(d[6]):int(d[6]) + 6 * NWV] for d in desc]).reshape(-1, NWV, 6)  # [window, wave, segment + hw id]
hw = P[:, :, 5].astype(np.int64)
P = P[:, :, :5]
per_it = P / it[:, None, None]
names = ["primal", "wait1", "dual", "wait2", "checks"]
print(f"windows {pb.count} iters {int(it.mean())}: {el * 1e3:.1f} ms, {el / (pb.count * it.mean()) * 512 * 1e6:.3f} us "
      f"per window-iteration per slot ({s.timing()})")
simd = (hw >> 4) & 3
print("SIMD of wave w (rows: wave, cols: SIMD 0..3, windows):")
for w in range(NWV):
    print(f"  wave {w}: " + " ".join(f"{int((simd[:, w] == q).sum()):6d}" for q in range(4)))
print("wave 0's SIMD minus wave w's (mod 4), all windows:", np.bincount(((simd[:, 1] - simd[:, 0]) % 4), minlength=4))
for w in range(NWV):
    m = per_it[:, w, :].mean(0)
    print(f"wave {w}: " + "  ".join(f"{n} {v:7.1f}" for n, v in zip(names, m)) + f"  total {m.sum():7.1f} cycles/iter")

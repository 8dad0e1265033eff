"""Raw per-iteration cost of the PDHG kernels: fixed iteration counts, no convergence (dev helper)."""
import sys, time, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "der-vet_amd"))
import numpy as np, torch
from dervet_hip import BatchSolver, _lib
from dervet_hip.lp import scenarios, builder
S = int(sys.argv[1]) if len(sys.argv) > 1 else 256
if len(sys.argv) > 2:  # A/B: load an alternative build (scripts/build_variants.sh)
    _lib.LIB_PATH = sys.argv[2]
ONLY = sys.argv[3].split(",") if len(sys.argv) > 3 else None
gs = scenarios.config4(range(S)); pb = builder.pack_groups(gs)
dev = pb.to_torch("cuda:0").alloc_outputs()
s = BatchSolver(0)
nwin = pb.count
for label, kw in [("nochecks", dict(check_every=100000, kkt_every=1)), ("chk16", dict(check_every=16, kkt_every=1000000)),
                  ("chk16kkt4", dict(check_every=16, kkt_every=4)), ("chk64kkt1", dict(check_every=64, kkt_every=1)),
                  ("chk64", dict(check_every=64, kkt_every=1000000)), ("chk64kkt2", dict(check_every=64, kkt_every=2))]:
    if ONLY and label not in ONLY:
        continue
    for iters in (1024, 4096):
        s.set_options(eps=1e-30, max_iters=iters, **kw)
        s.solve_packed(dev); torch.cuda.synchronize()
        tm = s.timing()
        per = tm["pdhg_ms"] * 1e3 / (nwin / 256.0) / iters
        print(f"{label:10s} iters={iters}: pdhg {tm['pdhg_ms']:.1f} ms  -> {per:.3f} us/iter/window-slot  setup {tm['setup_ms']:.1f}", flush=True)

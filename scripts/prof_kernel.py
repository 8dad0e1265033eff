"""Profile helper: one solve of a config-4 sample (run under rocprofv3)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "der-vet_amd"))
import numpy as np, torch
from dervet_hip import BatchSolver, _lib
if os.environ.get("DVH_AB_LIB"):  # A/B builds (dev helper)
    _lib.LIB_PATH = os.path.abspath(os.environ["DVH_AB_LIB"])
from dervet_hip.lp import scenarios, builder
S = int(sys.argv[1]) if len(sys.argv) > 1 else 256
gs = scenarios.config4(range(S)); pb = builder.pack_groups(gs)
dev = pb.to_torch("cuda:0").alloc_outputs()
s = BatchSolver(0)
s.solve_packed(dev)
torch.cuda.synchronize()
ist = dev.istats.cpu().numpy()
print("windows", pb.count, "iters sum", int(ist[:, 1].sum()), "mean", ist[:, 1].mean(), "pct", np.percentile(ist[:, 1], [50, 90, 99, 100]), s.timing())
np.save(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpurun_out", "iters_S%d.npy" % S), ist)

"""Quick throughput / correctness probe on the GPU box (development helper)."""
import sys, time, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "der-vet_amd"))
import numpy as np, torch
from dervet_hip import BatchSolver
from dervet_hip.lp import scenarios, builder
S = int(sys.argv[1]) if len(sys.argv) > 1 else 512
paths = sys.argv[2].split(",") if len(sys.argv) > 2 else ["ell", "generic"]
t = time.time(); gs = scenarios.config4(range(S)); pb = builder.pack_groups(gs); print("build", time.time() - t, flush=True)
dev = pb.to_torch("cuda:0").alloc_outputs()
s = BatchSolver(0)
d = pb.desc
n, m, nnz = d[:, 0], d[:, 1], d[:, 3]
B = 24 * nnz + 4 * (n + m) + 72 * n + 48 * m
res = {}
for path in paths:
    s.set_kernel_path(path == "generic")
    for rep in range(2):
        torch.cuda.synchronize(); t = time.time(); s.solve_packed(dev); torch.cuda.synchronize(); el = time.time() - t
        ist = dev.istats.cpu().numpy(); st = dev.stats.cpu().numpy()
        tm = s.timing()
        print(f"{path} rep{rep}: {pb.count} windows in {el:.3f}s -> {pb.count/el:.0f} win/s; timing {tm}; {s.kernel_stats()}", flush=True)
        print("  status counts", np.bincount(ist[:, 0] + 1, minlength=6), "iters mean", ist[:, 1].mean(), "max", ist[:, 1].max())
        it_tot = ist[:, 1].sum()
        print(f"  us/iter/window-slot (256 CUs): {tm['pdhg_ms']*1e3*256/it_tot:.3f}   alg TB/s {((B*ist[:,1]).sum())/(tm['pdhg_ms']*1e-3)/1e12:.2f}")
    res[path] = (dev.x.cpu().numpy().copy(), st.copy(), ist.copy())
if len(res) == 2:
    a, b = res["ell"], res["generic"]
    print("ell vs generic: max |obj diff| rel", np.max(np.abs(a[1][:, 0] - b[1][:, 0]) / np.abs(b[1][:, 0])),
          "iters equal frac", np.mean(a[2][:, 1] == b[2][:, 1]))

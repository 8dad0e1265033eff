"""Warm-start study (dev helper): how many PDHG iterations does a config-4 window need when started from the
solution of a NEIGHBOURING scenario's window of the same month, instead of from zero?

Usage: python scripts/warm_study.py <scenarios>
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "der-vet_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402


def runs(desc):
    """Maximal runs of consecutive windows with identical (n, m) -> [(a, b, n, m)]."""
    out, a = [], 0
    for k in range(1, len(desc) + 1):
        if k == len(desc) or desc[k, 0] != desc[a, 0] or desc[k, 1] != desc[a, 1]:
            out.append((a, k, int(desc[a, 0]), int(desc[a, 1])))
            a = k
    return out


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    pb = builder.pack_groups(scenarios.config4(range(S)))
    dev = pb.to_torch("cuda:0").alloc_outputs()
    s = BatchSolver(0)
    s.solve_packed(dev)
    torch.cuda.synchronize()
    cold_ms = s.timing()["pdhg_ms"]
    cold_it = dev.istats[:, 1].cpu().numpy().copy()
    cold_obj = dev.stats[:, 0].cpu().numpy().copy()
    x0, y0 = dev.x.clone(), dev.y.clone()
    u = torch.as_tensor(pb.u, device="cuda:0")
    desc = np.asarray(pb.desc)
    c = torch.as_tensor(pb.c, device="cuda:0")
    for label in ("raw", "scaled", "scaled+duals", "nearestE+scaled", "nearestE+scaled+duals"):
        xw, yw = torch.zeros_like(x0), torch.zeros_like(y0)
        for a, b, n, m in runs(desc):
            G = b - a
            on, om = int(desc[a, 6]), int(desc[a, 7])
            U = u[on:on + G * n].view(G, n)
            C = c[on:on + G * n].view(G, n)
            T = int(desc[a, 2]) - 1
            if label.startswith("nearestE"):  # pair with the neighbour in battery-energy order
                order = torch.argsort(U[:, 2 * T])
                pos = torch.empty_like(order)
                pos[order] = torch.arange(G, device=order.device)
                nb = torch.where(pos % 2 == 0, torch.clamp(pos + 1, max=G - 1), pos - 1)
                perm = order[nb]
            else:
                perm = torch.as_tensor(np.arange(G) ^ 1, device="cuda:0").clamp(max=G - 1)
            X = x0[on:on + G * n].view(G, n)
            Xw = X[perm].clone()
            if "scaled" in label:  # bounded columns (ch, dis, ene) by the ratio of their upper bounds
                r = torch.where(torch.isfinite(U) & torch.isfinite(U[perm]) & (U[perm] > 0), U / U[perm],
                                torch.ones_like(U))
                Xw = Xw * r
            xw[on:on + G * n] = Xw.reshape(-1)
            Yw = y0[om:om + G * m].view(G, m)[perm].clone()
            if "duals" in label and n > 3 * T:  # DCM duals sum to the demand charge; SOE duals ~ energy price
                cd = C[:, 3 * T:3 * T + 1] / C[perm][:, 3 * T:3 * T + 1].clamp(min=1e-12)
                Yw[:, T + 1:] *= cd
                cp = C[:, :T].abs().mean(1, keepdim=True) / C[perm][:, :T].abs().mean(1, keepdim=True).clamp(min=1e-12)
                Yw[:, :T + 1] *= cp
            yw[om:om + G * m] = Yw.reshape(-1)
        dev.x.copy_(xw)
        dev.y.copy_(yw)
        s.set_options(warm_start=1)
        s.solve_packed(dev)
        torch.cuda.synchronize()
        ms = s.timing()["pdhg_ms"]
        it = dev.istats[:, 1].cpu().numpy()
        st = dev.istats[:, 0].cpu().numpy()
        obj = dev.stats[:, 0].cpu().numpy()
        rel = np.abs(obj - cold_obj) / np.maximum(np.abs(cold_obj), 1e-12)
        print(f"{label:7s} warm: pdhg {ms:7.1f} ms (cold {cold_ms:.1f})  iters mean {it.mean():7.1f} (cold "
              f"{cold_it.mean():.1f})  p99 {np.percentile(it, 99):.0f} (cold {np.percentile(cold_it, 99):.0f})  "
              f"optimal {(st == 0).sum()}/{len(st)}  obj rel diff vs cold max {rel.max():.1e}  "
              f"paths {s.kernel_stats()}", flush=True)
        s.set_options(warm_start=0)


if __name__ == "__main__":
    main()

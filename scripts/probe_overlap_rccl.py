#!/usr/bin/env python3
"""Dev probe: the library's own RCCL all-gather (dvh_gather_results, a world-size-1 communicator on the one-GPU box)
beside the persistent band grid, in bench.py's order -- the gather issued on its stream first, the next solve launched
right after -- against each alone.  The rows are bench-sized (GIB GiB of float64).  A world-size-1 all-gather moves
the rows once through RCCL's own kernel on the device (no xGMI): what it shows is whether RCCL's kernel gets slots
beside a grid that claims every resident workgroup slot (2 per CU), not the xGMI rate.
Usage (GPU box): python scripts/probe_overlap_rccl.py [scenarios] [gib]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "der-vet_amd")]
import torch  # noqa: E402
from dervet_hip import BatchSolver, parallel  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
GIB = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
pb = builder.pack_groups(scenarios.config4(range(S)))
dev = pb.to_torch("cuda:0").alloc_outputs()
solver = BatchSolver(0)
lg = parallel.LibraryGather(solver, 0, 1, solver.comm_unique_id())
cols = 2248
rows = torch.ones((int(GIB * (1 << 30)) // (8 * cols), cols), dtype=torch.float64, device="cuda:0")
out = torch.empty_like(rows)
s1 = torch.cuda.Stream()


def ev():
    return torch.cuda.Event(enable_timing=True)


def gather_on(e0, e1):
    e0.record(lg.stream)
    solver.gather_results(rows, out, lg.stream)
    e1.record(lg.stream)


def alone_gather():
    e0, e1 = ev(), ev()
    gather_on(e0, e1)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def alone_band():
    e0, e1 = ev(), ev()
    e0.record(s1)
    solver.solve_packed(dev, stream=s1.cuda_stream)
    e1.record(s1)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def together():
    b0, b1, c0, c1 = ev(), ev(), ev(), ev()
    torch.cuda.synchronize()
    gather_on(c0, c1)  # bench.py's order: the gather first ...
    b0.record(s1)      # ... then the next step's solve
    solver.solve_packed(dev, stream=s1.cuda_stream, sync=False)
    b1.record(s1)
    torch.cuda.synchronize()
    return b0.elapsed_time(b1), b0.elapsed_time(c1), c0.elapsed_time(c1)


alone_gather(), alone_band()
g = min(alone_gather() for _ in range(3))
b = min(alone_band() for _ in range(3))
print(f"rows {rows.numel() * 8 / 2**30:.2f} GiB; library all-gather alone {g:.2f} ms; band pass alone {b:.2f} ms", flush=True)
for r in range(3):
    bt, cend, cspan = together()
    print(f"together: band {bt:.2f} ms ({100 * (bt / b - 1):+.1f} %), gather ended {cend:.2f} ms after the band pass "
          f"started (span {cspan:.2f} ms)", flush=True)
assert torch.equal(out, rows)
print("gathered rows equal the input (world size 1)")

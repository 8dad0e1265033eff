#!/usr/bin/env python3
"""Dev probe: can a transfer run beside the persistent band grid, which claims every resident
workgroup slot (2 per CU at 256 VGPRs)?  RCCL's all-gather runs as kernels on its own stream; two ranks cannot share
this one GPU, so a 2 GiB device copy on a second stream stands in for it: a shader copy (torch elementwise kernel) and
torch's copy_ (hipMemcpyAsync D2D).  The band solve (a seeded-sweep-sized batch of config-4 windows, every window
warm-free cold) runs on stream S1 from one host thread; the copy is issued on S2 from another thread `delay` ms after
the solve was started.  Reported from HIP events: the copy alone, the band pass alone, and with both -- when the
copy ended relative to the band pass (its span within the band pass = it overlapped; ending after = queued behind).
DVH_BAND_RESERVE (if the library honours it) leaves that many CUs' slots to other kernels.
Usage (GPU box): python scripts/probe_overlap.py [scenarios] [gib]"""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "der-vet_amd")]
import torch  # noqa: E402
from dervet_hip import BatchSolver  # noqa: E402
from dervet_hip.lp import builder, scenarios  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
GIB = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
pb = builder.pack_groups(scenarios.config4(range(S)))
dev = pb.to_torch("cuda:0").alloc_outputs()
solver = BatchSolver(0)
n = int(GIB * (1 << 30) // 8)
src = torch.ones(n, dtype=torch.float64, device="cuda:0")
dst = torch.empty_like(src)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def copy(kind):
    if kind == "shader":
        torch.mul(src, 1.0, out=dst)
    else:
        dst.copy_(src)


def ev():
    return torch.cuda.Event(enable_timing=True)


def alone_copy(kind):
    e0, e1 = ev(), ev()
    with torch.cuda.stream(s2):
        e0.record(s2)
        copy(kind)
        e1.record(s2)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def alone_band():
    e0, e1 = ev(), ev()
    e0.record(s1)
    solver.solve_packed(dev, stream=s1.cuda_stream)
    e1.record(s1)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def together(kind, delay_ms):
    b0, b1, c0, c1 = ev(), ev(), ev(), ev()
    torch.cuda.synchronize()
    if delay_ms < 0:  # bench.py's order: the gather enqueued first, the next solve launched right after (one thread)
        with torch.cuda.stream(s2):
            c0.record(s2)
            copy(kind)
            c1.record(s2)
        b0.record(s1)
        solver.solve_packed(dev, stream=s1.cuda_stream, sync=False)
        b1.record(s1)
        torch.cuda.synchronize()
        return b0.elapsed_time(b1), b0.elapsed_time(c0), b0.elapsed_time(c1), c0.elapsed_time(c1)

    def band():
        b0.record(s1)
        solver.solve_packed(dev, stream=s1.cuda_stream, sync=False)
        b1.record(s1)

    th = threading.Thread(target=band)
    th.start()
    time.sleep(delay_ms / 1e3)
    with torch.cuda.stream(s2):
        c0.record(s2)
        copy(kind)
        c1.record(s2)
    th.join()
    torch.cuda.synchronize()
    return b0.elapsed_time(b1), b0.elapsed_time(c0), b0.elapsed_time(c1), c0.elapsed_time(c1)


print(f"DVH_BAND_RESERVE={os.environ.get('DVH_BAND_RESERVE', '0')}")
for kind in ("shader", "copy_"):
    alone_copy(kind)
    ca = min(alone_copy(kind) for _ in range(3))
    alone_band()
    ba = min(alone_band() for _ in range(2))
    print(f"{kind}: copy alone {ca:.2f} ms ({GIB * (1 << 30) * 2 / ca / 1e6:.0f} GB/s r+w), band pass alone {ba:.2f} ms",
          flush=True)
    for delay in (-1.0, 0.0, 5.0, 20.0):
        bt, cs, ce, cd = together(kind, delay)
        verdict = "ran beside the grid" if cd < 4 * ca + 5.0 else "queued behind the grid's resident workgroups"
        when = "enqueued before the solve" if delay < 0 else f"issued {delay:4.1f} ms after the solve"
        print(f"  {when}: band {bt:.2f} ms (alone {ba:.2f}); copy recorded at {cs:.2f}, ended at {ce:.2f} ms after "
              f"band start, its own span {cd:.2f} ms -> {verdict}", flush=True)

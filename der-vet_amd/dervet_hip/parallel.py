"""Multi-GPU sharding of independent windows / scenarios (one process per GPU, torch.distributed).

The reference runs sensitivity cases serially (dervet/DERVET.py:75) and windows serially
(dervet/MicrogridScenario.py:310); every window LP is independent, so ranks take disjoint,
contiguous scenario ranges, solve with no inter-GPU traffic, and ONE all-gather (RCCL over xGMI with the
"nccl" backend, gloo in CPU tests) returns every window's result rows to every rank in global order.
"""
import numpy as np


def shard(total, world, rank):
    """Contiguous, balanced [start, stop) range of `total` units for `rank` (rank-stable, deterministic)."""
    base, extra = divmod(int(total), int(world))
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def weak_shard(per_rank, rank):
    """Weak scaling: every rank owns the same number of units; global ids rank*per_rank ..."""
    return rank * per_rank, (rank + 1) * per_rank


def gather_rows(rows, group=None):
    """All-gather a [k_r, w] float64 tensor of per-window result rows from every rank (k_r may differ);
    returns the concatenation in rank order (identical on every rank)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    k = torch.tensor([rows.shape[0]], dtype=torch.int64, device=rows.device)
    ks = [torch.zeros_like(k) for _ in range(world)]
    dist.all_gather(ks, k, group=group)
    kmax = int(max(int(v.item()) for v in ks))
    pad = torch.zeros((kmax, rows.shape[1]), dtype=rows.dtype, device=rows.device)
    pad[: rows.shape[0]] = rows
    outs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad, group=group)
    return torch.cat([o[: int(n.item())] for o, n in zip(outs, ks)], dim=0)


def result_rows(stats, istats):
    """Per-window result rows {obj, primal_res_rel, dual_res_rel, gap_rel, status, iters} (float64)."""
    import torch
    return torch.cat([stats.to(torch.float64), istats.to(torch.float64)], dim=1).contiguous()


def rows_to_numpy(rows):
    r = rows.detach().cpu().numpy()
    return dict(obj=r[:, 0], primal_res_rel=r[:, 1], dual_res_rel=r[:, 2], gap_rel=r[:, 3],
                status=r[:, 4].astype(np.int32), iters=r[:, 5].astype(np.int64))

"""N > 1 path on CPU: two gloo ranks shard the scenario sweep with dervet_hip.parallel and all-gather the
per-window result rows; the gathered rows equal a single-process run in global window order.

The per-window "solve" here is the oracle (HiGHS) standing in for the GPU kernel, because this container
has no GPU; the sharding, ordering and the gather are exactly the code bench.py runs over RCCL.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from dervet_hip import parallel


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rows_for(scenario_ids):
    """Result rows (obj, 0, 0, 0, status, iters) for the windows of the given scenarios, via HiGHS."""
    import scipy.sparse as sp
    from dervet_hip.lp import builder, scenarios
    from oracle import window_lp
    groups = scenarios.config4(scenario_ids)
    pb = builder.pack_groups(groups)
    rows = []
    for k in range(pb.count):
        lp = window_lp.from_packed_window(pb.window(k))
        r = window_lp.solve_highs(lp)
        rows.append([r["obj"], 0.0, 0.0, 0.0, float(r["status"]), 0.0])
    return torch.tensor(rows, dtype=torch.float64), pb.desc


def _worker(rank, world, port, total, out):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a, b = parallel.shard(total, world, rank)
    rows, _ = _rows_for(range(a, b))
    g = parallel.gather_rows(rows)
    if rank == 0:
        torch.save(g, out)
    dist.destroy_process_group()


def test_shard_ranges_cover_exactly_once():
    for total in (0, 1, 7, 10000):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                a, b = parallel.shard(total, world, r)
                seen += list(range(a, b))
            assert seen == list(range(total))
    assert parallel.weak_shard(10000, 3) == (30000, 40000)


@pytest.mark.timeout(300)
def test_two_rank_gloo_gather_matches_single_process(tmp_path):
    total = 3  # scenarios -> 36 windows, windows of a scenario split across ranks in rank order
    out = str(tmp_path / "g.pt")
    mp.spawn(_worker, args=(2, _free_port(), total, out), nprocs=2, join=True)
    g = torch.load(out, weights_only=True)
    # single-process order: shard 0 = scenario 0 (then 1 on rank 1 ...): rebuild per shard and concatenate
    ref = torch.cat([_rows_for(range(*parallel.shard(total, 2, r)))[0] for r in range(2)])
    assert g.shape == (36, 6)
    assert torch.equal(g, ref)
    assert (g[:, 4] == 0).all()

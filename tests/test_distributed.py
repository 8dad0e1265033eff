"""N > 1 path on CPU: two gloo ranks shard the scenario sweep with dervet_hip.parallel and all-gather the
per-window result rows (objective, residuals, status, iterations and the ch / dis / ene dispatch in a fixed
stride); the gathered rows equal a single-process run in global window order, bit for bit.

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


def _rows_for(scenario_ids, tmax=744, seeded=False):
    """Result rows (obj, 0, 0, 0, status, 0, scenario, window, ch, dis, ene padded to tmax) for the windows of the
    given scenarios, via HiGHS.  seeded: packed as bench.py's seeded sweep packs them (seed scenarios first)."""
    from dervet_hip.lp import builder, scenarios
    from dervet_hip.sweep import SeededSweep
    from oracle import window_lp
    if seeded:
        ids = list(scenario_ids)
        P = scenarios.sweep_parameters(ids)
        sw = SeededSweep(scenarios.config4, ids, P["E"], stride=2, features=scenarios.sweep_features(P))
        pb, tags = sw.packed, sw.tags
    else:
        groups = scenarios.config4(scenario_ids)
        pb, tags = builder.pack_groups(groups), [t for g in groups for t in g.tags]
    stats = torch.zeros((pb.count, 4), dtype=torch.float64)
    istats = torch.zeros((pb.count, 2), dtype=torch.int32)
    x = torch.zeros(len(pb.c), dtype=torch.float64)
    for k in range(pb.count):
        w = pb.window(k)
        r = window_lp.solve_highs(window_lp.from_packed_window(w))
        stats[k, 0] = r["obj"]
        istats[k, 0] = r["status"]
        on = int(pb.desc[k, 6])
        x[on:on + w["n"]] = torch.from_numpy(r["x"])
    return parallel.result_rows(stats, istats, x, pb.desc, tmax, tags=parallel.tag_array(tags)), pb


def _worker(rank, world, port, total, out, seeded=False):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a, b = parallel.shard(total, world, rank)
    rows, _ = _rows_for(range(a, b), seeded=seeded)
    counts = [12 * (lambda ab: ab[1] - ab[0])(parallel.shard(total, world, r)) for r in range(world)]
    g = parallel.gather_rows(rows, counts=counts if total % world == 0 else None)
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
    parts = [_rows_for(range(*parallel.shard(total, 2, r))) for r in range(2)]
    ref = torch.cat([p[0] for p in parts])
    C = parallel.RESULT_COLS
    assert g.shape == (36, C + 3 * 744)
    assert torch.equal(g, ref)
    assert (g[:, 4] == 0).all()
    # the dispatch columns are the windows' ch / dis / ene; every row names its (scenario, window)
    d = parallel.rows_to_numpy(g)
    o = parallel.by_tag(d)
    assert np.array_equal(o["scenario"], np.repeat(np.arange(3), 12)) and np.array_equal(o["window"], np.tile(np.arange(12), 3))
    pb = parts[0][1]
    w = pb.window(5)
    T = w["m_eq"] - 1
    assert np.array_equal(d["ch"][5, :T], ref.numpy()[5, C:C + T])
    assert np.all(d["ene"][5, T:] == 0.0) or T == 744


@pytest.mark.timeout(300)
def test_two_rank_gather_in_seeded_order_maps_back_by_tag(tmp_path):
    """bench.py's N > 1 path: each rank packs its shard seed-first (SeededSweep); the gathered rows, re-ordered by
    the (scenario, window) they carry, equal a single-process run's rows in (scenario, window) order -- no
    SeededSweep rebuild on the consumer's side."""
    total = 6
    out = str(tmp_path / "g.pt")
    mp.spawn(_worker, args=(2, _free_port(), total, out, True), nprocs=2, join=True)
    g = parallel.by_tag(parallel.rows_to_numpy(torch.load(out, weights_only=True)))
    ref = parallel.by_tag(parallel.rows_to_numpy(_rows_for(range(total))[0]))
    assert np.array_equal(g["scenario"], np.repeat(np.arange(total), 12))
    for k in ("status", "window", "ch", "dis", "ene"):
        assert np.array_equal(g[k], ref[k]), k
    # the objective constant c0 is a numpy row sum whose last bit depends on the group's size (a seed group of one
    # scenario vs all of them): objectives agree to rounding, the dispatch bit for bit
    assert np.allclose(g["obj"], ref["obj"], rtol=1e-14, atol=0.0)


def test_weighted_shard_balances_cost_and_covers_once():
    from dervet_hip.lp import builder, scenarios
    w = np.array([1.0] * 50 + [40.0] + [1.0] * 49)
    for world in (1, 2, 3, 4, 8):
        seen, loads = [], []
        for r in range(world):
            a, b = parallel.shard_weighted(w, world, r)
            seen += list(range(a, b))
            loads.append(w[a:b].sum())
        assert seen == list(range(len(w)))
        assert max(loads) <= w.sum() / world + w.max()
    pb = builder.pack_groups(scenarios.config4([0]))
    c = parallel.window_cost(pb.desc)
    assert np.all(c == 1.0)
    big = pb.desc.copy()
    big[0, 0] = 315360
    big[0, 3] = 735840
    assert parallel.window_cost(big)[0] == pytest.approx(735840 / 5208)


def _bench(args, env=None, timeout=240):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, env=e, capture_output=True,
                          text=True, timeout=timeout)


@pytest.mark.timeout(300)
def test_bench_gpus_2_launches_two_ranks_itself():
    """`bench.py --gpus 2` with no outside launcher starts 2 rank processes (gloo here, RCCL on the GPU box), shards
    the scenarios, gathers every rank's tagged rows and prints ONE line from rank 0 with n_gpus 2."""
    import json
    r = _bench(["--gpus", "2", "--dry-run", "--scenarios", "3", "--steps", "2", "--warmup", "1"])
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and len(set(j["rank_pids"])) == 2
    assert j["gather"]["per_rank_windows"] == [36, 36] and j["gather"]["rows"] == 72
    assert j["gather"]["scenarios"] == list(range(6))  # rank r owns scenarios 3r .. 3r + 2 (weak scaling)


@pytest.mark.timeout(300)
def test_bench_launcher_failure_and_world_mismatch():
    r = _bench(["--gpus", "2", "--dry-run", "--scenarios", "2"], env={"DVH_DRY_RUN_FAIL_RANK": "1"}, timeout=120)
    assert r.returncode != 0 and "rank exit statuses" in r.stderr  # rank 0 is ended, not left waiting
    r = _bench(["--gpus", "1", "--dry-run"], env={"WORLD_SIZE": "2", "RANK": "0"}, timeout=120)
    assert r.returncode != 0 and "refusing" in r.stderr
    r = _bench(["--gpus", "1", "--dry-run", "--scenarios", "2", "--steps", "1"])
    assert r.returncode == 0 and '"n_gpus": 1' in r.stdout


def test_untagged_rows_stay_distinct_across_ranks():
    tags = ["a", "b", "c"]
    t0 = parallel.tag_array(tags, offset=0)
    t1 = parallel.tag_array(tags, offset=3)
    keys = {tuple(r) for r in np.concatenate([t0, t1])}
    assert len(keys) == 6
    st = torch.zeros((3, 4), dtype=torch.float64)
    ist = torch.zeros((3, 2), dtype=torch.int32)
    rows = parallel.result_rows(st, ist, offset=3)
    assert rows[:, 7].tolist() == [3.0, 4.0, 5.0]


def _async_worker(rank, world, port, out):
    """bench.py --overlap-gather: each step's rows start their all-gather at once (async_op) and are collected at the
    next step, while that step's rows are being made; the last gather is drained before the end."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    got, pending = [], None
    for step in range(3):
        rows = torch.full((5, parallel.RESULT_COLS + 6), float(100 * step + rank), dtype=torch.float64)
        rows[:, 0] = torch.arange(5, dtype=torch.float64) + 10 * rank
        if pending is not None:
            got.append(pending.wait())
        pending = parallel.gather_rows(rows, counts=[5] * world, async_op=True)
        del rows  # the pending gather keeps its input alive
    got.append(pending.wait())
    if rank == 0:
        torch.save(torch.stack(got), out)
    with pytest.raises(ValueError):
        parallel.gather_rows(torch.zeros((4, 3), dtype=torch.float64), counts=[4, 5], async_op=True)
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_two_rank_async_gather_overlapping_the_next_step(tmp_path):
    out = str(tmp_path / "a.pt")
    mp.spawn(_async_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    g = torch.load(out, weights_only=True)
    assert g.shape == (3, 10, parallel.RESULT_COLS + 6)
    for step in range(3):
        assert torch.equal(g[step, :5, 1], torch.full((5,), 100.0 * step, dtype=torch.float64))
        assert torch.equal(g[step, 5:, 1], torch.full((5,), 100.0 * step + 1, dtype=torch.float64))
        assert torch.equal(g[step, :, 0], torch.cat([torch.arange(5.0), torch.arange(5.0) + 10]).double())


def _agree_worker(rank, world, port, fail_rank, out):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def make():  # stands in for LibraryGather.from_torch: fails on fail_rank (RCCL not openable there)
        if rank == fail_rank:
            raise RuntimeError("RCCL could not be opened (test)")
        return ("library gather of rank", rank)

    lib, err = parallel.agreed_library_gather(None, device="cpu", make=make)
    torch.save({"lib": lib, "err": err}, f"{out}.{rank}")
    dist.destroy_process_group()


@pytest.mark.parametrize("fail_rank", [-1, 0, 1])
def test_ranks_agree_on_the_library_gather(tmp_path, fail_rank):
    """bench.py's N > 1 all-gather: the library's communicator on every rank or on none -- a rank that cannot form it
    makes every rank fall back to torch.distributed's all-gather (never a mixed pair of collectives)."""
    out = str(tmp_path / "agree")
    mp.spawn(_agree_worker, args=(2, _free_port(), fail_rank, out), nprocs=2, join=True)
    got = [torch.load(f"{out}.{r}", weights_only=False) for r in range(2)]
    if fail_rank < 0:
        assert [g["lib"] for g in got] == [("library gather of rank", 0), ("library gather of rank", 1)]
        assert all(g["err"] is None for g in got)
    else:
        assert all(g["lib"] is None for g in got)
        assert "RCCL could not be opened" in got[fail_rank]["err"]
        assert "another rank" in got[1 - fail_rank]["err"]

"""Multi-GPU sharding of independent windows / scenarios (one process per GPU, torch.distributed).

The reference runs sensitivity cases serially (dervet/DERVET.py:75) and windows serially
(dervet/MicrogridScenario.py:310); every window LP is independent, so ranks take disjoint,
contiguous ranges of windows, solve with no inter-GPU traffic, and ONE all-gather (RCCL over xGMI with the "nccl"
backend, gloo in CPU tests) returns every window's result row -- objective, residuals, status, iterations and the
dispatch time series (ch, dis, ene, padded to a fixed stride) -- to every rank in global order, where the
ServiceAggregator / POI results consume them.

Partitions:
  * ``weak_shard``: every rank owns the same number of scenarios (the bench's weak scaling);
  * ``shard``: a fixed total split into near-equal contiguous counts;
  * ``shard_weighted``: a fixed batch split into contiguous ranges of near-equal estimated cost
    (``window_cost``: on-chip windows cost one workgroup each, grid-wide windows in proportion to their nonzeros),
    for heterogeneous batches (strong scaling).
"""
import numpy as np

# obj, primal_res_rel, dual_res_rel, gap_rel, status, iters, scenario, window: every gathered row names its own
# (scenario, window), so a consumer maps rows without rebuilding the packing order (a seeded sweep packs seed
# scenarios first)
RESULT_COLS = 8


def shard(total, world, rank):
    """Contiguous, balanced [start, stop) range of `total` units for `rank` (rank-stable, deterministic)."""
    base, extra = divmod(int(total), int(world))
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def weak_shard(per_rank, rank):
    """Weak scaling: every rank owns the same number of units; global ids rank*per_rank ..."""
    return rank * per_rank, (rank + 1) * per_rank


def window_cost(desc, small_max=4096, ref_nnz=5208):
    """Estimated relative solve cost per window from its descriptor rows {n, m, m_eq, nnz, ...}: windows the
    on-chip kernels take (n, m <= small_max) cost one workgroup each (per-iteration time does not depend on their
    size); larger windows run grid-wide, in proportion to their nonzeros (ref_nnz: a monthly battery + DCM window)."""
    d = np.asarray(desc)
    big = (d[:, 0] > small_max) | (d[:, 1] > small_max)
    return np.where(big, np.maximum(d[:, 3] / float(ref_nnz), 1.0), 1.0)


def shard_weighted(weights, world, rank):
    """Contiguous [start, stop) of the units whose cumulative weight falls in rank's equal share (deterministic;
    every unit assigned exactly once, ranges in rank order)."""
    w = np.asarray(weights, np.float64)
    if len(w) == 0:
        return 0, 0
    cum = np.concatenate([[0.0], np.cumsum(w)])
    total = cum[-1]
    # boundary r: first unit whose cumulative weight (up to its midpoint) reaches r / world of the total
    mids = cum[:-1] + 0.5 * w
    bounds = [0] + [int(np.searchsorted(mids, total * r / world)) for r in range(1, world)] + [len(w)]
    return bounds[rank], bounds[rank + 1]


def dispatch_runs(desc):
    """Runs of consecutive windows with the same n and contiguous x offsets: (k0, k1, off_n of k0, n, T) with
    T = m_eq - 1 the steps of a battery window (its dispatch = x[:3T] = ch, dis, ene)."""
    d = np.asarray(desc)
    runs = []
    k = 0
    while k < len(d):
        k1 = k + 1
        while k1 < len(d) and d[k1, 0] == d[k, 0] and d[k1, 2] == d[k, 2] and d[k1, 6] == d[k1 - 1, 6] + d[k, 0]:
            k1 += 1
        runs.append((k, k1, int(d[k, 6]), int(d[k, 0]), int(d[k, 2]) - 1))
        k = k1
    return runs


def tag_array(tags, offset=0):
    """[count, 2] float64 (scenario, window) of packed windows' tags ((scenario, window) tuples; any other tag:
    (-1, offset + its position)).  offset: the shard's first global window, so that untagged rows stay distinct
    after a gather (every rank's local positions start at 0)."""
    out = np.empty((len(tags), 2), np.float64)
    for i, t in enumerate(tags):
        if isinstance(t, tuple) and len(t) == 2 and all(isinstance(v, (int, np.integer)) for v in t):
            out[i] = t
        else:
            out[i] = (-1, offset + i)
    return out


def result_rows(stats, istats, x=None, desc=None, tmax=None, runs=None, tags=None, offset=0):
    """Per-window result rows (float64): {obj, primal_res_rel, dual_res_rel, gap_rel, status, iters, scenario,
    window} and, with x / desc, the window's dispatch ch, dis, ene in a fixed stride of 3 * tmax (zero padded).
    tags: [count, 2] (scenario, window) per window (``tag_array``; a tensor on the rows' device, or numpy); None:
    (-1, offset + local position), offset = the shard's first global window.  Works on device or host tensors
    (strided copies per run of equal windows; no index tensors)."""
    import torch
    k = stats.shape[0]
    if tags is None:
        tg = torch.stack([torch.full((k,), -1.0, dtype=torch.float64, device=stats.device),
                          torch.arange(offset, offset + k, dtype=torch.float64, device=stats.device)], dim=1)
    else:
        tg = torch.as_tensor(tags, dtype=torch.float64).to(stats.device)
    base = torch.cat([stats.to(torch.float64), istats.to(torch.float64), tg], dim=1)
    if x is None:
        return base.contiguous()
    runs = runs if runs is not None else dispatch_runs(desc)
    tmax = int(tmax or max(r[4] for r in runs))
    rows = torch.zeros((base.shape[0], RESULT_COLS + 3 * tmax), dtype=torch.float64, device=base.device)
    rows[:, :RESULT_COLS] = base
    for k0, k1, on, n, T in runs:
        xs = x[on:on + (k1 - k0) * n].view(k1 - k0, n)
        for v in range(3):  # ch, dis, ene blocks, each padded to tmax
            rows[k0:k1, RESULT_COLS + v * tmax:RESULT_COLS + v * tmax + T] = xs[:, v * T:(v + 1) * T]
    return rows


class PendingGather:
    """An all-gather in flight (``gather_rows(..., async_op=True)``): ``wait()`` returns the gathered rows.  The
    rows tensor it reads stays referenced until then."""

    def __init__(self, work, out, rows):
        self._work, self._out, self._rows = work, out, rows

    def wait(self):
        self._work.wait()
        self._rows = None
        return self._out


def gather_rows(rows, group=None, counts=None, async_op=False):
    """All-gather a [k_r, w] float64 tensor of per-window result rows from every rank; returns the concatenation in
    rank order (identical on every rank).  counts: every rank's k_r when known on all ranks (weak scaling, a
    deterministic shard): then the rows go out in ONE all-gather; otherwise the counts are exchanged first.
    async_op (equal counts only): start the all-gather and return a ``PendingGather`` at once, so the caller can
    solve the next batch while the rows travel (RCCL runs on its own stream)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if async_op:
        if counts is None or any(n != rows.shape[0] for n in counts):
            raise ValueError("an asynchronous gather needs every rank's count, all equal to this rank's")
        pad = rows.contiguous()
        out = torch.empty((world * pad.shape[0], pad.shape[1]), dtype=pad.dtype, device=pad.device)
        if hasattr(dist, "all_gather_into_tensor") and dist.get_backend(group) != "gloo":
            work = dist.all_gather_into_tensor(out, pad, group=group, async_op=True)
        else:
            work = dist.all_gather(list(out.chunk(world)), pad, group=group, async_op=True)
        return PendingGather(work, out, pad)
    if counts is None:
        k = torch.tensor([rows.shape[0]], dtype=torch.int64, device=rows.device)
        ks = [torch.zeros_like(k) for _ in range(world)]
        dist.all_gather(ks, k, group=group)
        counts = [int(v.item()) for v in ks]
    kmax = max(counts)
    if rows.shape[0] == kmax:
        pad = rows.contiguous()
    else:
        pad = torch.zeros((kmax, rows.shape[1]), dtype=rows.dtype, device=rows.device)
        pad[: rows.shape[0]] = rows
    out = torch.empty((world * kmax, rows.shape[1]), dtype=rows.dtype, device=rows.device)
    if hasattr(dist, "all_gather_into_tensor") and dist.get_backend(group) != "gloo":
        dist.all_gather_into_tensor(out, pad, group=group)
    else:
        dist.all_gather(list(out.chunk(world)), pad, group=group)
    if all(n == kmax for n in counts):
        return out
    return torch.cat([out[r * kmax:r * kmax + n] for r, n in enumerate(counts)], dim=0)


class LibraryGather:
    """The result all-gather through libdervet_hip's own RCCL communicator (``dvh_comm_init`` / ``dvh_gather_results``,
    include/dervet_hip.h): what ``gather_rows`` does over torch.distributed, with the collective inside the library, so
    that a consumer without PyTorch can shard too.  torch.distributed (when present) only carries the 128-byte unique id
    from rank 0 to the others (``from_torch``).  The gather runs on a stream of its own: ``gather(rows,
    async_op=True)`` returns at once (the next solve runs beside it) and its ``wait()`` orders the caller's stream after
    it."""

    def __init__(self, solver, rank, world, uid):
        import torch
        self.solver, self.rank, self.world = solver, int(rank), int(world)
        solver.comm_init(rank, world, uid)
        self.stream = torch.cuda.Stream()

    @classmethod
    def from_torch(cls, solver, group=None):
        """Rank 0 draws the id, torch.distributed broadcasts it (the launcher's role only)."""
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        box = [solver.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0, group=group)
        return cls(solver, rank, world, box[0])

    def gather(self, rows, async_op=False):
        import torch
        pad = rows.contiguous()
        out = torch.empty((self.world * pad.shape[0],) + tuple(pad.shape[1:]), dtype=pad.dtype, device=pad.device)
        cur = torch.cuda.current_stream(pad.device)
        self.stream.wait_stream(cur)  # the rows are ready before the gather reads them
        self.solver.gather_results(pad, out, self.stream)
        done = PendingLibraryGather(self.stream, out, pad)
        return done if async_op else done.wait()


def agreed_library_gather(solver, device="cpu", group=None, make=None):
    """The library's all-gather on every rank, or on none: each rank tries to form the communicator
    (``LibraryGather.from_torch``, or ``make()``), and one MIN all-reduce of the outcome over torch.distributed decides
    before the first gather, so that no rank gathers through RCCL while another uses torch.distributed's all-gather.
    Returns (LibraryGather or None, the reason it is None or None).  ``device``: where the all-reduce's flag lives
    (the rank's GPU for the nccl backend, "cpu" for gloo)."""
    import torch
    import torch.distributed as dist
    lib, err = None, None
    try:
        lib = make() if make is not None else LibraryGather.from_torch(solver, group)
    except (RuntimeError, OSError) as e:
        err = str(e) or type(e).__name__
    ok = torch.tensor([0 if err else 1], dtype=torch.int32, device=device)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
    if int(ok.item()) == 0:
        return None, err or "another rank could not form the library's communicator"
    return lib, None


class PendingLibraryGather:
    """A library all-gather in flight: ``wait()`` makes the current stream wait for it and returns the rows (the input
    stays referenced until then)."""

    def __init__(self, stream, out, rows):
        import torch
        self._ev = torch.cuda.Event()
        self._ev.record(stream)
        self._out, self._rows = out, rows

    def wait(self):
        import torch
        torch.cuda.current_stream(self._out.device).wait_event(self._ev)
        self._ev.synchronize()
        self._rows = None
        return self._out


def rows_to_numpy(rows, tmax=None):
    r = rows.detach().cpu().numpy()
    out = dict(obj=r[:, 0], primal_res_rel=r[:, 1], dual_res_rel=r[:, 2], gap_rel=r[:, 3],
               status=r[:, 4].astype(np.int32), iters=r[:, 5].astype(np.int64), scenario=r[:, 6].astype(np.int64),
               window=r[:, 7].astype(np.int64))
    if r.shape[1] > RESULT_COLS:
        tm = tmax or (r.shape[1] - RESULT_COLS) // 3
        out.update(ch=r[:, RESULT_COLS:RESULT_COLS + tm], dis=r[:, RESULT_COLS + tm:RESULT_COLS + 2 * tm],
                   ene=r[:, RESULT_COLS + 2 * tm:RESULT_COLS + 3 * tm])
    return out


def by_tag(rows_np):
    """rows_to_numpy output re-ordered by (scenario, window) -- the consumer's order, whatever the packing."""
    order = np.lexsort((rows_np["window"], rows_np["scenario"]))
    return {k: v[order] for k, v in rows_np.items()}

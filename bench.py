#!/usr/bin/env python3
"""Bench: dispatch-LP windows/s of the batched HIP PDHG solver (BASELINE.json metric, config 4).

Workload (N=1): BASELINE.json configs[3] -- the synthetic scenario sweep, 10,000 perturbations of the
config-2 battery + PV + demand-charge + retail scenario (data/multi_der_hourly_timeseries.csv,
data/tariff.csv) x 12 monthly windows (T = 672..744 hourly steps) = 120,000 window LPs per GPU.
Multi-GPU (one process per GPU): `bench.py --gpus N` starts its N ranks itself (child processes, rendezvous on
127.0.0.1) unless an outside launcher (torch.distributed.run) already set WORLD_SIZE, which must then equal N.
Every rank solves its own 10,000-scenario shard (global scenario ids rank*S .. rank*S+S-1, weak scaling); no
traffic during the solve, then ONE RCCL all-gather returns every window's {objective, residuals, status,
iterations, (scenario, window) tag, ch / dis / ene dispatch} to all ranks, overlapped with the next step's solve.

A step = one solve of the rank's whole batch, already resident in HBM (setup kernel: transpose +
scaling + ||K|| estimate; PDHG kernel: the iterations), plus the result all-gather when N > 1.
Default schedule "seeded" (dervet_hip/sweep.py): the windows of 1 in 32 scenarios (battery-energy order) are
solved from zero first, then every other window warm from its nearest seed's solution of the same month --
two solver calls per step, every window solved once per step to the same KKT tolerance; nothing carries over
between steps (the seed phase starts from zero and the warm phase overwrites every warm start).  After the
timed steps the same batch is solved once more with every window cold, reported as schedule.cold_*.
The CPU baseline (rank 0, N=1 only) times two CPU solvers on bounded samples of the same windows, on the box's
16-core CPU share: the same restarted-Halpern PDHG in C++/OpenMP behind the same C ABI (oracle/cpu_pdhg.cpp, every
window cold -- compare with schedule.cold_windows_per_s), which is the faster of the two and gives `value`, and
the restated LP + HiGHS on a process pool (oracle/cpu_baseline.py), which is also the parity check of the GPU
objectives on its sample.
"""
import argparse
import functools
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "der-vet_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "dispatch LP windows/sec (whole node, 8760h monthly windows); % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# VALU issue peak: 256 CUs x 4 SIMDs x 2.4 GHz, one wave instruction per 2 cycles per SIMD (MI355X_MICROARCH.md:
# "issues each VALU instruction over 2 cycles"); FP64 FMA / ADD / MUL issue at half that (78.6 TF FP64 vector)
VALU_PEAK_WAVE_INSTS = 256 * 4 * 2.4e9 / 2


def alg_bytes_per_iter(desc):
    """B_iter = 24 nnz + 4 (n + m) + 72 n + 48 m bytes per PDHG iteration per window."""
    n, m, nnz = desc[:, 0].astype(np.float64), desc[:, 1].astype(np.float64), desc[:, 3].astype(np.float64)
    return 24 * nnz + 4 * (n + m) + 72 * n + 48 * m

# FP64 vector peak: 256 CUs x 4 SIMDs x 16 FP64 FMA lanes per clock x 2 FLOP x 2.4 GHz = 78.6 TFLOP/s (AMD spec; half the
# 157.3 TFLOP/s FP32 vector rate of MI355X_MICROARCH.md "Chip-level parameters")
FP64_PEAK_TFLOPS = 256 * 4 * 16 * 2 * 2.4e9 / 1e12


@functools.lru_cache(maxsize=None)
def source_key(config=None):
    """Hash of what decides the kernels' machine code -- the sources (csrc/, the public header) AND the build
    configuration (dervet_hip/build.py FLAGS + per-source EXTRA_FLAGS, and the hipcc / clang version): PMC profiles
    under profiles/ are used only for the kernels they measured, so a flag-only change nulls the roofline until it
    is re-profiled.  ``config`` (a JSON string) overrides the build configuration (tests)."""
    import hashlib
    h = hashlib.sha1()
    csrc = os.path.join(ROOT, "der-vet_amd", "csrc")
    for f in sorted(os.listdir(csrc)):
        with open(os.path.join(csrc, f), "rb") as fh:
            h.update(f.encode() + fh.read())
    with open(os.path.join(ROOT, "include", "dervet_hip.h"), "rb") as fh:
        h.update(b"include/dervet_hip.h" + fh.read())
    if config is None:
        from dervet_hip import build as _build
        config = json.dumps(_build.build_config(), sort_keys=True)
    h.update(config.encode())
    return h.hexdigest()[:12]


def pmc_profiles(count, launches):
    """PMC results of this exact workload and kernel build (profiles/pdhg_traffic.json: FETCH_SIZE / WRITE_SIZE
    passes; profiles/pdhg_valu.json: SQ instruction counters), or {} when they were measured on other sources."""
    out = {}
    key = source_key()
    for name in ("pdhg_traffic", "pdhg_valu"):
        fn = os.path.join(ROOT, "profiles", f"{name}.json")
        if not os.path.exists(fn):
            continue
        with open(fn) as f:
            j = json.load(f)
        if j.get("windows") == count and j.get("source_key") == key and \
                j.get("launches_per_step", j.get("dispatches_per_step")) == launches:
            out[name] = j
    return out


def outputs_sha(dev):
    """SHA-256 of the batch's outputs (x, y, stats, istats), in that order, as host bytes."""
    import hashlib
    h = hashlib.sha256()
    for t in (dev.x, dev.y, dev.stats, dev.istats):
        h.update(t.detach().cpu().numpy().tobytes())
    return h.hexdigest()


def stream_copy_gbps(dev, gib=2.0, reps=10):
    """Measured HBM copy ceiling on this GPU (torch device-to-device copy, read + write bytes / time)."""
    n = int(gib * 2 ** 30 / 8)
    a = torch.empty(n, dtype=torch.float64, device=f"cuda:{dev}").fill_(1.0)
    b = torch.empty_like(a)
    b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    gbps = 2.0 * 8 * n * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del a, b
    torch.cuda.empty_cache()
    return gbps


def roofline_object(alg, pdhg_s, prof, kname, launches, copy_gbps):
    """The dominant kernel's bound.  The iterate and scaled K of a window stay in VGPRs / LDS for the whole solve, so
    HBM moves only inputs, warm starts and outputs: the binding resource is the FP64 VALU pipe and its latency, and
    that is the headline (achieved FP64 FLOP/s from PMC instruction counts / PDHG kernel time, vs the 78.6 TFLOP/s
    FP64 vector peak).  HBM: PMC bytes / time vs 8 TB/s and the measured copy ceiling.  The SURVEY.md 8d
    algorithmic bytes / time is reported as the "effective" rate of an HBM-streaming formulation."""
    r = {"bound": "valu-fp64", "achieved": None, "peak": round(FP64_PEAK_TFLOPS, 2), "unit": "TFLOP/s", "frac": None,
         "traffic": None, "kernel": kname + f": {launches} launch(es) per step; times from HIP events on the solver "
                                             "stream", "source_key": source_key()}
    v = prof.get("pdhg_valu")
    if v and pdhg_s > 0:
        c = v["counters_per_step"]
        fl = 64.0 * (2.0 * c.get("SQ_INSTS_VALU_FMA_F64", 0.0) + c.get("SQ_INSTS_VALU_ADD_F64", 0.0) +
                     c.get("SQ_INSTS_VALU_MUL_F64", 0.0))
        r["achieved"] = round(fl / pdhg_s / 1e12, 3)
        r["frac"] = round(fl / pdhg_s / 1e12 / FP64_PEAK_TFLOPS, 4)
        r["fp64_flops_per_step"] = fl
        valu = c.get("SQ_INSTS_VALU", 0.0)
        r["issue"] = {"valu_wave_insts_per_s": valu / pdhg_s, "peak": VALU_PEAK_WAVE_INSTS,
                      "frac": round(valu / pdhg_s / VALU_PEAK_WAVE_INSTS, 4),
                      "fp64_share_of_valu": round((c.get("SQ_INSTS_VALU_FMA_F64", 0.0) + c.get("SQ_INSTS_VALU_ADD_F64", 0.0)
                                                   + c.get("SQ_INSTS_VALU_MUL_F64", 0.0)) / max(valu, 1.0), 4)}
        r["pmc_counters"] = "profiles/pdhg_valu.json"
    t = prof.get("pdhg_traffic")
    hbm = {"peak": HBM_PEAK_GBS, "unit": "GB/s", "stream_copy": round(copy_gbps, 1)}
    if t and pdhg_s > 0:
        r["traffic"] = t["hbm_bytes_per_step"]
        a = t["hbm_bytes_per_step"] / pdhg_s / 1e9
        hbm.update(achieved=round(a, 1), frac=round(a / HBM_PEAK_GBS, 5), frac_of_stream_copy=round(a / copy_gbps, 5),
                   pmc_counters="profiles/pdhg_traffic.json (FETCH_SIZE x2 + WRITE_SIZE)")
    r["hbm"] = hbm
    r["effective"] = {"alg_bytes_per_step": alg, "GBps": round(alg / pdhg_s / 1e9, 1) if pdhg_s > 0 else None,
                      "note": "SURVEY.md 8d B_iter = 24 nnz + 4 (n + m) + 72 n + 48 m per window-iteration x iterations; "
                              "what an HBM-streaming formulation of the same iterations would move"}
    return r


# the full-population certification of the bench kernel: every one of the 120,000 windows, seeded and cold, re-solved
# by HiGHS on the host (scripts/certify_dump.py + scripts/certify_highs.py)
CERTIFICATION = ("profiles/r06z_certify.json (all 120,000 windows vs HiGHS, seeded with blended warm starts and cold: "
                 "every window optimal, max 9.72e-7 / 9.78e-7; final round-6 library: wave-0 issue priority, pinned "
                 "blends, batched KKT factor loads, scalar window offsets, late lane-local SOE rows)")


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n):
    """``--gpus N`` with no outside launcher (WORLD_SIZE unset): start N child processes of this script, one rank per
    GPU (RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1), before this process makes any GPU call.
    Rank 0 prints the JSON line; the others print nothing.  A rank that fails ends the others (they would wait in a
    collective forever).  Returns the worst exit status.  The reference's own loop over cases
    (dervet/DERVET.py:75-83) is what the ranks' shards replace."""
    import signal
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [None] * n
    try:
        while any(rc is None for rc in rcs):
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    rcs[i] = p.poll()
            if any(rc not in (None, 0) for rc in rcs):
                for i, p in enumerate(procs):
                    if rcs[i] is None:
                        p.send_signal(signal.SIGTERM)
                for i, p in enumerate(procs):
                    if rcs[i] is None:
                        try:
                            rcs[i] = p.wait(timeout=30)
                        except subprocess.TimeoutExpired:
                            p.kill()
                            rcs[i] = p.wait()
                break
            time.sleep(0.05)
    except KeyboardInterrupt:
        for p in procs:
            p.kill()
        raise
    bad = [rc for rc in rcs if rc != 0]
    if bad:
        sys.stderr.write(f"bench.py: rank exit statuses {rcs}\n")
        # a signal death (negative) is reported as 128 + signal, as a shell would
        return max(128 - rc if rc < 0 else rc for rc in bad)
    return 0


def rank_counts(dist, count, device):
    """Every rank's window count, on every rank (one small all-gather)."""
    t = torch.tensor([count], dtype=torch.int64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [int(v.item()) for v in out]


def dry_run(args, world, rank):
    """The N > 1 plumbing of ``main`` without a GPU (the CPU test of ``--gpus N``): gloo process group, the weak shard
    of scenarios, tagged result rows of a stub solve (every window 'optimal' at 0 iterations, dispatch zero), the
    overlapped all-gather, barrier-bracketed timing with the max over ranks, and the JSON line from rank 0."""
    import torch.distributed as dist
    from dervet_hip import parallel
    dist_on = world > 1
    if os.environ.get("DVH_DRY_RUN_FAIL_RANK") == str(rank):  # test hook: a rank that dies before the rendezvous
        raise SystemExit(3)
    if dist_on:
        dist.init_process_group("gloo")
    S = args.scenarios
    scen = range(*parallel.weak_shard(S, rank))
    tags = [(s, w) for s in scen for w in range(12)]
    count = len(tags)
    stats = torch.zeros((count, 4), dtype=torch.float64)
    stats[:, 0] = torch.arange(count, dtype=torch.float64) + rank * count
    istats = torch.zeros((count, 2), dtype=torch.int32)
    tg = torch.as_tensor(parallel.tag_array(tags, offset=rank * count))
    per_rank = rank_counts(dist, count, "cpu") if dist_on else [count]
    pending, gathered, gather = None, None, {}

    def step():
        nonlocal pending, gathered
        rows = parallel.result_rows(stats, istats, tags=tg)
        if dist_on:
            if pending is not None:
                gathered = pending.wait()
            pending = parallel.gather_rows(rows, counts=per_rank, async_op=True)
        else:
            gathered = rows

    def drain():
        nonlocal pending, gathered
        if pending is not None:
            gathered = pending.wait()
            pending = None

    for _ in range(args.warmup):
        step()
    drain()
    if dist_on:
        dist.barrier()
    t = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()
    if dist_on:
        dist.barrier()
    el = time.perf_counter() - t
    if dist_on:
        tt = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    g = parallel.by_tag(parallel.rows_to_numpy(gathered))
    gather.update(per_rank_windows=per_rank, rows=int(len(g["obj"])),
                  scenarios=sorted(set(int(v) for v in g["scenario"])) if len(g["obj"]) <= 1200 else None)
    line = {"metric": METRIC, "value": None, "unit": "windows/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * el / max(args.steps, 1), 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "dry run (stub solve, no GPU)",
            "config": {"workload": f"dry run: {S} scenarios x 12 windows per rank", "scenarios_per_gpu": S,
                       "windows_per_gpu": count, "parallelism": f"dp{world} (gloo, dry run)"},
            "rank_pids": None, "gather": gather}
    pids = [None] * world
    if dist_on:
        dist.all_gather_object(pids, os.getpid())
        dist.destroy_process_group()
    else:
        pids = [os.getpid()]
    line["rank_pids"] = pids
    if rank == 0:
        print(json.dumps(line), flush=True)
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scenarios", type=int, default=10000, help="scenarios per GPU (x 12 monthly windows)")
    ap.add_argument("--cpu-sample", type=int, default=960, help="windows in the HiGHS CPU-baseline sample")
    ap.add_argument("--cpu-procs", type=int, default=0)
    ap.add_argument("--cpu-pdhg-sample", type=int, default=960, help="windows in the C++ CPU PDHG baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--check-every", type=int, default=0, help="restart-check period (0: library default)")
    ap.add_argument("--kkt-every", type=int, default=0, help="KKT check every n restart checks (0: default)")
    ap.add_argument("--schedule", choices=("seeded", "cold"), default="seeded",
                    help="seeded: every seed-stride-th scenario (battery-energy order) solved cold, the rest warm "
                         "from their nearest seed (dervet_hip/sweep.py); cold: every window from zero")
    ap.add_argument("--seed-stride", type=int, default=32)
    ap.add_argument("--blend", type=int, default=4,
                    help="seeded schedule: every warm window starts from the inverse-distance-weighted blend of its "
                         "BLEND nearest seeds' transferred solutions (1: the nearest seed alone)")
    ap.add_argument("--blend-power", type=float, default=1.0, help="blend weights 1 / distance^POWER")
    ap.add_argument("--blend-lam", type=float, default=-1.0,
                    help="> 0: blend weights moved toward the partners' affine combination that reproduces the window's "
                         "features, regularised toward the inverse-distance weights by LAM (dervet_hip.sweep."
                         "affine_weights); <= 0: inverse-distance weights")
    ap.add_argument("--no-cold-ref", action="store_true", help="skip the untimed all-cold reference solve")
    ap.add_argument("--sha", action="store_true", help="add the SHA-256 of the last step's x / y / stats / istats "
                    "(bit-identity of two library builds on the same batch)")
    ap.add_argument("--warm-options", default="", help="seeded schedule: dvh_options of the warm phase as JSON "
                    "(default: sweep.WARM_OPTIONS)")
    ap.add_argument("--seed-options", default="", help="seeded schedule: dvh_options of the cold seed phase as JSON "
                    "(default: sweep.SEED_OPTIONS)")
    ap.add_argument("--kkt-predict", type=int, default=4,
                    help="dvh_options.kkt_predict for cold solves (--schedule cold and the cold reference; the seeded "
                         "schedule's phases use sweep.SEED_OPTIONS / WARM_OPTIONS); 0 = every due KKT check runs")
    ap.add_argument("--overlap-gather", type=int, default=1,
                    help="N > 1: 1 = a step's result all-gather travels while the next step solves (one in flight; "
                         "the last one completes inside the timed region), 0 = gather then the next solve")
    ap.add_argument("--series", choices=("device", "host"), default="device",
                    help="with --build device: the scenarios' series generated on the GPU (lp/gpu_series.py) or by "
                         "numpy on the host (bit-identical)")
    ap.add_argument("--build", choices=("device", "host"), default="device",
                    help="window expansion: on the GPU from compact inputs (lp/gpu_builder.py) or by the host "
                         "builder + upload (bit-identical batches; untimed by the contract, reported as build)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: every rank runs the launch, sharding, tagged result rows, the overlapped gather "
                         "(gloo) and the max-over-ranks timing with a stub solve; for the CPU test of --gpus N")
    args = ap.parse_args()

    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # --gpus N without an outside launcher: N rank processes of this script, started before this process touches
        # the GPU (children, never an exec of this process)
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} from the launcher but --gpus {args.gpus}: refusing a run whose "
                         "rank count differs from the GPUs it would report")
    if args.dry_run:
        return dry_run(args, world, rank)
    source_key()  # (cached now, before this process touches the GPU: without the build's record it runs hipcc)
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU (the solver has no CPU fallback)")
    # RCCL over xGMI; DVH_BENCH_BACKEND=gloo only to rehearse several ranks on one GPU (RCCL refuses that)
    backend = os.environ.get("DVH_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if world > 1 and backend == "nccl" and world > ndev:
        raise SystemExit(f"bench.py: {world} ranks over RCCL need {world} GPUs, {ndev} visible")
    local = local % ndev  # one rank per GPU; wraps only in a several-ranks-per-GPU (gloo) rehearsal
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(backend, **({"device_id": torch.device("cuda", local)} if backend == "nccl" else {}))

    from dervet_hip import BatchSolver
    from dervet_hip.lp import builder, scenarios

    from dervet_hip import parallel
    from dervet_hip.sweep import SeededSweep, WARM_OPTIONS

    S = args.scenarios
    scen = range(*parallel.weak_shard(S, rank))
    solver = BatchSolver(local)
    t0 = time.time()
    sweep = None
    series = None
    if args.build == "device" and args.series == "device":
        # the scenarios' draws and every window's series generated in HBM, bit-identical to the host generator
        from dervet_hip.lp import gpu_series
        series = gpu_series.DeviceSeries(scen, solver, f"cuda:{local}")
        make = series.config4
    else:
        make = functools.partial(scenarios.config4, spec=args.build == "device")
    if args.schedule == "seeded":
        P = series.parameters() if series is not None else scenarios.sweep_parameters(scen)
        sweep = SeededSweep(make, scen, P["E"], stride=args.seed_stride, features=scenarios.sweep_features(P),
                            blend=args.blend, blend_power=args.blend_power,
                            blend_lam=args.blend_lam if args.blend_lam > 0 else None)
        t1 = time.time()
        dev = sweep.to_device(solver, f"cuda:{local}")
        desc = sweep.desc
    elif args.build == "device":
        from dervet_hip.lp import gpu_builder
        specs = make(scen)
        t1 = time.time()
        dev = gpu_builder.pack_specs_device(specs, solver, f"cuda:{local}")
        desc = gpu_builder.desc_of(specs)[0]
        specs_tags = [s_.tags for s_ in specs]
        del specs
    else:
        groups = make(scen)
        specs_tags = [g.tags for g in groups]
        hb = builder.pack_groups(groups)
        del groups
        t1 = time.time()
        dev = hb.to_torch(f"cuda:{local}").alloc_outputs()
        desc = np.asarray(hb.desc)
        del hb
    torch.cuda.synchronize()
    build_s = time.time() - t0
    build = {"kind": args.build, "series": args.series if args.build == "device" else "host", "s": round(build_s, 2),
             "inputs_s": round(t1 - t0, 3), "expand_s": round(time.time() - t1, 3),
             "note": "inputs: per-scenario draws + series + the windows' builder inputs (device: dvh_series_draws / "
                     "dvh_series_windows, host: numpy / scipy); expand: the windows' LPs in HBM (dvh_build_battery_group)"}
    del series
    pb = dev  # windows are read back from the device for the CPU legs
    count = len(desc)
    opts = {k: v for k, v in (("check_every", args.check_every), ("kkt_every", args.kkt_every)) if v > 0}
    opts["kkt_predict"] = args.kkt_predict
    if opts:
        solver.set_options(**opts)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    gathered = None
    phase = {}
    runs = parallel.dispatch_runs(desc) if dist is not None else None
    tmax = max(r[4] for r in runs) if runs else 0
    gather = {}
    tags_dev = None
    per_rank = None
    if dist is not None:  # every gathered row carries its (scenario, window): no packing-order rebuild downstream
        tg = sweep.tags if sweep is not None else [t for s_ in specs_tags for t in s_]
        tags_dev = torch.as_tensor(parallel.tag_array(tg, offset=rank * count), device=f"cuda:{local}")
        per_rank = rank_counts(dist, count, f"cuda:{local}")
        if len(set(per_rank)) != 1:
            raise SystemExit(f"bench.py: unequal windows per rank {per_rank} under weak scaling")

    pending = None  # the previous step's all-gather, still in flight (--overlap-gather)
    # the seeded schedule's check options (None: sweep.WARM_OPTIONS / SEED_OPTIONS)
    warm_opts = json.loads(args.warm_options) if args.warm_options else None
    seed_opts = json.loads(args.seed_options) if args.seed_options else None
    # the all-gather through the library's own RCCL communicator (dvh_comm_init / dvh_gather_results; torch.distributed
    # only carries the unique id); DVH_GATHER=torch keeps torch.distributed's, and gloo rehearsals always use it
    lib_gather = None
    if dist is not None and backend == "nccl" and os.environ.get("DVH_GATHER", "library") == "library":
        # every rank forms the communicator or none uses it: a rank whose RCCL could not be opened (the same image on
        # every rank, so in practice all or none) reports it, and the ranks agree before the first gather
        lib_gather, err = parallel.agreed_library_gather(solver, device=f"cuda:{local}")
        if lib_gather is None:
            gather["library_error"] = err
            if rank == 0:
                print(f"bench.py: library all-gather unavailable ({gather['library_error']}); torch.distributed's "
                      "all-gather is used", file=sys.stderr, flush=True)
    if dist is not None:
        gather["impl"] = "libdervet_hip dvh_gather_results (RCCL)" if lib_gather else f"torch.distributed ({backend})"

    def all_gather(rows, async_op):
        if lib_gather is not None:
            return lib_gather.gather(rows, async_op=async_op)
        return parallel.gather_rows(rows, counts=[count] * world, async_op=async_op)

    def step():
        nonlocal gathered, pending
        if sweep is not None:
            phase["timing"], phase["paths"] = sweep.solve(solver, dev, warm_options=warm_opts, seed_options=seed_opts)
        else:
            solver.solve_packed(dev)
        if dist is not None:
            # the single RCCL all-gather of every window's result row: objective, residuals, status, iterations and
            # the ch / dis / ene dispatch (fixed stride 3 * tmax); equal window counts per rank (weak scaling)
            torch.cuda.synchronize()
            tg = time.perf_counter()
            rows = parallel.result_rows(dev.stats, dev.istats, dev.x, desc, tmax, runs, tags=tags_dev)
            if args.overlap_gather:
                # the rows are a copy: once it is made, the next step's solve may overwrite the batch's outputs
                # while RCCL carries this step's rows over xGMI (at most one gather in flight)
                torch.cuda.current_stream().synchronize()
                tw = time.perf_counter()
                if pending is not None:
                    gathered = pending.wait()
                gather.update(wait_ms=round(1e3 * (time.perf_counter() - tw), 2))
                pending = all_gather(rows, True)
            else:
                gathered = all_gather(rows, False)
                torch.cuda.synchronize()
            gather.update(ms=round(1e3 * (time.perf_counter() - tg), 2), bytes_per_rank=int(rows.numel() * 8),
                          bytes_total=int(rows.numel() * 8 * world), cols=int(rows.shape[1]), tmax=int(tmax),
                          overlapped=bool(args.overlap_gather))

    def drain():
        nonlocal gathered, pending
        if pending is not None:
            gathered = pending.wait()
            pending = None

    for _ in range(args.warmup):
        step()
    drain()
    barrier()
    t = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()  # the last step's rows have arrived on every rank inside the timed region
    barrier()
    el = time.perf_counter() - t
    if dist is not None:
        tt = torch.tensor([el], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    ms_per_step = 1e3 * el / args.steps
    if gather:  # the all-gather's share of a step (this rank's last step)
        gather["frac"] = round(gather["ms"] / ms_per_step, 4)
        gather["per_rank_windows"] = per_rank
    windows_total = count * world
    value = windows_total / (el / args.steps)

    # ---- per-window results of the last step (this rank), roofline of the PDHG kernel
    ist = dev.istats.cpu().numpy()
    st = dev.stats.cpu().numpy()
    tm = phase.get("timing") or solver.timing()
    ks = solver.kernel_stats()
    if sweep is not None:
        ks.update(phase["paths"])
    kname = ("pdhg_band_kernel (battery-banded)" if ks["band_windows"] == count else
             "pdhg_ell_kernel" if ks["ell_windows"] == count else "mixed band / ELL / generic kernels")
    iters = ist[:, 1].astype(np.float64)
    alg = float((alg_bytes_per_iter(desc) * iters).sum())
    pdhg_s = tm["pdhg_ms"] * 1e-3
    achieved = alg / pdhg_s / 1e9 if pdhg_s > 0 else None
    status_counts = np.bincount(ist[:, 0] + 1, minlength=6)[1:].tolist()  # OPTIMAL..NUMERICAL
    optimal_frac = float(np.mean(ist[:, 0] == 0))
    lps_step = 2 if sweep is not None and count > sweep.n_seed else 1
    prof = pmc_profiles(count, lps_step)
    roofline = roofline_object(alg, pdhg_s, prof, kname, lps_step, stream_copy_gbps(local))

    schedule = {"kind": args.schedule}
    if sweep is not None:
        ns = sweep.n_seed
        from dervet_hip.sweep import SEED_OPTIONS
        schedule.update(warm_options=warm_opts or WARM_OPTIONS, seed_options=seed_opts or SEED_OPTIONS)
        schedule.update(seed_stride=args.seed_stride, blend=sweep.blend, seed_windows=ns, iters_mean_seed=round(float(iters[:ns].mean()), 1),
                        iters_mean_warm=round(float(iters[ns:].mean()), 1) if count > ns else None,
                        pdhg_launches_per_step=2 if count > ns else 1)
    if sweep is not None and not args.no_cold_ref:
        # the same batch once more with every window started from zero (untimed by the contract; for reference)
        st_seeded = st[:, 0].copy()
        solver.set_options(warm_start=0)
        for _ in range(2):  # the first call also re-sizes the workspace for the whole batch
            barrier()
            tc = time.perf_counter()
            solver.solve_packed(dev)
            barrier()
            cold_s = time.perf_counter() - tc
        ist_c = dev.istats.cpu().numpy()
        st_c = dev.stats.cpu().numpy()
        schedule.update(cold_windows_per_s=round(count / cold_s, 1), cold_iters_mean=round(float(ist_c[:, 1].mean()), 1),
                        cold_optimal_frac=float(np.mean(ist_c[:, 0] == 0)),
                        max_obj_rel_diff_seeded_vs_cold=float(np.max(np.abs(st_seeded - st_c[:, 0]) /
                                                                     np.maximum(np.abs(st_c[:, 0]), 1.0))))

    cpu = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu and args.cpu_sample > 0:
        from oracle import cba, cpu_baseline, window_lp
        idx = np.linspace(0, count - 1, min(args.cpu_sample, count)).astype(np.int64)
        lps = [window_lp.from_packed_window(pb.window(int(k))) for k in idx]
        objs, sts, wall, procs = cpu_baseline.highs_batch(lps, args.cpu_procs or None)
        highs = {"value": round(len(idx) / wall, 2), "unit": "windows/s", "cores": procs,
                 "sample": f"{len(idx)} of the {count} config-4 windows (evenly spaced), restated LP + HiGHS "
                           f"(scipy {__import__('scipy').__version__}), one LP per process, {procs} processes "
                           f"(the GPU box's CPU share; os.cpu_count() there reports the whole host), {wall:.1f} s wall"}
        cpu = dict(highs, kind="port", cpu_model=cpu_baseline.cpu_model(), solver="HiGHS")
        if args.cpu_pdhg_sample > 0:
            from oracle.cpu_pdhg import CpuPdhgSolver
            threads = args.cpu_procs or 16
            jdx = np.linspace(0, count - 1, min(args.cpu_pdhg_sample, count)).astype(np.int64)
            plps = [pb.window_lp(int(k)) for k in jdx]
            cs = CpuPdhgSolver(threads=threads)
            tc = time.perf_counter()
            pres = cs.solve(plps)
            cwall = time.perf_counter() - tc
            cs.close()
            pobj = np.array([r.obj for r in pres])
            cpu_pdhg = {"value": round(len(jdx) / cwall, 2), "unit": "windows/s", "cores": threads,
                        "iters_mean": round(float(np.mean([r.iters for r in pres])), 1),
                        "optimal_frac": float(np.mean([r.status == 0 for r in pres])),
                        "sample": f"{len(jdx)} of the {count} config-4 windows (evenly spaced), every window cold, "
                                  f"oracle/cpu_pdhg.cpp (same algorithm and options as the GPU, C++ -O3, OpenMP "
                                  f"{threads} threads, one window per thread), {cwall:.1f} s wall",
                        "compare_to": "schedule.cold_windows_per_s (the GPU, every window cold)"}
            highs_rate = highs["value"]
            cpu = {"value": cpu_pdhg["value"], "unit": "windows/s", "cores": threads, "kind": "port",
                   "cpu_model": cpu_baseline.cpu_model(), "solver": "C++ PDHG restatement (the faster CPU path)",
                   "sample": cpu_pdhg["sample"], "pdhg": cpu_pdhg, "highs": highs}
            if highs_rate > cpu_pdhg["value"]:
                cpu.update(value=highs_rate, cores=highs["cores"], solver="HiGHS (the faster CPU path)",
                           sample=highs["sample"])
        g = st[idx, 0]
        ok = sts == 0
        rel = np.abs(g[ok] - objs[ok]) / np.maximum(np.abs(objs[ok]), 1e-12)
        # battery benefit: obj_no_battery - obj, the error of the GPU's relative to HiGHS'
        nb = np.array([cba.no_battery_objective(lp) for lp in lps])
        ben_h = nb[ok] - objs[ok]
        ben_rel = np.abs(g[ok] - objs[ok]) / np.maximum(np.abs(ben_h), 1e-12)
        parity = {"sample_windows": int(len(idx)), "highs_optimal": int(ok.sum()),
                  "max_obj_rel_err_vs_highs": float(rel.max()) if ok.any() else None,
                  "frac_obj_rel_err_le_1e-5": float(np.mean(rel <= 1e-5)) if ok.any() else None,
                  "max_benefit_rel_err": float(ben_rel.max()) if ok.any() else None,
                  "median_benefit_usd": float(np.median(ben_h)) if ok.any() else None,
                  "full_population": CERTIFICATION}

    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "windows/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: config-4 generator (PCG64 seeds 20250217+s) over data/multi_der_hourly_timeseries.csv "
                "and data/tariff.csv",
        "config": {"workload": f"config4 sweep: {S:,} scenarios x 12 monthly windows per GPU (battery + PV + "
                               "DCM + retailETS, T=672-744 h)",
                   "scenarios_per_gpu": S, "windows_per_gpu": count, "eps_rel_kkt": 1e-6, **opts,
                   "schedule": (f"seeded (1 in {args.seed_stride} scenarios cold, the rest warm from the "
                                f"inverse-distance-weighted blend of the {sweep.blend} nearest seeds in (log E/load, "
                                f"duration, PV/load); warm phase {warm_opts or WARM_OPTIONS})" if sweep is not None else "cold"),
                   "parallelism": f"dp{world} (independent windows, 1 RCCL all-gather of results)"},
        "scenario_years_per_s": round(value / 12.0, 2),
        "iters_mean": round(float(iters.mean()), 1),
        "iters_max": int(iters.max()),
        "optimal_frac": optimal_frac,
        "status_counts": status_counts,
        "max_primal_res_rel": float(np.nanmax(st[:, 1])),
        "kernel_ms": {"setup": round(tm["setup_ms"], 2), "pdhg": round(tm["pdhg_ms"], 2),
                      "solve_total": round(tm["total_ms"], 2)},
        "kernel_path": ks,
        "roofline": roofline,
        "schedule": schedule,
        "outputs_sha256": outputs_sha(dev) if args.sha else None,
        "cpu_baseline": cpu,
        "gather": gather or None,
        "parity": parity,
        "build": build,
        # inputs generated + windows expanded + one timed step, all on this GPU: what a sweep costs end to end
        "end_to_end": {"windows_per_s": round(count / (build_s + el / args.steps), 1),
                       "s": round(build_s + el / args.steps, 3)},
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

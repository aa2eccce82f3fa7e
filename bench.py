#!/usr/bin/env python3
"""Benchmark: device-resident MPI_Reduce_local, fp32 MPI_SUM, 256 MiB per operand per GPU.

BASELINE.json metric "GiB/s device-resident MPI_Reduce_local (fp32 SUM,
256 MiB) at 1/2/4/8 GPUs".  One process per GPU (torchrun for N > 1); every
rank combines its own resident (inbuf, inoutbuf) pair -- MPI_Reduce_local is
element-wise and has no exchange step, so ranks shard with no collective on
the data path ("scaling": "weak").  torch.distributed is used only for the
barrier and the max-over-ranks of the elapsed time.

A step is one MPI_Reduce_local(inbuf, inoutbuf, 67108864, MPI_FLOAT, MPI_SUM)
call through the C ABI -- the public, synchronous entry point (it returns
with the result complete).  Timed: exactly K steps between barrier +
torch.cuda.synchronize() on both sides, after W untimed warm-up steps, the
last of which runs after the opening barrier so the first timed call does not
pay the command processor's idle wake-up (BENCH_WARMUP_ORDER=before: all W
before the barrier).
    value = 3 * 256 MiB * K * N / max_rank_seconds / 2^30   (GiB/s, algorithmic bytes:
            read inbuf, read inoutbuf, write inoutbuf -- SURVEY.md §8d)

Runtime: nothing is tuned by the bench.  The library (libmpir_hip.so) defaults
HSA_ALLOCATE_QUEUE_DEV_MEM to 1 when it is loaded -- before the HSA runtime
starts -- unless the environment sets it: AQL rings in VRAM, the CP fetches each
dispatch packet locally, 1.4 us off every synchronous call.  The
bench therefore loads the library before its first GPU call, as a program linked
against libmpi does before main().  `value` is that default; `sync_variants`
shows what the headline loop gives without it and without kernarg-cache hits.

Extra fields (rank 0):
  value_conditions  what `value` was measured under (the headline).
  sync_variants the headline loop again with fresh kernel arguments on every
                call (each misses the kernarg cache: BAR write + HDP flush), and
                -- in a child process started before this one touches the GPU --
                with HSA_ALLOCATE_QUEUE_DEV_MEM=0 (ROCm's own ring placement),
                with cached and with fresh arguments (N = 1).
  roofline      dominant kernel: mpir_tile_SUM_MPIR_HIP_F32, which the synchronous
                call dispatches on the library's own AQL queue (direct_dispatch.hip);
                its duration is the CP's dispatch start / end timestamps
                (MPIR_Hip_direct_profile, the clock rocprofv3 reads), averaged over K
                profiled repeats of the timed step; achieved = algorithmic bytes per
                launch / that mean, vs the 8.0 TB/s HBM3E peak.  Its HIP-launched twin
                k_reduce_tile_lean<OpSum,float> (same reduce_tile body), timed with HIP
                events on its stream, is reported beside it; traffic = per-launch HBM
                bytes from the committed rocprofv3 PMC summary (profiles/).
  stream_api    the same combine enqueued back-to-back with MPIX_Reduce_local_stream
                (the async variant the library's own schedules use).
  pcie_inclusive  pinned / pageable / registered host buffers -> MPI_Reduce_local forced onto the
                GPU (host limit 0: H2D + kernel + D2H), the rate when rank buffers
                arrive in host memory over PiP shm.  Reported for DESIGN.md; never
                `value`.
  host_resident the same host buffers under the default dispatch (host combine
                split over the copy threads, SURVEY §8b "both host -> CPU").
  cpu_baseline  the oracle's C loop (reference algorithm, gcc -O2) on this box's host
                cores, one pinned thread per physical core (as many as the job's CPU
                quota allows; every physical core as a secondary, throttled figure),
                NUMA-local operands, a bounded sample, per socket; rank 0 at every N,
                after the GPU work, the other ranks parked on a blocking store read.
  call_distribution  rank 0's K timed calls one by one (median, p10 / p90,
                mean, min / max; per-call clock stamps in the C loop), the call
                split into kernel + fixed cost, the first timed call and the host
                gap before it.
"""
from __future__ import annotations

import argparse
import ctypes
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))
sys.path.insert(0, ROOT)

MIB = 1 << 20
GIB = 1 << 30
HBM_PEAK_BPS = 8.0e12          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
METRIC = "GiB/s device-resident MPI_Reduce_local (fp32 SUM, 256 MiB) at 1/2/4/8 GPUs"
NPAIRS = 4                     # operand pairs rotated through (>= 3)
FRESH_OFFSETS = 256            # fresh-argument loop: 256 B steps x NPAIRS = 1024 distinct argument sets
SLACK = FRESH_OFFSETS * 256    # bytes past each operand the fresh-argument offsets reach into


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without WORLD_SIZE in the environment, N > 1 starts N ranks "
                         "itself through torch.distributed.run before any GPU call")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=50,
                    help="untimed calls first: the GPU clocks and the kernarg cache settle (profiles/archive/r02/warmup_ab.log)")
    ap.add_argument("--mib", type=int, default=256, help="MiB per operand (metric: 256)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="only the timed MPI_Reduce_local loop")
    ap.add_argument("--cpu-iters", type=int, default=24, help="cpu_baseline calls per thread")
    ap.add_argument("--collectives", choices=["auto", "on", "off"], default="auto",
                    help="configs 4-5 via bench_coll.py in isolated child processes (auto: when N > 1)")
    ap.add_argument("--cpu-standin", action="store_true",
                    help="TEST ONLY: gloo + a numpy step instead of the GPU call, to exercise the rank "
                         "launch and the max-over-ranks timing on a machine without GPUs")
    ap.add_argument("--no-variants", action="store_true", help="skip sync_variants")
    ap.add_argument("--only-config5", action="store_true",
                    help="only the config5_combine block (fp16 two-operand and CHAIN8 kernels), for rocprofv3 passes")
    ap.add_argument("--variant-child", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


def spawn_ranks(args) -> int | None:
    """`python bench.py --gpus N` with no WORLD_SIZE: start N ranks (one per GPU)
    through torch.distributed.run on 127.0.0.1 and return their exit code.
    Called before anything touches a GPU; the ranks find WORLD_SIZE set and
    run main() themselves, rank 0 printing the JSON line."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def cpu_standin(args) -> None:
    """TEST ONLY (--cpu-standin): the rank plumbing of main() with gloo and a
    numpy a += b step, so a CPU test can check that `bench.py --gpus N` runs N
    ranks and reports n_gpus = N.  Never a measurement."""
    import numpy as np
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group(backend="gloo")
    import torch
    a = np.ones(1 << 16, np.float32)
    b = np.ones(1 << 16, np.float32)

    def step(i):
        np.add(a, b, out=a)

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    own, calls = [], []
    dt = time_steps(step, args.steps, args.warmup, lambda: None, barrier, max_over_ranks, own, calls)
    alg = 3 * a.nbytes
    cstats = call_stats(calls, alg)
    rows = gather_rows([float(rank), own[0], cstats["median_us"]], world, dist, "cpu")
    out = {"metric": METRIC, "value": None, "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
           "per_rank": [{"rank": int(r[0]), "seconds": round(r[1], 6),
                         "ms_per_step": round(r[1] / args.steps * 1e3, 4), "call_median_us": r[2]} for r in rows],
           "call_distribution": dict(cstats, source="perf_counter after each stand-in step (rank 0)"),
           "data": "cpu stand-in (test only, not a measurement)"}
    # the collectives block's row format (bench_coll.coll_row) over the
    # stand-in's per-rank times, as the GPU run reports configs 4 and 5
    import bench_coll
    per = [r[1] / args.steps for r in rows]
    out["collectives"] = {"stand_in": True,
                          "config4_allreduce_fp32_sum_256MiB": {"rccl": bench_coll.coll_row(per, world, alg, "allreduce")},
                          "config5_reduce_scatter_block_fp16_sum_1GiB": {
                              "rccl": bench_coll.coll_row(per, world, alg, "reduce_scatter")}}
    if rank == 0 and not args.no_cpu_baseline:
        # the real baseline routine on a small sample
        try:
            out["cpu_baseline"] = cpu_baseline(args, 1 << 16, 3 * (1 << 18))
        except Exception as exc:        # noqa: BLE001
            out["cpu_baseline"] = {"error": repr(exc)}
        out["cpu_baseline"]["ranks_parked"] = world - 1
    if not args.no_cpu_baseline:
        park_until_rank0(world > 1, world, rank, dist, "bench_cpu_baseline_done")
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def time_steps(step, k: int, w: int, sync, barrier, max_over_ranks, own: list | None = None,
               calls: list | None = None) -> float:
    """W untimed steps, then exactly K steps bracketed by barrier + device sync; max over ranks.
    `own`, if given, receives this rank's own seconds (for the per-rank report);
    `calls` each timed step's own duration (a clock read after every step).
    Python's cyclic garbage collector is held off while the K steps run, as
    timeit does: a full collection over torch's objects can take milliseconds,
    which the Python-stepped loops would otherwise count as a step."""
    for i in range(w):
        step(i)
    sync()
    barrier()
    sync()
    gc_on = gc.isenabled()
    gc.disable()
    stamps = [] if calls is not None else None
    t0 = time.perf_counter()
    if stamps is None:
        for i in range(k):
            step(w + i)
    else:
        for i in range(k):
            step(w + i)
            stamps.append(time.perf_counter())
    sync()
    t1 = time.perf_counter()
    if gc_on:
        gc.enable()
    barrier()
    if own is not None:
        own.append(t1 - t0)
    if calls is not None:
        calls.extend(b - a for a, b in zip([t0] + stamps[:-1], stamps))
    return max_over_ranks(t1 - t0)


def gather_rows(row: list, world: int, dist, tensor_device: str) -> list:
    """Every rank's `row` (floats), in rank order, on every rank (all_gather over
    the timing group; one row when there is no group)."""
    if world == 1 or not dist.is_initialized():
        return [row]
    import torch
    t = torch.tensor(row, dtype=torch.float64, device=tensor_device)
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [x.cpu().tolist() for x in out]


def run_collectives_child(rank: int, world: int, local: int, barrier, timeout: float = 180.0):
    """Configs 4-5 (Allreduce fp32 256 MiB, Reduce_scatter_block fp16 1 GiB) in a
    child process per rank with its own RCCL communicator, so a failure there
    cannot take this process's measurement down: the child is killed after
    `timeout` seconds and the error is reported instead.  main() runs it before
    this process touches the GPU, so the child never shares the card with its
    own live rank; the children meet over their own TCPStore, and `barrier`
    (a no-op there) only lines the ranks up when they have a group already."""
    import subprocess
    barrier()
    env = dict(os.environ, RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(local),
               COLL_STORE_PORT=str(int(os.environ.get("MASTER_PORT", "29500")) + 101))
    p = subprocess.Popen([sys.executable, os.path.join(ROOT, "bench_coll.py")], env=env,
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, start_new_session=True)
    try:
        so, se = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, 9)
        p.communicate()
        return {"error": f"timeout after {timeout:.0f} s"}
    if p.returncode != 0:
        return {"error": f"exit {p.returncode}", "stderr_tail": se.strip().splitlines()[-3:]}
    lines = [ln for ln in so.splitlines() if ln.startswith("{")]
    if rank == 0:
        return json.loads(lines[-1]) if lines else {"error": "no output"}
    return {}


def time_loop(run, k: int, w: int, sync, barrier, max_over_ranks, own: list | None = None,
              calls: list | None = None, gap: list | None = None, bracket: list | None = None) -> float:
    """time_steps for a C loop: run(start, n[, stamps]) makes steps start ..
    start + n - 1 back to back; W untimed steps, then exactly K timed ones
    between barrier + device sync, max over ranks.  `calls`, if given, receives
    the K timed calls' own durations (seconds), from the loop's per-call clock
    stamps; `gap`, if given, the host time between the last warm-up call's
    return and the first timed call (seconds, same clock).

    The last warm-up step runs after the barrier (BENCH_WARMUP_ORDER=before:
    all W before it): the command processor drops into a deeper idle state
    after 50-100 us without a doorbell (DESIGN.md "Idle gaps"), and a barrier
    over a process group takes longer than that, so without it the first timed
    call would pay a wake-up that back-to-back calls never see."""
    late = w > 0 and os.environ.get("BENCH_WARMUP_ORDER", "late") != "before"
    stamps = wst = None
    if calls is not None:
        import numpy as np
        stamps = np.zeros(k + 1, np.int64)
        # the warm-up steps take the stamped path of the C loop too: its first
        # use (the buffer protocol on the stamps array) otherwise lands inside
        # the timed region (~2.3 us once, measured r06u: timed_region_loop_entry_us)
        wst = np.zeros(w + 1, np.int64)

    def warm(start, n):
        if wst is None:
            run(start, n)
        else:
            run(start, n, wst)
    warm(0, w - 1 if late else w)
    if late:
        sync()
        barrier()
        warm(w - 1, 1)
    warm_end = time.monotonic_ns()         # CLOCK_MONOTONIC, the C loop's clock
    if not late:
        sync()
        barrier()
    ts0 = time.perf_counter()
    sync()
    ts1 = time.perf_counter()
    # Python's cyclic collector held off while the K calls run, as in
    # time_steps (and timeit)
    gc_on = gc.isenabled()
    gc.disable()
    t0 = time.perf_counter()
    if stamps is None:
        run(w, k)
    else:
        run(w, k, stamps)
    tm = time.perf_counter()
    sync()
    t1 = time.perf_counter()
    if gc_on:
        gc.enable()
    barrier()
    if bracket is not None and stamps is not None:
        # the timed region around the K calls: the Python -> C loop entry and
        # exit and the closing torch.cuda.synchronize() (same clock)
        # (perf_counter is CLOCK_MONOTONIC on Linux, the stamps' clock: the
        # entry into and the exit from the C loop split out)
        bracket.append(((t1 - t0) - (int(stamps[k]) - int(stamps[0])) * 1e-9, t1 - tm,
                        int(stamps[0]) * 1e-9 - t0, tm - int(stamps[k]) * 1e-9, ts1 - ts0))
    if own is not None:
        own.append(t1 - t0)
    if calls is not None:
        calls.extend((np.diff(stamps) * 1e-9).tolist())
        if gap is not None:
            gap.append((int(stamps[0]) - warm_end) * 1e-9)
    return max_over_ranks(t1 - t0)


def call_stats(calls: list, alg_bytes: int, pair_of: list | None = None) -> dict:
    """The timed calls' own distribution: median, p10 / p90,
    mean, min / max in us, the median call's fraction of the HBM peak, the share
    of slow calls (> median + 4 us) and what they add to the mean call; with
    `pair_of` (each call's operand pair), the median per pair."""
    v = sorted(calls)
    n = len(v)
    med = v[n // 2]
    slow = [x for x in calls if x > med + 4e-6]
    out = {"calls": n, "median_us": round(med * 1e6, 2), "p10_us": round(v[n // 10] * 1e6, 2),
           "p90_us": round(v[min(n - 1, (n * 9) // 10)] * 1e6, 2), "mean_us": round(sum(v) / n * 1e6, 2),
           "min_us": round(v[0] * 1e6, 2), "max_us": round(v[-1] * 1e6, 2),
           "frac_of_hbm_peak_at_median": round(alg_bytes / med / HBM_PEAK_BPS, 4),
           "slow_share": round(len(slow) / n, 4),
           "slow_excess_us_per_call": round(sum(x - med for x in slow) / n * 1e6, 3)}
    if pair_of:
        byp = {}
        for x, g in zip(calls, pair_of):
            byp.setdefault(g, []).append(x)
        out["median_us_by_pair"] = [round(sorted(byp[g])[len(byp[g]) // 2] * 1e6, 2) for g in sorted(byp)]
    return out


def park_until_rank0(use_pg: bool, world: int, rank: int, dist, key: str, timeout_s: float = 600.0):
    """Ranks other than 0 wait for rank 0's `key` on the process group's store
    (a blocking socket read, no spin), so rank 0's CPU work runs beside idle
    ranks; rank 0 sets it.  Falls back to a barrier if the store is unavailable."""
    if not use_pg or world == 1:
        return
    import datetime
    try:
        store = dist.distributed_c10d._get_default_store()
    except Exception:       # noqa: BLE001
        store = None
    if store is None:
        dist.barrier()
        return
    if rank == 0:
        store.set(key, "1")
    else:
        store.wait([key], datetime.timedelta(seconds=timeout_s))


def sync_loops(m, lib, reduce_local, ptrs, count, k: int, w: int, sync, barrier, max_over_ranks,
               own: list | None = None, c_loop=None, calls: list | None = None, gap: list | None = None,
               bracket: list | None = None):
    """The headline loop (NPAIRS pairs rotated: every call after the first
    NPAIRS repeats its kernel arguments, which the direct dispatch's kernarg
    cache then holds) and the same loop with fresh arguments on every call: the
    pairs shifted by multiples of 256 B (same count, same alignment, same
    kernel), 1024 distinct argument sets, so every call writes its arguments
    into a VRAM slot (before ringing the doorbell, for the checked kernel).
    With `c_loop` (the compiled binding's reduce_local_loop) the K calls run
    back to back in C, as a C caller issues them; the same loop stepped from
    Python, one compiled call per step, is timed last (`dt_py`).
    Returns seconds of each, the kernarg writes per timed fresh call, a
    one-call step function and dt_py (None without c_loop); `calls` receives
    the headline loop's per-call durations."""
    dt_f32, op_sum = m.MPI_FLOAT, m.MPI_SUM
    call_args = tuple((pin, pio, count, dt_f32, op_sum) for pin, pio in ptrs)
    fresh_args = tuple((pin + o, pio + o, count, dt_f32, op_sum) for o in range(0, SLACK, 256) for pin, pio in ptrs)

    def step(i):
        rc = reduce_local(*call_args[i % NPAIRS])
        if rc:
            raise RuntimeError(m.error_string(rc))

    def fstep(i):
        rc = reduce_local(*fresh_args[i % len(fresh_args)])
        if rc:
            raise RuntimeError(m.error_string(rc))

    def runner(sets):
        def run(start, n, stamps=None):
            rc = c_loop(sets, start, n, stamps)
            if rc:
                raise RuntimeError(m.error_string(rc))
        return run
    dt_py = None
    if c_loop is not None:
        dt = time_loop(runner(call_args), k, w, sync, barrier, max_over_ranks, own, calls, gap, bracket)
        kw0 = lib.MPIR_Hip_direct_kernarg_writes()
        dtf = time_loop(runner(fresh_args), k, w, sync, barrier, max_over_ranks, own)
        writes = (lib.MPIR_Hip_direct_kernarg_writes() - kw0) / (k + w)
        dt_py = time_steps(step, k, w, sync, barrier, max_over_ranks)
    else:
        dt = time_steps(step, k, w, sync, barrier, max_over_ranks, own, calls)
        kw0 = lib.MPIR_Hip_direct_kernarg_writes()
        dtf = time_steps(fstep, k, w, sync, barrier, max_over_ranks, own)
        writes = (lib.MPIR_Hip_direct_kernarg_writes() - kw0) / (k + w)
    return dt, dtf, writes, step, dt_py


def process_env(name: str) -> str:
    """The variable as the C runtime holds it (the library may have set it at
    load; os.environ is Python's snapshot from start-up)."""
    import ctypes
    libc = ctypes.CDLL(None)
    libc.getenv.restype = ctypes.c_char_p
    v = libc.getenv(name.encode())
    return v.decode() if v is not None else ""


def variant_child(args) -> None:
    """--variant-child: the headline loop and its fresh-argument twin in this
    process's environment (the parent sets HSA_ALLOCATE_QUEUE_DEV_MEM=0, or
    BENCH_BIND=none); one JSON line."""
    import torch
    import mpich_pip_amd as m
    lib = m.load()
    lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN)
    reduce_local = m.fast_reduce_local()
    torch.cuda.set_device(0)
    bind = bind_near_gpu(m, 0)
    count = args.mib * MIB // 4
    g = torch.Generator(device="cuda").manual_seed(0x5EED)
    pairs = [((torch.rand(count + SLACK // 4, device="cuda", generator=g) * 2 - 1),
              (torch.rand(count + SLACK // 4, device="cuda", generator=g) * 2 - 1)) for _ in range(NPAIRS)]
    torch.cuda.synchronize()
    ptrs = [(a.data_ptr(), b.data_ptr()) for a, b in pairs]
    dt, dtf, writes, _, _ = sync_loops(m, lib, reduce_local, ptrs, count, args.steps, args.warmup,
                                       torch.cuda.synchronize, lambda: None, lambda x: x,
                                       c_loop=m.fast_reduce_local_loop())
    place = placement_record(m, 0)
    print(json.dumps({"dt": dt, "dt_fresh": dtf, "kernarg_writes_per_fresh_call": writes,
                      "HSA_ALLOCATE_QUEUE_DEV_MEM": process_env("HSA_ALLOCATE_QUEUE_DEV_MEM"),
                      "direct_state": lib.MPIR_Hip_direct_state(0), "bind": bind,
                      "placement": {k: place[k] for k in ("cpu", "cpu_node", "gpu_node", "ring_in_vram")}}),
          flush=True)


def run_variant_child(args, env_over: dict | None = None) -> dict:
    """Start --variant-child with ROCm's own AQL ring placement
    (HSA_ALLOCATE_QUEUE_DEV_MEM=0), or with `env_over`; called before this
    process touches a GPU."""
    import subprocess
    env = dict(os.environ, **(env_over or {"HSA_ALLOCATE_QUEUE_DEV_MEM": "0"}))
    cmd = [sys.executable, os.path.abspath(__file__), "--variant-child", "--steps", str(args.steps),
           "--warmup", str(args.warmup), "--mib", str(args.mib)]
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    except subprocess.TimeoutExpired:
        return {"error": "timeout"}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"exit {r.returncode}", "stderr_tail": r.stderr.strip().splitlines()[-3:]}
    return json.loads(lines[-1])


def event_launch_us(launch, k: int, w: int, stream, stat: str = "mean") -> float:
    """Mean (or median) per-launch kernel time (us) from HIP events recorded on `stream`."""
    import torch
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
    for i in range(w):
        launch(i)
    for i, (e0, e1) in enumerate(evs):
        e0.record(stream)
        launch(w + i)
        e1.record(stream)
    stream.synchronize()
    ms = sorted(e0.elapsed_time(e1) for e0, e1 in evs)
    if stat == "median":
        return ms[len(ms) // 2] * 1e3
    return sum(ms) / k * 1e3


def direct_kernel_ns(lib, call, k: int, w: int, splits: list | None = None):
    """Device durations (ns) of the kernels K synchronous calls run through the
    direct AQL dispatch: the CP's dispatch start / end timestamps
    (MPIR_Hip_direct_profile; what rocprofv3 reports), or None where the
    direct path did not take the calls (then the caller uses HIP events).
    `splits`, if given, receives each call's timeline (MPIR_Hip_direct_last_split:
    ns from entering the dispatch to the doorbell, the CP's start and end, and
    the host seeing the completion signal)."""
    lib.MPIR_Hip_direct_profile(1)
    sp = (ctypes.c_uint64 * 4)()
    try:
        for i in range(w):
            call(i)
        before = lib.MPIR_Hip_direct_dispatches()
        ns = []
        for i in range(k):
            call(w + i)
            ns.append(lib.MPIR_Hip_direct_last_kernel_ns())
            if splits is not None:
                lib.MPIR_Hip_direct_last_split(sp)
                splits.append(tuple(v - (1 << 64) if v >= (1 << 63) else v for v in sp))     # (signed ns)
        if lib.MPIR_Hip_direct_dispatches() - before != k or min(ns) <= 0:
            return None
        return ns
    finally:
        lib.MPIR_Hip_direct_profile(0)


def split_medians(splits: list) -> dict | None:
    """Medians (us) of the synchronous call's intervals over the profiled calls'
    timelines (direct_kernel_ns): entry -> doorbell (host), doorbell -> CP
    dispatch start, the kernel (CP start -> end), CP end -> host sees the
    completion signal.  The profiled calls run on the timestamped twin queue."""
    # (the CP's timestamps reach the host clock through the runtime's clock
    # translation, whose offset can be a few us: the split keeps the intervals
    # that do not depend on it -- entry -> doorbell (host clock), the kernel (CP
    # clock), doorbell -> host sees completion minus the kernel -- and reports
    # doorbell -> dispatch start as translated)
    rows = [s for s in splits if 0 < s[0] < s[3] and 0 < s[2] - s[1] < s[3] - s[0]]
    if not rows:
        return None

    def med(v):
        v = sorted(v)
        return round(v[len(v) // 2] * 1e-3, 2)
    return {"calls": len(rows),
            "host_to_doorbell_us": med([s[0] for s in rows]),
            "kernel_us": med([s[2] - s[1] for s in rows]),
            "doorbell_to_seen_minus_kernel_us": med([(s[3] - s[0]) - (s[2] - s[1]) for s in rows]),
            "doorbell_to_dispatch_start_us_translated": med([s[1] - s[0] for s in rows]),
            "source": "MPIR_Hip_direct_last_split over the K profiled calls (timestamped twin queue; host clock "
                      "stamps around the CP's dispatch timestamps)"}


def placement_record(m, dev: int) -> dict:
    """Where this rank's calling thread runs relative to its GPU
    (MPIR_Hip_direct_placement), and the CPUs it may run on."""
    rec = m.placement(dev)
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except OSError:
        allowed = []
    nodes = sorted({cpu_node(c) for c in allowed})
    rec["allowed_cpus"] = len(allowed)
    rec["allowed_nodes"] = nodes
    return rec


def node_cpus(node: int) -> set:
    """CPUs of NUMA node `node` (sysfs cpulist)."""
    out = set()
    try:
        txt = open(f"/sys/devices/system/node/node{node}/cpulist").read().strip()
    except OSError:
        return out
    for part in txt.split(","):
        if "-" in part:
            a, b = part.split("-")
            out.update(range(int(a), int(b) + 1))
        elif part:
            out.add(int(part))
    return out


def bind_near_gpu(m, dev: int) -> dict:
    """Bind the calling thread (the one that makes the timed calls) to the CPUs
    of its GPU's NUMA node, within the CPUs the job may use -- what a launcher's
    binding does for a GPU rank (Hydra -bind-to, Slurm --cpu-bind / numactl
    --cpunodebind).  Near against far callers, alternated fresh processes on one
    box (tools/placement_ab.py, DESIGN.md §(d) "Where the caller runs"): the
    synchronous call ~0.5 us faster near with the library's VRAM rings (~2 us
    with ROCm's host-memory rings).  BENCH_BIND=none keeps the placement the
    process was launched with."""
    if os.environ.get("BENCH_BIND", "gpu-node") == "none":
        return {"mode": "none (as launched)"}
    gnode = m.placement(dev)["gpu_node"]
    try:
        allowed = os.sched_getaffinity(0)
    except OSError:
        return {"mode": "unbound", "reason": "no affinity interface"}
    want = node_cpus(gnode) & allowed if gnode >= 0 else set()
    if not want:
        return {"mode": "unbound", "reason": f"no allowed CPU on the GPU's node ({gnode})", "gpu_node": gnode}
    _LAUNCH_AFFINITY[:] = sorted(allowed)
    os.sched_setaffinity(0, want)          # this thread (and the threads it starts later)
    return {"mode": "gpu-node", "gpu_node": gnode, "cpus": len(want), "of_allowed": len(allowed)}


_LAUNCH_AFFINITY: list = []


def unbind() -> None:
    """Back to the CPUs the process was launched with (the CPU baseline deals
    its threads over every socket the job may use)."""
    if _LAUNCH_AFFINITY:
        os.sched_setaffinity(0, _LAUNCH_AFFINITY)


def library_hip_runtime(lib):
    """The HIP runtime libmpir_hip.so links (as loaded in this process, found
    through dladdr of one of its symbols), or None if it cannot be opened."""
    try:
        class DlInfo(ctypes.Structure):
            _fields_ = [("dli_fname", ctypes.c_char_p), ("dli_fbase", ctypes.c_void_p),
                        ("dli_sname", ctypes.c_char_p), ("dli_saddr", ctypes.c_void_p)]
        libdl = ctypes.CDLL(None)
        info = DlInfo()
        # hipHostRegister as libmpich_reduce_local.so resolved it
        addr = ctypes.cast(ctypes.CDLL(lib._name).hipHostRegister, ctypes.c_void_p).value
        if addr and libdl.dladdr(ctypes.c_void_p(addr), ctypes.byref(info)) and info.dli_fname:
            return ctypes.CDLL(info.dli_fname.decode())
        return ctypes.CDLL("libamdhip64.so.7")
    except (OSError, AttributeError):
        return None


def cpu_node(cpu: int) -> int:
    try:
        for e in os.listdir(f"/sys/devices/system/cpu/cpu{cpu}"):
            if e.startswith("node") and e[4:].isdigit():
                return int(e[4:])
    except OSError:
        pass
    return -1


def config3_sweep(m, lib, pairs, nbytes: int, stream, k: int = 15, w: int = 5):
    """BASELINE config 3: {SUM, MAX, MIN, PROD} x {int32, int64, fp32, fp64} at 256 MiB
    per operand, kernel roofline fraction per (op, type).  The resident pairs are
    reinterpreted per type; PROD multiplies by an all-ones inbuf so repeated
    in-place calls stay finite; NPAIRS such buffers rotate like the
    pairs, so no launch re-reads what the previous one left in the Infinity Cache."""
    import torch
    types = [("int32", m.MPI_INT32_T, torch.int32), ("int64", m.MPI_INT64_T, torch.int64),
             ("fp32", m.MPI_FLOAT, torch.float32), ("fp64", m.MPI_DOUBLE, torch.float64)]
    ops = [("SUM", m.MPI_SUM), ("MAX", m.MPI_MAX), ("MIN", m.MPI_MIN), ("PROD", m.MPI_PROD)]
    res = {op: {} for op, _ in ops}
    hows = set()
    for tname, dt, tt in types:
        esz = torch.tensor([], dtype=tt).element_size()
        count = nbytes // esz
        ones = [torch.ones(count, dtype=tt, device="cuda") for _ in range(NPAIRS)]
        torch.cuda.synchronize()    # the fills run on torch's stream, the timing on `stream`
        for oname, op in ops:
            def call(i):
                a, b = pairs[i % NPAIRS]
                pin = ones[i % NPAIRS].data_ptr() if oname == "PROD" else b.data_ptr()
                rc = lib.MPI_Reduce_local(pin, a.data_ptr(), count, dt, op)
                assert rc == 0, m.error_string(rc)

            def launch(i):
                a, b = pairs[i % NPAIRS]
                pin = ones[i % NPAIRS].data_ptr() if oname == "PROD" else b.data_ptr()
                rc = lib.MPIX_Reduce_local_stream(pin, a.data_ptr(), count, dt, op, stream.cuda_stream)
                assert rc == 0, m.error_string(rc)
            ns = direct_kernel_ns(lib, call, k, w)
            if ns is not None:
                us = sorted(ns)[len(ns) // 2] * 1e-3
                how = "dispatch timestamps"
            else:
                with torch.cuda.stream(stream):
                    us = event_launch_us(launch, k, w, stream, stat="median")
                how = "HIP events"
            hows.add(how)
            res[oname][tname] = round(3 * nbytes / (us * 1e-6) / HBM_PEAK_BPS, 4)
        del ones
    torch.cuda.empty_cache()
    return {"unit": "fraction of 8.0 TB/s (algorithmic bytes / median kernel time of 15 synchronous "
                    "MPI_Reduce_local calls: direct-dispatch timestamps, HIP events where that path is not taken)",
            "operand_MiB": nbytes // MIB, "timing": sorted(hows), **res}


def config2(m, lib, pairs, stream, k: int, w: int):
    """BASELINE config 2: fp32 SUM, 64 MiB per operand.  4 * NPAIRS distinct 64 MiB
    (inbuf, inoutbuf) windows of the resident buffers are rotated, 2 GiB of
    footprint per cycle, so no call finds its operands in the 256 MB Infinity Cache."""
    import torch
    count = 16 * MIB
    wins = [(a[j * count:(j + 1) * count], b[j * count:(j + 1) * count]) for a, b in pairs for j in range(4)]

    def launch(i):
        a, b = wins[i % len(wins)]
        assert lib.MPIX_Reduce_local_stream(b.data_ptr(), a.data_ptr(), count, m.MPI_FLOAT, m.MPI_SUM,
                                            stream.cuda_stream) == 0

    # the synchronous call as the headline step makes it: compiled binding,
    # arguments built once (ctypes + per-call tensor slicing cost ~2.5 us of
    # Python per call, 7 % of a 64 MiB call)
    try:
        reduce_local = m.fast_reduce_local()
    except ImportError:
        reduce_local = lib.MPI_Reduce_local
    call_args = [(b.data_ptr(), a.data_ptr(), count, m.MPI_FLOAT, m.MPI_SUM) for a, b in wins]

    def call(i):
        rc = reduce_local(*call_args[i % len(call_args)])
        if rc:
            raise RuntimeError(m.error_string(rc))
    try:
        c_loop = m.fast_reduce_local_loop()
    except ImportError:
        c_loop = None

    def timed_sync():
        """W untimed synchronous calls, then K timed ones back to back: from C
        (the compiled binding's loop, as the headline's calls), else stepped
        from Python; seconds for the K"""
        if c_loop is not None:
            sets = tuple(call_args)
            rc = c_loop(sets, 0, w)
            t0 = time.perf_counter()
            rc = rc or c_loop(sets, w, k)
            dt = time.perf_counter() - t0
            if rc:
                raise RuntimeError(m.error_string(rc))
            return dt
        for i in range(w):
            call(i)
        t0 = time.perf_counter()
        for i in range(k):
            call(w + i)
        return time.perf_counter() - t0
    alg = 3 * count * 4
    out = {"windows": len(wins), "sync_caller": "C loop" if c_loop is not None else "Python-stepped"}
    ns = direct_kernel_ns(lib, call, k, w)
    if ns is not None:
        us = sum(ns) / len(ns) * 1e-3
        out.update({"kernel_us": round(us, 2), "kernel_frac": round(alg / (us * 1e-6) / HBM_PEAK_BPS, 4),
                    "kernel_timing": "mean of K direct-dispatch timestamps (the synchronous call's kernel)"})
    with torch.cuda.stream(stream):
        ev = event_launch_us(launch, k, w, stream)
        # back to back: one event pair around K launches (no event packets between
        # launches, so one launch's ramp-up overlaps the previous one's drain)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(k):
            launch(w + k + i)
        e1.record(stream)
    stream.synchronize()
    us_b2b = e0.elapsed_time(e1) * 1e3 / k
    torch.cuda.synchronize()
    dt = timed_sync()
    out.update({"hip_event_launch_us": round(ev, 2),
                "back_to_back_us": round(us_b2b, 2), "back_to_back_frac": round(alg / (us_b2b * 1e-6) / HBM_PEAK_BPS, 4),
                "sync_api_GiBps": round(alg * k / dt / GIB, 1),
                "sync_api_frac": round(alg * k / dt / HBM_PEAK_BPS, 4)})
    if "kernel_us" not in out:
        out.update({"kernel_us": round(ev, 2), "kernel_frac": round(alg / (ev * 1e-6) / HBM_PEAK_BPS, 4),
                    "kernel_timing": "HIP events around each stream launch"})
    # the same synchronous call with every store nt (MPIR_CVAR_REDUCE_LOCAL_KEEP_MB=0):
    # the default keeps a result of <= 64 MiB in the Infinity Cache for its next
    # reader (a schedule's next step), which costs a loop where nothing re-reads
    lib.MPIR_Hip_set_keep_bytes.restype = ctypes.c_uint64
    lib.MPIR_Hip_set_keep_bytes.argtypes = [ctypes.c_uint64]
    prev = lib.MPIR_Hip_set_keep_bytes(0)
    try:
        nt = {}
        ns = direct_kernel_ns(lib, call, k, w)
        if ns is not None:
            us = sum(ns) / len(ns) * 1e-3
            nt.update({"kernel_us": round(us, 2), "kernel_frac": round(alg / (us * 1e-6) / HBM_PEAK_BPS, 4)})
        dt = timed_sync()
        nt.update({"sync_api_frac": round(alg * k / dt / HBM_PEAK_BPS, 4), "policy": "MPIR_CVAR_REDUCE_LOCAL_KEEP_MB=0"})
        out["nt_stores"] = nt
    finally:
        lib.MPIR_Hip_set_keep_bytes(prev)
    return out


def config4_combine(m, stream, k: int, w: int):
    """Config 4's combine at one GPU: the fused TREE8 fold MPIX_Reduce_local_multi
    runs in Allreduce's reference-order mode at 8 ranks (the recursive-halving
    reduce-scatter, reduce_intra_reduce_scatter_gather.c:186-249): 8 blocks of
    32 MiB fp32 (256 MiB / 8), ((y0+y1)+(y2+y3))+... into a 32 MiB output, the
    blocks at the collective's staging stride (32 MiB + 4352 B), six sets
    rotated (1.7 GiB a cycle, past the 256 MB Infinity Cache); HIP events on the
    stream.  Fraction: 9 x 32 MiB over kernel time against 8.0 TB/s."""
    import torch
    blk = 8 * MIB                               # floats in 32 MiB
    stride = blk + 4352 // 4                    # coll_hip.c stage_stride, in floats
    g = torch.Generator(device="cuda").manual_seed(0xF32)
    nsets = 6
    sets = [torch.rand(8 * stride, device="cuda", generator=g) * 2 - 1 for _ in range(nsets)]
    outs = [torch.empty(blk, device="cuda") for _ in range(nsets)]
    torch.cuda.synchronize()
    ops = [[s_.data_ptr() + 4 * j * stride for j in range(8)] for s_ in sets]

    def launch(i):
        rc = m.reduce_local_multi(ops[i % nsets], outs[i % nsets].data_ptr(), blk, m.MPI_FLOAT, m.MPI_SUM,
                                  m.MPIX_ORDER_TREE, stream.cuda_stream)
        assert rc == 0, m.error_string(rc)
    with torch.cuda.stream(stream):
        us = event_launch_us(launch, k, w, stream)
        # back to back: one event pair around K launches (a ~50 us kernel loses
        # several per cent to a per-launch event bracket)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(k):
            launch(w + k + i)
        e1.record(stream)
    stream.synchronize()
    us_b2b = e0.elapsed_time(e1) * 1e3 / k
    alg = 9 * blk * 4
    del sets, outs
    torch.cuda.empty_cache()
    return {"tree8": {"blocks": 8, "block_MiB": 32, "kernel": "k_combine_multi<OpSum, float, P=8, TREE>",
                      "kernel_us": round(us_b2b, 2),
                      "frac": round(alg / (us_b2b * 1e-6) / HBM_PEAK_BPS, 4),
                      "timing": "K launches back to back between one HIP-event pair on the launch stream",
                      "per_launch_event_us": round(us, 2),
                      "per_launch_event_frac": round(alg / (us * 1e-6) / HBM_PEAK_BPS, 4)}}


def config5_combine(m, lib, stream, k: int, w: int):
    """Config 5's combine at one GPU, in its element type (MPIX_C_FLOAT16,
    mpir_op_util.h:315-319; configure.ac:3122-3131):
      two_operand  synchronous MPI_Reduce_local fp16 SUM at 256 MiB per operand
                   (the direct dispatch's mpir_tile_SUM_MPIR_HIP_F16), NPAIRS
                   pairs rotated, kernel time from the CP's dispatch timestamps;
      chain8       the fused CHAIN8 fold MPIX_Reduce_local_multi runs for
                   Reduce_scatter_block's pairwise schedule at 8 ranks
                   (reduce_scatter_block_intra_pairwise.c:97-134): 8 blocks of
                   128 MiB, ((x0+x1)+x2)+...+x7 into a 128 MiB output, the blocks
                   at the collective's skewed staging stride (coll_hip.c
                   stage_stride: 128 MiB + 6400 B), two sets alternated (2.25 GiB a
                   cycle, past the 256 MB Infinity Cache); HIP events on the stream.
    Fractions are algorithmic bytes (3 x 256 MiB; 9 x 128 MiB) over kernel time
    against 8.0 TB/s; per-launch HBM traffic from the committed PMC summary."""
    import torch
    out = {}
    count = 128 * MIB                           # halves in 256 MiB
    g = torch.Generator(device="cuda").manual_seed(0xF16)
    pairs = [((torch.rand(count, device="cuda", generator=g, dtype=torch.float16) * 2 - 1),
              (torch.rand(count, device="cuda", generator=g, dtype=torch.float16) * 2 - 1)) for _ in range(NPAIRS)]
    torch.cuda.synchronize()
    call_args = [(b.data_ptr(), a.data_ptr(), count, m.MPIX_C_FLOAT16, m.MPI_SUM) for a, b in pairs]

    def call(i):
        rc = lib.MPI_Reduce_local(*call_args[i % NPAIRS])
        assert rc == 0, m.error_string(rc)
    alg2 = 3 * count * 2
    ns = direct_kernel_ns(lib, call, k, w)
    if ns is not None:
        us = sum(ns) / len(ns) * 1e-3
        out["two_operand"] = {"operand_MiB": 256, "kernel": "mpir_tile_SUM_MPIR_HIP_F16 (direct AQL dispatch)",
                              "kernel_us": round(us, 2), "frac": round(alg2 / (us * 1e-6) / HBM_PEAK_BPS, 4),
                              "median_us": round(sorted(ns)[len(ns) // 2] * 1e-3, 2),
                              "timing": "mean of K CP dispatch timestamps"}
    del pairs, call_args
    torch.cuda.empty_cache()

    blk = 64 * MIB                              # halves in 128 MiB
    stride = (blk * 2 + 6400) // 2              # coll_hip.c stage_stride (128 MiB blocks: + 6400 B), in halves
    sets = [torch.empty(8 * stride, device="cuda", dtype=torch.float16) for _ in range(2)]
    outs = [torch.empty(blk, device="cuda", dtype=torch.float16) for _ in range(2)]
    for s_ in sets:
        s_.uniform_(-1, 1, generator=g)
    torch.cuda.synchronize()
    ops = [[s_.data_ptr() + 2 * j * stride for j in range(8)] for s_ in sets]

    def launch(i):
        rc = m.reduce_local_multi(ops[i % 2], outs[i % 2].data_ptr(), blk, m.MPIX_C_FLOAT16, m.MPI_SUM,
                                  m.MPIX_ORDER_CHAIN, stream.cuda_stream)
        assert rc == 0, m.error_string(rc)
    with torch.cuda.stream(stream):
        us = event_launch_us(launch, k, w, stream)
    alg8 = 9 * blk * 2
    out["chain8"] = {"blocks": 8, "block_MiB": 128, "kernel": "k_combine_multi<OpSum, f16, P=8, CHAIN>",
                     "kernel_us": round(us, 2), "frac": round(alg8 / (us * 1e-6) / HBM_PEAK_BPS, 4),
                     "timing": "mean of K HIP-event brackets on the launch stream"}
    del sets, outs
    torch.cuda.empty_cache()
    traffic = {}
    try:
        traffic = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json"))).get("config5_fp16", {})
    except (OSError, ValueError):
        pass
    for key, alg in (("two_operand", alg2), ("chain8", alg8)):
        t = traffic.get(key)
        if key in out and t:
            out[key].update(traffic=t["hbm_bytes_per_launch"], traffic_over_algorithmic=round(
                t["hbm_bytes_per_launch"] / alg, 5), rocprof_avg_us=t.get("rocprof_avg_us"),
                traffic_source="profiles/pmc_traffic.json (config5_fp16)")
    return out


def load_traffic(count_bytes: int):
    """Per-launch HBM bytes of the dominant kernel from the committed PMC summary."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(p))
    except (OSError, ValueError):
        return None, None
    if d.get("operand_bytes") != count_bytes:
        return None, None
    return d.get("hbm_bytes_per_launch"), os.path.relpath(p, ROOT)


def lscpu_topology() -> dict:
    """The lines of `lscpu` that describe the host's cores."""
    import subprocess
    keys = ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core", "NUMA node(s)", "CPU(s)")
    try:
        txt = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=20).stdout
    except (OSError, subprocess.SubprocessError):
        return {}
    out = {}
    for ln in txt.splitlines():
        k, _, v = ln.partition(":")
        if k.strip() in keys and k.strip() not in out:
            out[k.strip()] = v.strip()
    return out


def cpu_baseline(args, count: int, alg_bytes: int) -> dict:
    """The reference's fp32 SUM loop (oracle/op_oracle.c, gcc -O2 like MPICH) on
    the host cores this process may use: one thread pinned per physical core,
    dealt over the sockets, each with its own NUMA-local (first-touched)
    256 MiB operand pair, all started by one barrier; aggregate = all threads'
    algorithmic bytes / slowest thread, per socket likewise.
    "Usable" is the physical cores of the CPU affinity, capped by the cgroup
    CPU quota: the GPU box shows 128 physical cores but grants 16 CPUs' worth of
    time, and 128 threads under that quota run 1/8 of each period (measured:
    130 GiB/s, against ~335 for 16 threads), a throttling figure, not a CPU
    rate -- it is reported beside the main figure as `all_physical_cores`.
    Also the clang -O2 build on the same cores."""
    import oracle
    machine = oracle.physical_cores()
    quota = oracle.cpu_quota()
    usable = min(len(machine), int(quota)) if quota else len(machine)
    cores = oracle.spread_over_sockets(machine, max(1, usable))
    iters = args.cpu_iters

    def run(cs, per, its, compiler):
        secs = oracle.cpu_baseline_pinned([c for c, _ in cs], per, its, compiler)
        if min(secs) <= 0:
            return None
        bpt = 3 * per * 4 * its             # algorithmic bytes per thread
        agg = bpt * len(cs) / max(secs) / GIB
        sockets = {}
        for (c, pkg), t in zip(cs, secs):
            sockets.setdefault(pkg, []).append(t)
        return {"value": round(agg, 2), "per_core": round(agg / len(cs), 2),
                "per_socket": {str(k): round(bpt * len(v) / max(v) / GIB, 2) for k, v in sorted(sockets.items())},
                "seconds": round(max(secs), 3)}

    # at most 16 GiB of operands over all threads (two per thread): a node whose
    # quota grants many cores (an 8-GPU node) gets smaller per-thread operands,
    # still far past every cache
    per = min(count, (16 << 30) // (8 * len(cores)))
    per -= per % 64
    g = run(cores, per, iters, "gcc")
    if g is None:
        return {"error": "cpu baseline thread failure"}
    res = {"unit": "GiB/s", "kind": "port", "cores": len(cores)}
    res.update(g)
    res["sample"] = (f"{len(cores)} threads, one pinned per physical core (dealt over the sockets), {iters} calls each "
                     f"of MPI_SUM MPI_FLOAT count {per} on its own first-touched {per * 4 / MIB:g} MiB (inbuf, inoutbuf) pair; "
                     f"oracle/op_oracle.c SUM loop, gcc -O2 (MPICH's default build); aggregate = algorithmic bytes of "
                     f"all threads / slowest thread")
    res["machine"] = {"physical_cores": len(machine), "cgroup_cpu_quota": quota, "lscpu": lscpu_topology()}
    try:
        c = run(cores, per, iters, "clang")
    except RuntimeError as e:
        c = {"error": str(e)}
    res["clang_O2"] = c if c is not None else {"error": "thread failure"}
    if quota and len(machine) > usable:
        small = int(min(count, (16 << 30) // (8 * len(machine))))
        a = run(machine, small - small % 64, max(4, iters // 3), "gcc")
        if a is not None:
            a["note"] = (f"{len(machine)} pinned threads (count {small - small % 64} each) under the "
                         f"{quota:g}-CPU cgroup quota: throttled, not a CPU rate")
            res["all_physical_cores"] = a
    return res


def main():
    args = parse()
    rc = spawn_ranks(args)
    if rc is not None:
        sys.exit(rc)
    if args.cpu_standin:
        return cpu_standin(args)
    if args.variant_child:
        return variant_child(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # ROCm's own ring placement, in a child, before this process starts the GPU
    ring_variant = launch_variant = None
    if world == 1 and not args.no_extras and not args.no_variants:
        ring_variant = run_variant_child(args)
        # the headline loop with the process left where it was launched
        launch_variant = run_variant_child(args, {"BENCH_BIND": "none"})
    # configs 4-5 (RCCL collectives) in a child per rank, also before this
    # process starts the GPU: one process per rank holds a GPU at any time
    # (a child beside a live rank would double the processes on each card)
    coll = None
    if args.collectives == "on" or (args.collectives == "auto" and world > 1 and not args.no_extras):
        coll = run_collectives_child(rank, world, local, lambda: None)
    import mpich_pip_amd as m
    # the library first, as a program linked against libmpi loads it before
    # main(): the process is still single-threaded (no numpy / torch yet), so the
    # library's load-time default puts the AQL rings into VRAM before the HSA
    # runtime starts (direct_dispatch.hip default_rings_in_vram)
    lib = m.load()
    import torch
    import torch.distributed as dist
    lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN)
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world} (launched by an external launcher); "
              f"measuring WORLD_SIZE ranks", file=sys.stderr)
    # BENCH_TEST_SHARE_GPU=1 (test only): N ranks on the GPUs there are
    # (rank -> device local % count) with a gloo process group, since RCCL
    # refuses two ranks on one GPU -- rehearses the whole N > 1 path (launch,
    # per-rank direct dispatch, extras, the collectives child's error report)
    # on a one-GPU box.  Never a measurement of N GPUs.
    share = os.environ.get("BENCH_TEST_SHARE_GPU") == "1"
    dev = local % torch.cuda.device_count() if share else local
    torch.cuda.set_device(dev)
    # the rank's calling thread near its GPU, as a launcher binds GPU ranks
    # (value_conditions.placement; BENCH_BIND=none keeps the launch placement)
    bind = bind_near_gpu(m, dev)
    if args.only_config5:
        print(json.dumps({"config5_combine": config5_combine(m, lib, torch.cuda.Stream(), args.steps, args.warmup)}),
              flush=True)
        return
    # BENCH_TEST_PG=1 (test only): the N > 1 plumbing -- RCCL process group,
    # barriers, max over ranks -- at WORLD_SIZE 1, to rehearse it on one GPU
    use_pg = world > 1 or os.environ.get("BENCH_TEST_PG") == "1"
    pg_backend = None
    if use_pg:
        if share:
            pg_backend = "gloo"
            dist.init_process_group(backend="gloo")
        else:
            # the group only carries the barriers and the max over ranks (no data
            # path collective): should RCCL fail to come up, a CPU (gloo) group
            # serves the same timing protocol rather than losing the run
            try:
                dist.init_process_group(backend="nccl", device_id=torch.device("cuda", dev))
                pg_backend = "nccl"
            except Exception as exc:       # noqa: BLE001
                print(f"warning: RCCL process group failed ({exc}); barriers over gloo", file=sys.stderr)
                if dist.is_initialized():
                    dist.destroy_process_group()
                addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
                port = int(os.environ.get("MASTER_PORT", "29500")) + 1
                dist.init_process_group(backend="gloo", init_method=f"tcp://{addr}:{port}", rank=rank,
                                        world_size=world)
                pg_backend = "gloo"
    cpu_pg = pg_backend == "gloo"

    def barrier():
        if use_pg:
            dist.barrier()

    def max_over_ranks(x: float) -> float:
        if not use_pg:
            return x
        t = torch.tensor([x], dtype=torch.float64, device="cpu" if cpu_pg else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    sync = torch.cuda.synchronize

    nbytes = args.mib * MIB
    count = nbytes // 4
    alg_bytes = 3 * nbytes
    # MPI_Init's share of the library's setup, before the application's data
    # exists (a program calls MPI_Init, builds its buffers, then reduces): the
    # direct path's HSA queue, code object and dispatch-id probe
    # (MPIR_Hip_direct_prepare) rather than inside the
    # first warm-up call
    lib.MPIR_Hip_direct_prepare(dev)
    g = torch.Generator(device="cuda").manual_seed(0x5EED + rank)
    # NPAIRS resident pairs, rotated, so no step finds its operands in the
    # 256 MB Infinity Cache (>= 3 pairs)
    # (SLACK bytes past each operand: the fresh-argument loop's offsets)
    pairs = [((torch.rand(count + SLACK // 4, device="cuda", generator=g) * 2 - 1),
              (torch.rand(count + SLACK // 4, device="cuda", generator=g) * 2 - 1)) for _ in range(NPAIRS)]
    ptrs = [(a.data_ptr(), b.data_ptr()) for a, b in pairs]
    sync()

    # MPI_Reduce_local from C, K calls back to back (the compiled binding's
    # reduce_local_loop, csrc/py/fastcall.c), as a C caller -- an MPICH
    # schedule, an OSU-style benchmark -- issues them; the same K calls stepped
    # from Python (one compiled call per step, the way mpi4py calls MPI, ~0.25 us
    # of Python each) are reported beside it (sync_variants.python_loop)
    try:
        reduce_local, c_loop = m.fast_reduce_local(), m.fast_reduce_local_loop()
        binding = "C loop of the compiled binding (csrc/py/fastcall.c reduce_local_loop)"
    except ImportError:     # extension not built: the same C entry point through ctypes
        reduce_local, c_loop, binding = lib.MPI_Reduce_local, None, "ctypes"
    own, calls, gap, bracket = [], [], [], []
    place_before = m.placement(dev)
    d_before = lib.MPIR_Hip_direct_dispatches()
    dt, dt_fresh, fresh_writes, step, dt_py = sync_loops(m, lib, reduce_local, ptrs, count, args.steps,
                                                         args.warmup, sync, barrier, max_over_ranks, own, c_loop,
                                                         calls, gap, bracket)
    # timed call i is step W + i: operand pair (W + i) % NPAIRS
    cstats = call_stats(calls, alg_bytes, [(args.warmup + i) % NPAIRS for i in range(len(calls))])
    if calls:
        # the first timed call follows the barrier and device syncs: the host
        # gap before it, and the call itself (the CP idles deeper after 50-100 us
        # without a doorbell, DESIGN.md "Idle gaps")
        cstats["first_call_us"] = round(calls[0] * 1e6, 2)
        if gap:
            cstats["idle_gap_before_first_us"] = round(gap[0] * 1e6, 1)
        if bracket:
            cstats["timed_region_outside_calls_us"] = round(bracket[0][0] * 1e6, 2)
            cstats["timed_region_closing_sync_us"] = round(bracket[0][1] * 1e6, 2)
            if time.get_clock_info("perf_counter").implementation.startswith("clock_gettime(CLOCK_MONOTONIC"):
                cstats["timed_region_loop_entry_us"] = round(bracket[0][2] * 1e6, 2)
                cstats["timed_region_loop_exit_us"] = round(bracket[0][3] * 1e6, 2)
            cstats["opening_sync_us"] = round(bracket[0][4] * 1e6, 2)      # before t0, outside the region
    direct_share = (lib.MPIR_Hip_direct_dispatches() - d_before) / ((3 if c_loop else 2) * (args.steps + args.warmup))
    value = alg_bytes * args.steps * world / dt / GIB
    # each rank's own figures beside the max-over-ranks `value`: a lagging GPU,
    # or a rank whose calls left the direct path, shows here
    # where the timed loop's thread ran, relative to the GPU
    place = placement_record(m, dev)
    rows = gather_rows([float(rank), float(dev), own[0], own[1], float(lib.MPIR_Hip_direct_state(dev)),
                        direct_share, cstats["median_us"], cstats["p10_us"], cstats["p90_us"],
                        cstats["slow_share"], float(place_before["cpu"]), float(place["cpu"]),
                        float(place["cpu_node"]), float(place["gpu_node"]), float(place["signal_node"]),
                        float(place["error_word_node"]), float(place["allowed_cpus"]),
                        float(place["ring_in_vram"])], world, dist,
                       "cpu" if pg_backend == "gloo" else "cuda")

    def rate(seconds):
        v = alg_bytes * args.steps * world / seconds / GIB
        return {"value": round(v, 1), "frac_of_hbm_peak": round(v / world * GIB / HBM_PEAK_BPS, 4),
                "ms_per_step": round(seconds / args.steps * 1e3, 4)}

    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (uniform [-1,1) fp32, seed 0x5EED+rank), device-resident",
        "config": {
            "workload": "MPI_Reduce_local MPI_SUM MPI_FLOAT, %d MiB per operand per GPU (count %d), "
                        "device-resident, one rank per GPU" % (args.mib, count),
            "count": count,
            "algorithmic_bytes_per_call": alg_bytes,
            "api": "MPI_Reduce_local (C ABI, synchronous; called through the " + binding + ")",
            "parallelism": "replica-per-gpu (no data-path collective)",
            "runtime": {"HSA_ALLOCATE_QUEUE_DEV_MEM": process_env("HSA_ALLOCATE_QUEUE_DEV_MEM"),
                        "HSA_ALLOCATE_QUEUE_DEV_MEM_in_job_environment": os.environ.get("HSA_ALLOCATE_QUEUE_DEV_MEM")},
            "process_group": pg_backend,
            # which sources the loaded binaries were built from (Makefile BUILD_ID)
            "build_id": m.build_id(),
        },
        "value_conditions": {
            "headline": "value",
            "environment": "as launched: the bench sets no runtime variable; HSA_ALLOCATE_QUEUE_DEV_MEM is the "
                           "library's load-time default (1) unless the job sets it (config.runtime)",
            "kernel_arguments": "%d rotating pairs: every call after the first %d repeats its arguments (kernarg "
                                "cache hit); sync_variants.fresh_args misses on every call" % (NPAIRS, NPAIRS),
            "caller": "K synchronous MPI_Reduce_local calls back to back from C (" + binding + "); "
                      "sync_variants.python_loop steps the same calls from Python",
            "placement": dict(bind, note="the timed calls' thread bound to the CPUs of its GPU's NUMA node "
                              "within the job's cpuset, as a launcher's -bind-to / --cpu-bind=closest would; "
                              "sync_variants.launch_placement: the same loop left where the process was launched "
                              "(BENCH_BIND=none)"),
            "warmup": "W untimed steps, the last of them after the barrier (BENCH_WARMUP_ORDER="
                      + os.environ.get("BENCH_WARMUP_ORDER", "late") + "), then a device sync and the K timed "
                      "steps: the first timed call does not pay the command processor's idle wake-up "
                      "(call_distribution.first_call_us, idle_gap_before_first_us)"},
        # the synchronous call per GPU (launch + completion included) against the HBM peak
        "per_gpu": {"GiBps": round(value / world, 1),
                    "frac_of_hbm_peak": round(value / world * GIB / HBM_PEAK_BPS, 4),
                    # the buffer rate count * sizeof(T) / t, for readability
                    "buffer_GiBps": round(value / world / 3, 1)},
        # every rank's own timed loop (value uses the slowest): seconds, rate,
        # direct-dispatch state and the share of its calls the direct path took
        "per_rank": [{"rank": int(r[0]), "device": int(r[1]), "seconds": round(r[2], 6),
                      "GiBps": round(alg_bytes * args.steps / r[2] / GIB, 1),
                      "frac_of_hbm_peak": round(alg_bytes * args.steps / r[2] / HBM_PEAK_BPS, 4),
                      "fresh_args_seconds": round(r[3], 6), "direct_state": int(r[4]),
                      "direct_share": round(r[5], 4),
                      "call_median_us": r[6], "call_p10_p90_us": [r[7], r[8]], "slow_share": r[9],
                      "placement": {"cpu_before_loop": int(r[10]), "cpu_after_loop": int(r[11]),
                                    "cpu_node": int(r[12]), "gpu_node": int(r[13]), "signal_node": int(r[14]),
                                    "error_word_node": int(r[15]), "allowed_cpus": int(r[16]),
                                    "ring_in_vram": int(r[17])}}
                     for r in rows],
        # rank 0's K timed calls, each on its own (clock stamps in the C loop)
        "call_distribution": dict(cstats, source="CLOCK_MONOTONIC after each call of the timed C loop (rank 0)"
                                  if c_loop else "perf_counter after each step of the timed loop (rank 0)"),
    }

    variants = {"fresh_args": dict(rate(dt_fresh), kernarg_writes_per_call=round(fresh_writes, 3),
                                   note="same loop, every call's arguments new (pairs shifted by multiples of "
                                        "256 B, 1024 distinct sets): kernarg BAR write + HDP flush per call")}
    if dt_py is not None:
        variants["python_loop"] = dict(rate(dt_py), note="the headline loop stepped from Python: one compiled-binding "
                                                         "call per step (mpi4py's way), timed after the C loops")
    if ring_variant is not None:
        if "dt" in ring_variant:
            variants["rocm_ring_placement"] = {
                "env": "HSA_ALLOCATE_QUEUE_DEV_MEM=0 (child process)",
                "cached_args": rate(ring_variant["dt"]), "fresh_args": rate(ring_variant["dt_fresh"]),
                "HSA_ALLOCATE_QUEUE_DEV_MEM_seen": ring_variant.get("HSA_ALLOCATE_QUEUE_DEV_MEM"),
                "ring_in_vram": (ring_variant.get("placement") or {}).get("ring_in_vram"),
                "direct_state": ring_variant.get("direct_state")}
        else:
            variants["rocm_ring_placement"] = ring_variant
    if launch_variant is not None:
        if "dt" in launch_variant:
            variants["launch_placement"] = dict(
                rate(launch_variant["dt"]), env="BENCH_BIND=none (child process): the calling thread where the "
                "process was launched", placement=launch_variant.get("placement"),
                fresh_args=rate(launch_variant["dt_fresh"]),
                HSA_ALLOCATE_QUEUE_DEV_MEM_seen=launch_variant.get("HSA_ALLOCATE_QUEUE_DEV_MEM"))
        else:
            variants["launch_placement"] = launch_variant
    out["sync_variants"] = variants

    if share:
        out["data"] = "REHEARSAL (BENCH_TEST_SHARE_GPU): %d ranks on %d GPU(s), not a measurement" % (
            world, torch.cuda.device_count())

    if not args.no_extras:
        # ---- roofline: the synchronous call's kernel, timed by the CP's dispatch
        # timestamps of the direct AQL path (what rocprofv3 reads); its
        # HIP-launched twin timed with HIP events on its stream as a second figure
        s = torch.cuda.Stream()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.steps)]
        with torch.cuda.stream(s):
            for i in range(args.warmup):
                pin, pio = ptrs[i % NPAIRS]
                lib.MPIX_Reduce_local_stream(pin, pio, count, m.MPI_FLOAT, m.MPI_SUM, s.cuda_stream)
            for i, (e0, e1) in enumerate(evs):
                pin, pio = ptrs[i % NPAIRS]
                e0.record(s)
                rc = lib.MPIX_Reduce_local_stream(pin, pio, count, m.MPI_FLOAT, m.MPI_SUM, s.cuda_stream)
                e1.record(s)
                assert rc == 0
        s.synchronize()
        ev_ms = sorted(e0.elapsed_time(e1) for e0, e1 in evs)
        ev_mean_us = sum(ev_ms) / len(ev_ms) * 1e3
        splits = []
        ns = direct_kernel_ns(lib, step, args.steps, args.warmup, splits)
        if ns is not None:
            us_sorted = sorted(x * 1e-3 for x in ns)
            kernel = ("mpir_tile_SUM_MPIR_HIP_F32 (the synchronous call's kernel, direct AQL dispatch, "
                      "reduce_tile<OpSum,float>)")
            timing = "mean of K CP dispatch timestamps (hsa_amd_profiling_get_dispatch_time) over K profiled repeats of the timed step"
        else:
            us_sorted = sorted(x * 1e3 for x in ev_ms)
            kernel = "mpir_hip::k_reduce_tile_lean<OpSum,float>"
            timing = "mean of K HIP-event brackets on the launch stream"
        mean_us = sum(us_sorted) / len(us_sorted)
        achieved = alg_bytes / (mean_us * 1e-6)
        traffic, tsrc = load_traffic(nbytes)
        out["roofline"] = {
            "bound": "hbm",
            "kernel": kernel,
            "achieved": round(achieved / 1e9, 1),
            "peak": HBM_PEAK_BPS / 1e9,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_BPS, 4),
            "traffic": traffic,
            "traffic_source": tsrc,
            "algorithmic_bytes_per_launch": alg_bytes,
            "mean_launch_us": round(mean_us, 2),
            "median_launch_us": round(us_sorted[len(us_sorted) // 2], 2),
            "p10_p90_us": [round(us_sorted[len(us_sorted) // 10], 2), round(us_sorted[(len(us_sorted) * 9) // 10], 2)],
            "timing": timing,
            "hip_launched_twin": {"kernel": "mpir_hip::k_reduce_tile_lean<OpSum,float>",
                                  "mean_launch_us_hip_events": round(ev_mean_us, 2),
                                  "frac": round(alg_bytes / (ev_mean_us * 1e-6) / HBM_PEAK_BPS, 4)},
        }
        # the synchronous call = kernel + a fixed cost (dispatch, completion,
        # host): what the kernel must reach for the call to reach 0.80
        call_mean_us = dt / args.steps * 1e6
        fixed = call_mean_us - mean_us
        out["call_distribution"]["decomposition"] = {
            "call_mean_us": round(call_mean_us, 2), "kernel_mean_us": round(mean_us, 2),
            "fixed_us": round(fixed, 2), "call_median_minus_kernel_median_us": round(
                cstats["median_us"] - us_sorted[len(us_sorted) // 2], 2),
            "kernel_us_for_call_at_0.80": round(alg_bytes / (0.8 * HBM_PEAK_BPS) * 1e6 - fixed, 2),
            "split_medians": split_medians(splits)}

        # ---- configs 2 and 3 (kernel time per synchronous call, same method)
        out["config3_sweep"] = config3_sweep(m, lib, pairs, nbytes, s)
        if nbytes >= 256 * MIB:
            out["config2_64MiB"] = config2(m, lib, pairs, s, args.steps, args.warmup)
            out["config5_combine"] = config5_combine(m, lib, s, args.steps, args.warmup)
            out["config4_combine"] = config4_combine(m, s, args.steps, args.warmup)

        # ---- stream-ordered API, back to back (what the library's schedules drive)
        def sstep(i):
            pin, pio = ptrs[i % NPAIRS]
            lib.MPIX_Reduce_local_stream(pin, pio, count, m.MPI_FLOAT, m.MPI_SUM, None)
        dts = time_steps(sstep, args.steps, args.warmup, sync, barrier, max_over_ranks)
        out["stream_api"] = {"value": round(alg_bytes * args.steps * world / dts / GIB, 1), "unit": "GiB/s",
                             "ms_per_step": round(dts / args.steps * 1e3, 4),
                             "api": "MPIX_Reduce_local_stream, synchronised once per K steps"}

        # ---- PCIe-inclusive: rank buffers in pinned host memory (PiP shm)
        ha = pairs[0][0].cpu().pin_memory()
        hb = pairs[0][1].cpu().pin_memory()
        hk = max(3, min(10, args.steps))

        def hstep(i):
            rc = lib.MPI_Reduce_local(hb.data_ptr(), ha.data_ptr(), count, m.MPI_FLOAT, m.MPI_SUM)
            assert rc == 0
        # pageable host memory (plain malloc'd / shm pages): through the pinned bounce slots
        pa = ha.numpy().copy()
        pb = hb.numpy().copy()

        def pstep(i):
            rc = lib.MPI_Reduce_local(pb.ctypes.data, pa.ctypes.data, count, m.MPI_FLOAT, m.MPI_SUM)
            assert rc == 0
        # both-host calls take the host combine by default (it beats the PCIe
        # round trip at every size, profiles/archive/r02/host_crossover.log); the
        # staging pipeline is forced here with a host limit of 0 so that the
        # PCIe-inclusive rate of the GPU path stays measured
        prev = lib.MPIR_Hip_set_host_max_bytes(0)
        try:
            dth = time_steps(hstep, hk, 1, sync, barrier, max_over_ranks)
            dtp = time_steps(pstep, hk, 1, sync, barrier, max_over_ranks)
            # the same pageable pages registered with hipHostRegister: how a PiP /
            # shm segment is pinned in place (SURVEY.md §8d host-inclusive rate),
            # through the library's own HIP runtime (not torch's bundled copy)
            hip = library_hip_runtime(lib)
            regd = []
            for arr in (pa, pb) if hip is not None else ():
                if hip.hipHostRegister(ctypes.c_void_p(arr.ctypes.data), ctypes.c_size_t(arr.nbytes), 0) == 0:
                    regd.append(arr)
            # every rank times the registered loop, or none does: its barrier and
            # max over ranks are collectives
            all_regd = max_over_ranks(0.0 if len(regd) == 2 else 1.0) == 0.0
            try:
                dtr = time_steps(pstep, hk, 1, sync, barrier, max_over_ranks) if all_regd else None
            finally:
                for arr in regd:
                    hip.hipHostUnregister(ctypes.c_void_p(arr.ctypes.data))
        finally:
            lib.MPIR_Hip_set_host_max_bytes(prev)
        out["pcie_inclusive"] = {"value": round(alg_bytes * hk * world / dth / GIB, 2), "unit": "GiB/s",
                                 "ms_per_step": round(dth / hk * 1e3, 3),
                                 "pageable_value": round(alg_bytes * hk * world / dtp / GIB, 2),
                                 "pageable_ms_per_step": round(dtp / hk * 1e3, 3),
                                 "registered_value": round(alg_bytes * hk * world / dtr / GIB, 2) if dtr else None,
                                 "registered_ms_per_step": round(dtr / hk * 1e3, 3) if dtr else None,
                                 "note": "host in/inout forced onto the GPU (host limit 0): 16 MiB chunks through "
                                         "the up (H2D x2) / comp / down (D2H) stream pipeline; pinned (hipHostMalloc) "
                                         "and registered (hipHostRegister'ed pageable pages) DMA'd directly, "
                                         "pageable via pinned bounce slots filled and drained by 4 copy threads"}
        # the default dispatch for the same host buffers: the host combine
        dhh = time_steps(hstep, hk, 1, sync, barrier, max_over_ranks)
        dhp = time_steps(pstep, hk, 1, sync, barrier, max_over_ranks)
        out["host_resident"] = {"value": round(alg_bytes * hk * world / dhh / GIB, 2), "unit": "GiB/s",
                                "ms_per_step": round(dhh / hk * 1e3, 3),
                                "pageable_value": round(alg_bytes * hk * world / dhp / GIB, 2),
                                "pageable_ms_per_step": round(dhp / hk * 1e3, 3),
                                "note": "same host buffers, default dispatch: combined on the host, split over "
                                        "the copy threads (SURVEY 8b: both operands host -> CPU)"}
        del ha, hb, pa, pb

    if coll is not None and rank == 0:
        out["collectives"] = coll

    # the CPU baseline on rank 0 at every N, after the GPU work, the other
    # ranks parked on a blocking store read (no spinning core beside it)
    unbind()
    if rank == 0 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(args, count, alg_bytes)
        except Exception as exc:        # noqa: BLE001  (the parked ranks must still be released)
            out["cpu_baseline"] = {"error": repr(exc)}
        if world > 1:
            out["cpu_baseline"]["ranks_parked"] = world - 1
    if not args.no_cpu_baseline:
        park_until_rank0(use_pg, world, rank, dist, "bench_cpu_baseline_done")
    if rank == 0:
        print(json.dumps(out), flush=True)
    if use_pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

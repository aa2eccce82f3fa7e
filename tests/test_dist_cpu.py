"""Multi-rank harness of bench.py on CPU (gloo, world_size 2).

bench.py's N > 1 path: one process per GPU, no data-path collective, a barrier
and device sync on both sides of exactly K timed steps, and the elapsed time
maxed over ranks.  Here the same `time_steps` runs in two gloo ranks with a
CPU step whose duration differs per rank, so the max-over-ranks and the
barrier bracketing are checked without a GPU.
"""
import os
import socket
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = []

    def step(i):
        calls.append(i)
        time.sleep(0.01 * (rank + 1))     # rank 1 is twice as slow

    def max_over_ranks(x):
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    dt = bench.time_steps(step, 5, 2, lambda: None, dist.barrier, max_over_ranks)
    q.put((rank, dt, calls))
    dist.destroy_process_group()


def test_time_steps_max_over_ranks_gloo():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    # every rank did W + K steps, in order, and all agree on the slowest rank's time
    for rank, dt, calls in res:
        assert calls == list(range(7))
    dts = [r[1] for r in res]
    assert dts[0] == pytest.approx(dts[1])
    assert dts[0] >= 5 * 0.02 * 0.95          # rank 1's 5 timed steps of 20 ms


def test_bench_defaults_parse():
    import sys
    import bench
    old = sys.argv
    try:
        sys.argv = ["bench.py"]
        a = bench.parse()
    finally:
        sys.argv = old
    assert a.gpus == 1 and a.steps > 0 and a.warmup >= 0 and a.mib == 256

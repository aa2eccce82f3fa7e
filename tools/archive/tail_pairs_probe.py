#!/usr/bin/env python3
"""Where do the headline loop's isolated slow kernels come from?  Per-call wall
time of the synchronous fp32 SUM at 256 MiB (compiled binding, direct dispatch)
against the number of rotating operand pairs and how they were allocated:
  sep   one torch tensor per operand (bench.py's layout)
  slab  every operand a view of one allocation (one contiguous VA range)
For each layout: the fraction of calls more than 4 us above the median, split by
pair index (a pair whose pages are placed badly would stand out), and the mean
excess the tail costs per call.
  python3 tools/tail_pairs_probe.py [calls per variant = 1500]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 1500
    import numpy as np
    import torch
    import mpich_pip_amd as m
    m.load()
    f = m.fast_reduce_local()
    count = 64 << 20
    alg = 3 * count * 4
    clk = time.perf_counter_ns
    variants = [("sep", 1), ("sep", 2), ("sep", 4), ("sep", 8), ("slab", 4), ("slab", 8)]
    for rnd in range(2):
        for kind, npairs in variants:
            if kind == "sep":
                bufs = [torch.empty(count, device="cuda") for _ in range(2 * npairs)]
            else:
                slab = torch.empty(2 * npairs * count, device="cuda")
                bufs = [slab[i * count:(i + 1) * count] for i in range(2 * npairs)]
            for b in bufs:
                b.uniform_(-1, 1)
            ptrs = [(bufs[2 * i].data_ptr(), bufs[2 * i + 1].data_ptr()) for i in range(npairs)]
            torch.cuda.synchronize()
            for i in range(40):
                pin, pio = ptrs[i % npairs]
                f(pin, pio, count, m.MPI_FLOAT, m.MPI_SUM)
            t = np.empty(calls, np.int64)
            for i in range(calls):
                pin, pio = ptrs[i % npairs]
                a = clk()
                f(pin, pio, count, m.MPI_FLOAT, m.MPI_SUM)
                t[i] = clk() - a
            us = t / 1e3
            med = float(np.median(us))
            slow = us > med + 4
            by_pair = [float(slow[k::npairs].mean()) for k in range(npairs)]
            excess = float(np.clip(us - med, 0, 30).mean())
            rate = alg / (us.mean() / 1e6) / 8e12
            print(f"round {rnd} {kind:4s} pairs {npairs}: median {med:.2f} us, mean {us.mean():.2f}, "
                  f"slow {slow.mean() * 100:.1f} % (by pair {' '.join(f'{x * 100:.1f}' for x in by_pair)}), "
                  f"excess/call (clipped 30) {excess:.2f} us, rate {rate:.4f} of 8 TB/s", flush=True)
            del bufs
            if kind == "slab":
                del slab
            torch.cuda.empty_cache()


if __name__ == "__main__" and not os.environ.get("MATRIX"):
    main()


def matrix(nbuf=8, reps=150):
    """Median call time for every ordered (inbuf, inoutbuf) pair of `nbuf`
    separately allocated 256 MiB operands: is a slow pair a property of one
    buffer or of the two buffers' relative placement?"""
    import numpy as np
    import torch
    import mpich_pip_amd as m
    m.load()
    f = m.fast_reduce_local()
    count = 64 << 20
    clk = time.perf_counter_ns
    bufs = [torch.empty(count, device="cuda").uniform_(-1, 1) for _ in range(nbuf)]
    torch.cuda.synchronize()
    print("buffers (VA, MiB offset from buffer 0):",
          " ".join(f"{i}:{(b.data_ptr() - bufs[0].data_ptr()) / 2**20:+.0f}" for i, b in enumerate(bufs)))
    med = np.zeros((nbuf, nbuf))
    for rnd in range(2):
        for i in range(nbuf):
            for j in range(nbuf):
                if i == j:
                    continue
                pin, pio = bufs[i].data_ptr(), bufs[j].data_ptr()
                for _ in range(10):
                    f(pin, pio, count, m.MPI_FLOAT, m.MPI_SUM)
                t = np.empty(reps)
                for k in range(reps):
                    a = clk()
                    f(pin, pio, count, m.MPI_FLOAT, m.MPI_SUM)
                    t[k] = (clk() - a) / 1e3
                med[i, j] = np.median(t)
        print(f"round {rnd}: median call time (us), row = inbuf, column = inoutbuf")
        for i in range(nbuf):
            print(f"  in {i}: " + " ".join("   -   " if i == j else f"{med[i, j]:7.2f}" for j in range(nbuf)), flush=True)


if __name__ == "__main__" and os.environ.get("MATRIX"):
    matrix()

#!/usr/bin/env python3
"""Kernel time of the synchronous fp32 SUM against the operands' address
alignment: both operands shifted by the same byte offset from a 2 MiB-aligned
base (the tile grid starts at inoutbuf, so the offset moves every 16 KiB tile
off the DRAM page / channel-interleave boundaries).  CP dispatch timestamps
(MPIR_Hip_direct_profile), NPAIRS pairs rotated past the Infinity Cache,
arguments repeated (kernarg-cache hits), variants interleaved per round.

    python3 tools/align_sweep.py [--mib 256] [--rounds 4] [--calls 40]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--calls", type=int, default=40)
    ap.add_argument("--offsets", default="0,64,256,1024,2048,4096,8192,16384,65536,1048576")
    args = ap.parse_args()
    import mpich_pip_amd as m
    lib = m.load()
    import torch
    f = m.fast_reduce_local()
    torch.cuda.set_device(0)
    offs = [int(x) for x in args.offsets.split(",")]
    n = args.mib << 18
    slack = (max(offs) + (2 << 20)) // 4
    npairs = 4
    pairs = [(torch.rand(n + slack, device="cuda"), torch.rand(n + slack, device="cuda")) for _ in range(npairs)]
    torch.cuda.synchronize()
    base = []
    for a, b in pairs:
        pa = (a.data_ptr() + (2 << 20) - 1) & ~((2 << 20) - 1)
        pb = (b.data_ptr() + (2 << 20) - 1) & ~((2 << 20) - 1)
        base.append((pb, pa))
    res = {o: [] for o in offs}
    lib.MPIR_Hip_direct_profile(1)
    for r in range(args.rounds):
        for o in (offs if r % 2 == 0 else offs[::-1]):
            for i in range(8 + args.calls):
                pb, pa = base[i % npairs]
                assert f(pb + o, pa + o, n, m.MPI_FLOAT, m.MPI_SUM) == 0
                if i >= 8:
                    res[o].append(lib.MPIR_Hip_direct_last_kernel_ns() * 1e-3)
    lib.MPIR_Hip_direct_profile(0)
    alg = 3 * n * 4
    for o in offs:
        xs = sorted(res[o])
        med = xs[len(xs) // 2]
        print(f"offset {o:8d} B  kernel median {med:8.2f} us  p10 {xs[len(xs) // 10]:8.2f}  p90 "
              f"{xs[len(xs) * 9 // 10]:8.2f}  frac {alg / (med * 1e-6) / 8e12:.4f}", flush=True)


if __name__ == "__main__":
    main()

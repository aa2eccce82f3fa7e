#!/usr/bin/env python3
"""Config 2 under rocprofv3: K synchronous fp32 SUM MPI_Reduce_local calls at
64 MiB per operand over bench.py's 16 windows (four 256 MiB pairs, 2 GiB of
footprint, so no call re-reads anything from the Infinity Cache).

    rocprofv3 --pmc FETCH_SIZE -- python3 tools/config2_pmc.py [--k 32]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))
os.environ.setdefault("HSA_ALLOCATE_QUEUE_DEV_MEM", "1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=32)
    args = ap.parse_args()
    import torch
    import mpich_pip_amd as m
    f = m.fast_reduce_local()
    count = 16 << 20
    g = torch.Generator(device="cuda").manual_seed(0x5EED)
    pairs = [(torch.rand(4 * count, device="cuda", generator=g), torch.rand(4 * count, device="cuda", generator=g))
             for _ in range(4)]
    torch.cuda.synchronize()
    wins = [(b.data_ptr() + j * count * 4, a.data_ptr() + j * count * 4) for a, b in pairs for j in range(4)]
    for i in range(args.k + 4):
        pin, pio = wins[i % len(wins)]
        assert f(pin, pio, count, m.MPI_FLOAT, m.MPI_SUM) == 0
    print("config2 calls:", args.k + 4, flush=True)


if __name__ == "__main__":
    main()

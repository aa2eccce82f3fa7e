#!/usr/bin/env python3
"""Fused schedule combines (MPIX_Reduce_local_multi) per (op, type, n, order):
kernel time per launch (HIP events on the launch stream, median of 7 after 3
warm-ups) as a fraction of the 8 TB/s HBM peak, algorithmic bytes (n + 1) x
block.  The (op, type) pairs the collectives use most run k_combine_multi;
the rest run the general one-pass k_combine_any.

    python tools/multi_sweep.py [block MiB]     (on the GPU box; default 32 = config 4's block)

Two operand sets alternate, so no launch finds the previous one's lines in
the Infinity Cache (n x block x 2 >= 512 MiB at the default).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpich-pip_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "tools")]

import torch  # noqa: E402

import _types as T  # noqa: E402
import mpich_pip_amd as m  # noqa: E402
from op_type_sweep import fill  # noqa: E402

PEAK = 8.0e12
CASES = [
    ("MPI_FLOAT", "MPI_SUM"), ("MPIX_C_FLOAT16", "MPI_SUM"), ("MPI_INT", "MPI_MAX"),
    ("MPI_DOUBLE", "MPI_MIN"),
    # k_combine_any
    ("MPI_2INT", "MPI_MAXLOC"), ("MPI_DOUBLE_INT", "MPI_MINLOC"), ("MPI_FLOAT_INT", "MPI_MAXLOC"),
    ("MPI_INT", "MPI_LAND"), ("MPI_LONG", "MPI_BXOR"), ("MPI_SHORT", "MPI_SUM"),
    ("MPI_UNSIGNED_CHAR", "MPI_BOR"), ("MPI_C_FLOAT_COMPLEX", "MPI_PROD"),
    ("MPI_C_DOUBLE_COMPLEX", "MPI_PROD"), ("MPI_LONG_DOUBLE", "MPI_SUM"),
]


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    block = mib << 20
    lib = m.load()
    lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN)
    nmax = 8
    sets = [[torch.empty(block, dtype=torch.uint8, device="cuda") for _ in range(nmax + 1)] for _ in range(2)]
    s = torch.cuda.Stream()
    for t, op in CASES:
        esz = T.elem_size(t)
        count = block // esz
        for k, st in enumerate(sets):
            for j, b in enumerate(st):
                fill(b, t, op, 100 * k + j)
        torch.cuda.synchronize()
        for n in (2, 8):
            for order, oname in ((m.MPIX_ORDER_TREE, "tree"), (m.MPIX_ORDER_CHAIN, "chain")):
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(7)]
                with torch.cuda.stream(s):
                    for i in range(10):
                        st = sets[i & 1]
                        ins = [b.data_ptr() for b in st[:n]]
                        if i >= 3:
                            ev[i - 3][0].record(s)
                        rc = m.reduce_local_multi(ins, st[nmax].data_ptr(), count, m.DATATYPES[t], m.OPS[op],
                                                  order, s.cuda_stream)
                        assert rc == 0, (t, op, n, m.error_string(rc))
                        if i >= 3:
                            ev[i - 3][1].record(s)
                s.synchronize()
                ms = sorted(a.elapsed_time(b) for a, b in ev)
                us = ms[len(ms) // 2] * 1e3
                frac = (n + 1) * block / (us * 1e-6) / PEAK
                print(f"{t:24s} {op:11s} n={n} {oname:5s} {us:9.2f} us  frac {frac:.3f}", flush=True)


if __name__ == "__main__":
    main()

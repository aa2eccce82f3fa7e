#!/usr/bin/env python3
"""Every (op, basic type) the reference accepts, at 256 MiB per operand, through
MPIX_Reduce_local_stream: kernel time per launch (HIP events on the launch
stream, median of 7 after 3 warm-ups) as a fraction of the 8 TB/s HBM peak.

    python tools/op_type_sweep.py [MiB]     (on the GPU box)

Operands: seeded random finite values (floats uniform in [-1, 1) or [0.5, 1.5)
for PROD, integers over their range); two operand pairs alternate so no launch
finds the previous one's lines in the Infinity Cache.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpich-pip_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import _types as T  # noqa: E402
import mpich_pip_amd as m  # noqa: E402

PEAK = 8.0e12


def fill(buf, t, op, seed):
    """Random finite operand bytes generated on the device (torch), viewed as type t."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    n = buf.numel()
    if t in ("MPI_FLOAT", "MPI_C_FLOAT_COMPLEX", "MPI_FLOAT_INT"):
        v = torch.rand(n // 4, generator=g, device="cuda")
        v = v + 0.5 if op == "MPI_PROD" else v * 2 - 1
        buf.view(torch.float32).copy_(v)
    elif t in ("MPI_DOUBLE", "MPI_C_DOUBLE_COMPLEX", "MPI_DOUBLE_INT"):
        v = torch.rand(n // 8, generator=g, device="cuda", dtype=torch.float64)
        v = v + 0.5 if op == "MPI_PROD" else v * 2 - 1
        buf.view(torch.float64).copy_(v)
    elif t == "MPIX_C_FLOAT16":
        v = torch.rand(n // 2, generator=g, device="cuda")
        v = v + 0.5 if op == "MPI_PROD" else v * 2 - 1
        buf.view(torch.float16).copy_(v.half())
    elif t in ("MPI_LONG_DOUBLE", "MPI_C_LONG_DOUBLE_COMPLEX", "MPI_LONG_DOUBLE_INT"):
        # x87 values in [1, 2): random 63-bit fraction, explicit integer bit, exponent 0x3fff
        w = buf.view(torch.int64).view(-1, 2)
        w[:, 0] = torch.randint(0, 2 ** 62, (w.shape[0],), generator=g, device="cuda") | -(2 ** 63)
        w[:, 1] = 0x3FFF
    else:
        buf.copy_(torch.randint(0, 256, (n,), generator=g, device="cuda", dtype=torch.uint8))


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    nbytes = mib << 20
    lib = m.load()
    lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN)
    bufs = [torch.empty(nbytes, dtype=torch.uint8, device="cuda") for _ in range(4)]
    s = torch.cuda.Stream()
    rows = []
    for t in T.ALL_TYPES:
        esz = T.elem_size(t)
        ops = [op for op in T.OPS if T.compute_ok(op, t)]
        if not ops:
            continue
        for op in ops:
            for k, b in enumerate(bufs):
                fill(b, t, op, 1000 + k)
            torch.cuda.synchronize()
            count = nbytes // esz
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(7)]
            with torch.cuda.stream(s):
                for i in range(10):
                    io, inp = bufs[2 * (i & 1)], bufs[2 * (i & 1) + 1]
                    if i >= 3:
                        ev[i - 3][0].record(s)
                    rc = lib.MPIX_Reduce_local_stream(inp.data_ptr(), io.data_ptr(), count, m.DATATYPES[t],
                                                      m.OPS[op], s.cuda_stream)
                    assert rc == 0, (t, op, m.error_string(rc))
                    if i >= 3:
                        ev[i - 3][1].record(s)
            s.synchronize()
            ms = sorted(a.elapsed_time(b) for a, b in ev)
            us = ms[len(ms) // 2] * 1e3
            frac = 3 * nbytes / (us * 1e-6) / PEAK
            rows.append((t, op, us, frac))
            print(f"{t:28s} {op:11s} {us:9.2f} us  frac {frac:.3f}", flush=True)
    fr = [r[3] for r in rows]
    print(f"{len(rows)} (op, type) pairs at {mib} MiB: frac min {min(fr):.3f} median {sorted(fr)[len(fr) // 2]:.3f} "
          f"max {max(fr):.3f}")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Stress of the synchronous paths: T host threads, each issuing a long mix of
calls -- direct-dispatch shapes, HIP-launch shapes (ragged counts, ops outside
the code object), the stream variant followed by a synchronous call, small
host and mixed-residency calls -- and checking every result against numpy.
Meant to flush out rare hangs or races before they reach a round-end run.

    timeout 300 python3 tools/stress_direct.py [--threads 4] [--iters 2000]
"""
import argparse
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))
os.environ.setdefault("HSA_ALLOCATE_QUEUE_DEV_MEM", "1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--iters", type=int, default=2000)
    args = ap.parse_args()
    import torch
    import mpich_pip_amd as m
    lib = m.load()
    lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN)
    f = m.fast_reduce_local()
    F, I, S, X = m.MPI_FLOAT, m.MPI_INT, m.MPI_SUM, m.MPI_BXOR
    errors = []
    d0 = lib.MPIR_Hip_direct_dispatches()

    def worker(k):
        rng = np.random.default_rng(1000 + k)
        sizes = [16, 4096, 65536, (1 << 20), 4099, 7]
        for it in range(args.iters):
            n = sizes[it % len(sizes)]
            kind = (it // len(sizes)) % 4
            a = rng.uniform(-1, 1, n).astype(np.float32)
            b = rng.uniform(-1, 1, n).astype(np.float32)
            want = a + b
            if kind == 0:                       # device, fp32 SUM (direct when aligned)
                da, db = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
                torch.cuda.current_stream().synchronize()
                rc = f(db.data_ptr(), da.data_ptr(), n, F, S)
                got = da.cpu().numpy()
            elif kind == 1:                     # device, int BXOR (HIP launch)
                ai = rng.integers(0, 1 << 30, n, dtype=np.int32)
                bi = rng.integers(0, 1 << 30, n, dtype=np.int32)
                want = ai ^ bi
                da, db = torch.from_numpy(ai).cuda(), torch.from_numpy(bi).cuda()
                torch.cuda.current_stream().synchronize()
                rc = f(db.data_ptr(), da.data_ptr(), n, I, X)
                got = da.cpu().numpy()
            elif kind == 2:                     # stream variant, then a synchronous call
                da, db = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
                torch.cuda.current_stream().synchronize()
                rc = m.reduce_local_stream(db.data_ptr(), da.data_ptr(), n, F, S, 0)
                if rc == 0:
                    rc = f(db.data_ptr(), da.data_ptr(), n, F, S)
                want = (a + b) + b
                got = da.cpu().numpy()
            else:                               # mixed: host in, device inout
                da = torch.from_numpy(a).cuda()
                torch.cuda.current_stream().synchronize()
                rc = f(b.ctypes.data, da.data_ptr(), n, F, S)
                got = da.cpu().numpy()
            if rc != 0:
                errors.append((k, it, "rc", rc))
                return
            if not np.array_equal(got, want):
                errors.append((k, it, "mismatch", n, kind))
                return

    t0 = time.time()
    th = [threading.Thread(target=worker, args=(k,)) for k in range(args.threads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.time() - t0
    print(f"threads {args.threads} x {args.iters} calls in {dt:.1f} s; direct dispatches "
          f"{lib.MPIR_Hip_direct_dispatches() - d0}; errors {errors[:5]}", flush=True)
    sys.exit(1 if errors else 0)


if __name__ == "__main__":
    main()

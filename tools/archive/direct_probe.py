#!/usr/bin/env python3
"""Probe of the direct AQL dispatch's preconditions and kernel timestamps.

    python3 tools/direct_probe.py

Prints, step by step: whether each synchronous call went direct (dispatch
counter), the null-stream-busy skip counter, and the kernel ns reported
with profiling on -- after torch work on the null stream with and without a
synchronize, and after sleeping.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))


def main():
    import torch
    import mpich_pip_amd as m
    lib = m.load()
    f = m.fast_reduce_local()
    F, S = m.MPI_FLOAT, m.MPI_SUM
    n = 16 << 20
    a = torch.rand(n, device="cuda")
    b = torch.rand(n, device="cuda")

    def call(tag):
        d0, s0 = lib.MPIR_Hip_direct_dispatches(), lib.MPIR_Hip_direct_busy_skips()
        t0 = time.perf_counter()
        assert f(b.data_ptr(), a.data_ptr(), n, F, S) == 0
        us = (time.perf_counter() - t0) * 1e6
        print(f"{tag:<34} {us:8.1f} us direct {lib.MPIR_Hip_direct_dispatches() - d0} skip {lib.MPIR_Hip_direct_busy_skips() - s0} "
              f"ns {lib.MPIR_Hip_direct_last_kernel_ns()} state {lib.MPIR_Hip_direct_state(0)}", flush=True)

    call("after rand, no sync")
    call("second")
    time.sleep(0.2)
    call("after 0.2 s sleep")
    torch.cuda.synchronize()
    call("after synchronize")
    call("again")
    lib.MPIR_Hip_direct_profile(1)
    call("profile on (1)")
    call("profile on (2)")
    call("profile on (3)")
    c = torch.rand(n, device="cuda")
    call("after another rand, no sync")
    time.sleep(0.2)
    call("after 0.2 s sleep")
    torch.cuda.synchronize()
    call("after synchronize")
    lib.MPIR_Hip_direct_profile(0)
    call("profile off")
    for r in range(3):
        torch.rand(n, device="cuda", out=c)
        call(f"rand then call ({r})")
    del c


if __name__ == "__main__":
    main()

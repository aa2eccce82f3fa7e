#!/usr/bin/env python3
"""What does a kernarg write that loses the race to the CP cost?  The
synchronous fp32 SUM call at 256 MiB with new arguments on every call (every
call a kernarg-cache miss: checked kernel, slot written after the doorbell),
with the test hook moving each write behind the doorbell, D us late
(MPIR_Hip_direct_test_write_delay_us), so that the first workgroups find the
slot stale and poll for it; D = 0 is the product's write before the doorbell.  Ideal cost
of a delay: max(0, D - (doorbell -> dispatch ~4.3 us)); anything above that is
the polling's own overhead.  Rounds alternate the delays; means per call.
  python3 tools/late_write_probe.py [calls per point = 200] [rounds = 3]
"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    import numpy as np
    import mpich_pip_amd as m
    lib = m.load()
    lib.MPIR_Hip_direct_test_write_delay_us.restype = ctypes.c_uint32
    lib.MPIR_Hip_direct_test_write_delay_us.argtypes = [ctypes.c_uint32]
    import torch
    count = 64 << 20
    slack = 1 << 16
    pairs = [(torch.rand(count + slack, device="cuda"), torch.rand(count + slack, device="cuda")) for _ in range(4)]
    torch.cuda.synchronize()
    sets = [(b.data_ptr() + o, a.data_ptr() + o) for o in range(0, slack * 4, 256) for a, b in pairs]
    f = m.fast_reduce_local()
    pos = 0
    res = {}
    delays = (0, 2, 4, 6, 10, 20)
    for r in range(rounds):
        for d in delays:
            lib.MPIR_Hip_direct_test_write_delay_us(d)
            t = []
            for i in range(calls + 10):
                pin, pio = sets[pos % len(sets)]
                pos += 1
                a = time.perf_counter_ns()
                f(pin, pio, count, m.MPI_FLOAT, m.MPI_SUM)
                if i >= 10:
                    t.append((time.perf_counter_ns() - a) / 1e3)
            res.setdefault(d, []).append(float(np.mean(t)))
            print(f"round {r} delay {d}: {np.mean(t):.2f} us", flush=True)
    lib.MPIR_Hip_direct_test_write_delay_us(0)
    base = min(res[0])
    for d in delays:
        v = res[d]
        print(f"write held back {d:3d} us: mean call {min(v):8.2f} .. {max(v):8.2f} us; over no delay "
              f"{min(v) - base:+6.2f} us (ideal {max(0.0, d - 4.3):+5.1f})", flush=True)


if __name__ == "__main__":
    main()

"""The two-operand tile kernel with inbuf and inoutbuf carved from one
allocation at a chosen distance (round 5).  MPICH's schedules reduce
sub-ranges of one buffer (recvbuf + disps[i] * extent, tmp_buf halves) that
often sit a power of two apart; separately allocated operands sit wherever the
allocator put them.  If HBM channel selection gives two operands at a
power-of-two distance the same channels at the same moment, the synchronous
call slows down the way the multi-operand folds did at an unskewed stride.

    python tools/archive/pair_offset.py [calls = 200]

fp32 SUM, 256 MiB per operand, the synchronous MPI_Reduce_local (direct
dispatch); kernel time from the CP timestamps (MPIR_Hip_direct_profile), the
median over `calls`; layouts interleaved over 3 rounds, each on fresh values
(the inout accumulates b, finite).
"""
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpich-pip_amd")]

import torch  # noqa: E402
import mpich_pip_amd as m  # noqa: E402

MIB = 1 << 20


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    lib = m.load()
    lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN)
    torch.cuda.set_device(0)
    lib.MPIR_Hip_direct_prepare(0)
    count = 64 * MIB                        # floats: 256 MiB
    nb = count * 4
    # one slab large enough for every distance below, plus separate buffers
    slab = torch.empty((nb * 3 + 4 * MIB) // 4, device="cuda").uniform_(-1, 1)
    sep_a = torch.empty(count, device="cuda").uniform_(-1, 1)
    sep_b = torch.empty(count, device="cuda").uniform_(-1, 1)
    base = slab.data_ptr()
    base = (base + 2 * MIB - 1) // (2 * MIB) * (2 * MIB)
    layouts = {"separate allocations": (sep_b.data_ptr(), sep_a.data_ptr())}
    for name, d in (("one slab, 256 MiB apart", nb), ("one slab, 256 MiB + 4352 B", nb + 4352),
                    ("one slab, 256 MiB + 2 MiB", nb + 2 * MIB), ("one slab, 512 MiB apart", 2 * nb),
                    ("one slab, 256 MiB + 64 KiB", nb + 64 * 1024)):
        layouts[name] = (base, base + d)
    for name, (pin, pio) in layouts.items():
        assert pio + nb <= slab.data_ptr() + slab.numel() * 4 or name.startswith("separate"), name
    torch.cuda.synchronize()
    lib.MPIR_Hip_direct_profile(1)
    res = {k: [] for k in layouts}
    for r in range(3):
        for name, (pin, pio) in layouts.items():
            for i in range(calls + 5):
                rc = lib.MPI_Reduce_local(ctypes.c_void_p(pin), ctypes.c_void_p(pio), count, m.MPI_FLOAT, m.MPI_SUM)
                assert rc == 0, m.error_string(rc)
                if i >= 5:
                    res[name].append(lib.MPIR_Hip_direct_last_kernel_ns() * 1e-3)
    lib.MPIR_Hip_direct_profile(0)
    for name, v in res.items():
        med = statistics.median(v)
        print(f"{name:32s} kernel median {med:8.2f} us  (p10 {sorted(v)[len(v) // 10]:.2f}, "
              f"p90 {sorted(v)[9 * len(v) // 10]:.2f})  frac of 8 TB/s {3 * nb / (med * 1e-6) / 8e12:.4f}", flush=True)


if __name__ == "__main__":
    main()

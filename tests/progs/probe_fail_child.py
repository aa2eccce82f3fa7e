"""Child of tests/test_direct_prepare_gpu.py::test_first_profiled_call_after_failed_probe
(ADVICE r3, medium): the probe of the timestamped twin queue, made inside the
first profiled call, reports (through MPIR_Hip_direct_test_fail_probe) that
dispatch ids are not packet indices.  That call must already follow the
read-back protocol it switched to -- complete, bit-exact, direct state 2 --
and so must the profiled and unprofiled calls after it, with fresh and with
repeated arguments.  Prints one JSON line."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))


def main():
    import mpich_pip_amd as m
    lib = m.load()
    assert lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN) == 0
    lib.MPIR_Hip_direct_dispatches.restype = ctypes.c_uint64
    lib.MPIR_Hip_direct_last_kernel_ns.restype = ctypes.c_uint64
    import torch
    torch.cuda.set_device(0)
    n = (1 << 22) + 5
    a0 = torch.rand(n + 64, device="cuda")
    b = torch.rand(n + 64, device="cuda")
    torch.cuda.synchronize()
    f = m.fast_reduce_local()
    out = {"state_before": lib.MPIR_Hip_direct_prepare(0), "calls": []}
    lib.MPIR_Hip_direct_test_fail_probe()
    d0 = lib.MPIR_Hip_direct_dispatches()
    ok = True
    # profiled (twin queue: the failing probe runs inside the first call), then
    # the calls' own queue; offsets give fresh arguments, repeats cache hits.
    # Small counts (grids of 1-7 workgroups, padded to span every XCD on a
    # miss, read-back mode included: ADVICE r4) fresh and repeated
    for prof in (1, 1, 1, 0, 0, 0, 0):
        lib.MPIR_Hip_direct_profile(prof)
        for cnt, off in ((n, 0), (n, 3), (n, 0), (3001, 0), (3001, 0), (77, 1), (77, 1), (4096 * 5, 2)):
            a = a0.clone()
            torch.cuda.synchronize()
            rc = f(b.data_ptr() + 4 * off, a.data_ptr() + 4 * off, cnt, m.MPI_FLOAT, m.MPI_SUM)
            want = a0.clone()
            want[off:off + cnt] += b[off:off + cnt]
            good = rc == 0 and bool(torch.equal(a, want))
            ok &= good
            out["calls"].append([prof, off, rc, good, int(lib.MPIR_Hip_direct_last_kernel_ns()) if prof else None])
    lib.MPIR_Hip_direct_profile(0)
    out.update(ok=ok, direct=int(lib.MPIR_Hip_direct_dispatches() - d0), state_after=lib.MPIR_Hip_direct_state(0))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

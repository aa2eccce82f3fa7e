"""Child of tests/test_direct_timeout_gpu.py: a kernarg slot that never lands
in time.  The test hook moves the kernarg write behind the doorbell, 2.2 s late, past
the checked kernel's 2 s wait, for a 64 MiB fp32 SUM (4,096 workgroups: two
resident rounds).  The first round gives up and sets the error word; the second
round starts after that and must give up at once rather than combine the
arguments that land 0.2 s later.  Expected: the call fails with MPI_ERR_OTHER
and leaves inoutbuf untouched, and the next call takes the HIP path (the
direct path closes), bit-exact.  Prints one JSON line."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))


def main():
    import mpich_pip_amd as m
    lib = m.load()
    assert lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN) == 0
    lib.MPIR_Hip_direct_test_write_delay_us.restype = ctypes.c_uint32
    lib.MPIR_Hip_direct_test_write_delay_us.argtypes = [ctypes.c_uint32]
    lib.MPIR_Hip_direct_dispatches.restype = ctypes.c_uint64
    import torch
    torch.cuda.set_device(0)
    n = 16 << 20
    a0 = torch.rand(n + 4096, device="cuda")
    b = torch.rand(n + 4096, device="cuda")
    a = a0.clone()
    torch.cuda.synchronize()
    out = {}
    # a normal call first: the direct path is up, in nonce mode
    rc = m.reduce_local(b.data_ptr(), a.data_ptr(), n, m.MPI_FLOAT, m.MPI_SUM)
    out["warm_ok"] = rc == 0 and bool(torch.equal(a[:n], a0[:n] + b[:n]))
    out["state"] = lib.MPIR_Hip_direct_state(0)
    a.copy_(a0)
    torch.cuda.synchronize()
    d0 = lib.MPIR_Hip_direct_dispatches()
    lib.MPIR_Hip_direct_test_write_delay_us(2200000)
    t0 = time.perf_counter()
    rc = m.reduce_local(b[64:].data_ptr(), a[64:].data_ptr(), n, m.MPI_FLOAT, m.MPI_SUM)   # new arguments
    out["failed_call_s"] = round(time.perf_counter() - t0, 3)
    lib.MPIR_Hip_direct_test_write_delay_us(0)
    out["failed_rc_class"] = m.error_class(rc) if rc else 0
    torch.cuda.synchronize()
    out["untouched"] = bool(torch.equal(a, a0))
    # the next call: HIP path, exact
    d1 = lib.MPIR_Hip_direct_dispatches()
    rc = m.reduce_local(b[128:].data_ptr(), a[128:].data_ptr(), n, m.MPI_FLOAT, m.MPI_SUM)
    torch.cuda.synchronize()
    out["after_ok"] = rc == 0 and bool(torch.equal(a[128:128 + n], a0[128:128 + n] + b[128:128 + n]))
    out["after_direct"] = int(lib.MPIR_Hip_direct_dispatches() - d1)
    out["failed_direct"] = int(d1 - d0)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

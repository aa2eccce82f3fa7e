"""Child of tests/test_direct_prepare_gpu.py: in a fresh process, time the
first synchronous MPI_Reduce_local (fp32 SUM, 4 Mi floats, device operands)
with and without MPIR_Hip_direct_prepare() beforehand (argv[1] = 1 / 0), and
check it bit-exact against torch's fp32 add.  Prints one JSON line."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))


def main():
    prepare = sys.argv[1] == "1"
    import mpich_pip_amd as m
    lib = m.load()
    assert lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN) == 0
    lib.MPIR_Hip_direct_dispatches.restype = ctypes.c_uint64
    import torch
    torch.cuda.set_device(0)
    n = 4 << 20
    a0 = torch.rand(n, device="cuda")
    a = a0.clone()
    b = torch.rand(n, device="cuda")
    torch.cuda.synchronize()
    out = {"prepare": prepare}
    if prepare:
        t0 = time.perf_counter()
        out["prepare_state"] = lib.MPIR_Hip_direct_prepare(0)
        out["prepare_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
    f = m.fast_reduce_local()
    t0 = time.perf_counter()
    rc = f(b.data_ptr(), a.data_ptr(), n, m.MPI_FLOAT, m.MPI_SUM)
    out["first_call_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
    out["ok"] = rc == 0 and bool(torch.equal(a, a0 + b))
    out["direct"] = int(lib.MPIR_Hip_direct_dispatches())
    out["state"] = lib.MPIR_Hip_direct_state(0)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

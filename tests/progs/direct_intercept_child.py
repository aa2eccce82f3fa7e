"""Child of tests/test_direct_intercept_gpu.py, run under rocprofv3
--kernel-trace (a tool that intercepts the library's AQL queue): synchronous
fp32 SUM calls through the direct dispatch with fresh arguments on every call
(kernarg-cache misses), then repeated arguments (hits), each result compared
bit for bit with torch's fp32 add of the same operands.  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))


def main():
    import mpich_pip_amd as m
    lib = m.load()
    assert lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN) == 0
    import torch
    torch.cuda.set_device(0)
    n = (1 << 20) + 3
    a0 = torch.rand(n + 4096, device="cuda")
    b = torch.rand(n + 4096, device="cuda")
    a = a0.clone()
    torch.cuda.synchronize()
    d0 = lib.MPIR_Hip_direct_dispatches()
    bad, calls = 0, 0
    # fresh arguments: a different element offset (and count) every call
    for i in range(48):
        off, cnt = (i * 37) % 4096, n - (i % 7)
        rc = m.reduce_local(b[off:].data_ptr(), a[off:].data_ptr(), cnt, m.MPI_FLOAT, m.MPI_SUM)
        calls += 1
        want = a0[off:off + cnt] + b[off:off + cnt]
        if rc != 0 or not torch.equal(a[off:off + cnt], want):
            bad += 1
        a.copy_(a0)
        torch.cuda.synchronize()
    # repeated arguments: kernarg-cache hits after the first
    for i in range(6):
        rc = m.reduce_local(b.data_ptr(), a.data_ptr(), n, m.MPI_FLOAT, m.MPI_SUM)
        calls += 1
        if rc != 0 or not torch.equal(a[:n], a0[:n] + b[:n]):
            bad += 1
        a.copy_(a0)
        torch.cuda.synchronize()
    print(json.dumps({"state": lib.MPIR_Hip_direct_state(0), "bad": bad, "calls": calls,
                      "direct": lib.MPIR_Hip_direct_dispatches() - d0}), flush=True)


if __name__ == "__main__":
    main()

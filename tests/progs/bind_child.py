"""Child of tests/test_bind_gpu.py: one synchronous device-resident
MPI_Reduce_local with MPIR_CVAR_REDUCE_LOCAL_BIND as the parent set it; prints
the calling thread's affinity before and after, and its placement.
BIND_CHILD_CALLS=n makes it n calls in a row (b += a each time)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "mpich-pip_amd"))
import mpich_pip_amd as m  # noqa: E402

lib = m.load()
import torch  # noqa: E402

lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN)
torch.cuda.set_device(0)
a = torch.ones(1 << 20, device="cuda")
b = torch.ones(1 << 20, device="cuda")
torch.cuda.synchronize()
before = sorted(os.sched_getaffinity(0))
calls = int(os.environ.get("BIND_CHILD_CALLS", "1"))
rc = 0
for _ in range(calls):
    rc = rc or m.reduce_local(a.data_ptr(), b.data_ptr(), 1 << 20, m.MPI_FLOAT, m.MPI_SUM)
after = sorted(os.sched_getaffinity(0))
ok = bool(torch.all(b == 1 + calls).item())
print(json.dumps({"rc": rc, "ok": ok, "before": before, "after": after, "placement": m.placement(0),
                  "direct": lib.MPIR_Hip_direct_dispatches()}))

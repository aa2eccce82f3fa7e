import os, sys, time, json
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "mpich-pip_amd"))
import numpy as np
import mpich_pip_amd as m
lib = m.load()
n = 64 << 20
a = np.random.default_rng(1).random(n, dtype=np.float32)
b = np.random.default_rng(2).random(n, dtype=np.float32)
def run(tag, a, b, k=8):
    assert lib.MPI_Reduce_local(b.ctypes.data, a.ctypes.data, n, m.MPI_FLOAT, m.MPI_SUM) == 0
    t0 = time.perf_counter()
    for _ in range(k):
        assert lib.MPI_Reduce_local(b.ctypes.data, a.ctypes.data, n, m.MPI_FLOAT, m.MPI_SUM) == 0
    dt = (time.perf_counter() - t0) / k
    print(tag, "%.2f ms %.1f GiB/s" % (dt * 1e3, 3 * n * 4 / dt / 2**30), flush=True)
run("numpy random (no torch)", a, b)
import torch
x = torch.rand(n, device="cuda"); torch.cuda.synchronize()
run("after torch init", a, b)
ha = x.cpu().pin_memory(); pa = ha.numpy().copy(); pb = ha.numpy().copy()
run("arrays from pinned-tensor copy", pa, pb)
run("numpy random again", a, b)

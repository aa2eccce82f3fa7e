import os, sys, time
sys.path.insert(0, "/root/repo/mpich-pip_amd")
os.environ.setdefault("HSA_ALLOCATE_QUEUE_DEV_MEM", "1")
import torch
import mpich_pip_amd as m
lib = m.load(); fast = m.fast_reduce_local()
n = 16 << 20
pairs = [(torch.rand(n, device="cuda"), torch.rand(n, device="cuda")) for _ in range(4)]
torch.cuda.synchronize()
args = [(b.data_ptr(), a.data_ptr(), n, m.MPI_FLOAT, m.MPI_SUM) for a, b in pairs]
def ntasks(): return len(os.listdir("/proc/self/task"))
print("threads before", ntasks(), "KA", os.environ.get("MPIR_CVAR_REDUCE_LOCAL_KEEPALIVE_US"), flush=True)
for rep in range(4):
    d0 = lib.MPIR_Hip_direct_dispatches()
    w = []
    for i in range(100):
        c0 = time.perf_counter(); fast(*args[i % 4]); w.append((time.perf_counter() - c0) * 1e6)
    w.sort()
    print(f"rep {rep}: median {w[50]:.2f} us p10 {w[10]:.2f} p90 {w[90]:.2f}  direct {lib.MPIR_Hip_direct_dispatches() - d0}  threads {ntasks()}", flush=True)
    time.sleep(0.001)

"""On a GPU box, host-buffer MPI_Reduce_local does not start the GPU runtime
(VERDICT r3 item 1a).  A CPU-only MPI program linked against a libmpi that
carries the drop-in must behave like MPICH's loop (opsum.c:21-76): no
/dev/kfd opened, no HSA runtime, no HIP query, however many host reductions
it makes.  A fresh child process (no torch) loads the library, reduces numpy
buffers of 1 element and of 4 MiB (bit-exact against the oracle), and
checks that /dev/kfd is neither open nor mapped and that the HSA runtime
still answers "not initialised".  It then starts HIP itself, and a device
reduction in the same process still takes the gfx950 kernel (the library
notices the runtime once it is up).
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import ctypes, os, sys
sys.path[:0] = [{root!r}, os.path.join({root!r}, "mpich-pip_amd")]
import numpy as np
import mpich_pip_amd as m
import oracle
lib = m.load()
oracle.load()

def kfd():
    maps = open("/proc/self/maps").read().count("/dev/kfd")
    fds = 0
    for fd in os.listdir("/proc/self/fd"):
        try:
            fds += os.readlink("/proc/self/fd/" + fd) == "/dev/kfd"
        except OSError:
            pass
    return maps + fds

hsa = ctypes.CDLL("libhsa-runtime64.so.1")
def hsa_status():
    v = ctypes.c_uint16(0)
    return hsa.hsa_system_get_info(0, ctypes.byref(v))

rng = np.random.default_rng(3)
for n in (1, (4 << 20) // 8 + 1):
    a = rng.uniform(-1, 1, n)
    b = rng.uniform(-1, 1, n)
    want = a.copy()
    assert oracle.reduce_local(b.copy(), want, n, m.MPI_DOUBLE, m.MPI_SUM) == 0
    assert lib.MPI_Reduce_local(b.ctypes.data, a.ctypes.data, n, m.MPI_DOUBLE, m.MPI_SUM) == 0
    assert np.array_equal(a.view(np.uint64), want.view(np.uint64))
print("host-only kfd", kfd(), "hsa", hex(hsa_status()))

# now the program starts HIP itself: device buffers take the kernel
hip = ctypes.CDLL("libamdhip64.so")
cnt = ctypes.c_int(0)
assert hip.hipGetDeviceCount(ctypes.byref(cnt)) == 0 and cnt.value > 0
n = 1 << 20
a = rng.uniform(-1, 1, n).astype(np.float32)
b = rng.uniform(-1, 1, n).astype(np.float32)
want = a.copy()
assert oracle.reduce_local(b.copy(), want, n, m.MPI_FLOAT, m.MPI_SUM) == 0
da, db = ctypes.c_void_p(), ctypes.c_void_p()
assert hip.hipMalloc(ctypes.byref(da), ctypes.c_size_t(4 * n)) == 0
assert hip.hipMalloc(ctypes.byref(db), ctypes.c_size_t(4 * n)) == 0
assert hip.hipMemcpy(da, a.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(4 * n), 1) == 0
assert hip.hipMemcpy(db, b.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(4 * n), 1) == 0
lib.MPIR_Hip_direct_dispatches.restype = ctypes.c_uint64
d0 = lib.MPIR_Hip_direct_dispatches()
assert lib.MPI_Reduce_local(db, da, n, m.MPI_FLOAT, m.MPI_SUM) == 0
got = np.empty_like(a)
assert hip.hipMemcpy(got.ctypes.data_as(ctypes.c_void_p), da, ctypes.c_size_t(4 * n), 2) == 0
assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
print("device kernel", lib.MPIR_Hip_direct_dispatches() - d0, "kfd", kfd() > 0)
"""


@pytest.mark.gpu
def test_host_only_calls_leave_gpu_runtime_closed():
    env = dict(os.environ, OMP_NUM_THREADS="1")
    p = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT)], capture_output=True, text=True,
                       timeout=110, env=env)
    assert p.returncode == 0, p.stdout[-1000:] + p.stderr[-2000:]
    lines = p.stdout.splitlines()
    host = next(ln for ln in lines if ln.startswith("host-only"))
    assert host == "host-only kfd 0 hsa 0x100b", host      # HSA_STATUS_ERROR_NOT_INITIALIZED
    dev = next(ln for ln in lines if ln.startswith("device kernel"))
    assert dev == "device kernel 1 kfd True", dev

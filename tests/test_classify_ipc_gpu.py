"""A device buffer imported from another process (hipIpcOpenMemHandle) as an
MPI_Reduce_local operand: MPICH's intra-node GPU path hands such IPC mappings
to the reduction.  HSA reports them as IPC memory (hsa_ext_amd.h:2364); the
library's classify() (hip_reduce.hip) must see a device buffer on the right
device and combine in place.  The parent allocates and fills the buffer and
exports its handle; a child process opens it, reduces into it (and from it),
and the parent checks the bytes against the oracle.  Both sides allocate through
the HIP runtime the library links (libamdhip64.so.7), not torch's bundled copy
(tests/test_classify_kinds_gpu.py explains why).
"""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = (1 << 20) + 5

CHILD = r"""
import ctypes, json, os, sys
import numpy as np
sys.path[:0] = [{root!r}, os.path.join({root!r}, "mpich-pip_amd")]
import mpich_pip_amd as m
lib = m.load()
lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN)
hip = ctypes.CDLL("libamdhip64.so.7")
class H(ctypes.Structure):
    _fields_ = [("reserved", ctypes.c_char * 64)]
n = {n}
assert hip.hipSetDevice(0) == 0
h = H()
ctypes.memmove(ctypes.byref(h), bytes.fromhex(sys.argv[1]), 64)
ipc = ctypes.c_void_p()
rc = hip.hipIpcOpenMemHandle(ctypes.byref(ipc), h, ctypes.c_uint(1))
assert rc == 0, "hipIpcOpenMemHandle: %d" % rc
out = {{"is_device": lib.MPIR_Hip_is_device_ptr(ipc)}}
b = np.random.default_rng(5).uniform(-1, 1, n).astype(np.float32)
d = ctypes.c_void_p()
assert hip.hipMalloc(ctypes.byref(d), ctypes.c_size_t(4 * n)) == 0
assert hip.hipMemcpy(d, ctypes.c_void_p(b.ctypes.data), ctypes.c_size_t(4 * n), 4) == 0
# inout = the imported buffer
out["rc_into_ipc"] = lib.MPI_Reduce_local(d, ipc, n, m.MPI_FLOAT, m.MPI_SUM)
# inbuf = the imported buffer, inout = a local device buffer holding b
out["rc_from_ipc"] = lib.MPI_Reduce_local(ipc, d, n, m.MPI_FLOAT, m.MPI_SUM)
got = np.empty(n, np.float32)
assert hip.hipMemcpy(ctypes.c_void_p(got.ctypes.data), d, ctypes.c_size_t(4 * n), 4) == 0
np.save(sys.argv[2], got)
assert hip.hipIpcCloseMemHandle(ipc) == 0
print(json.dumps(out), flush=True)
"""


def test_ipc_imported_buffer(mpi, orc, tmp_path):
    lib = mpi.load()
    if lib.MPIR_Hip_device_count() <= 0:
        pytest.fail("gpu test requires a HIP device")
    hip = ctypes.CDLL("libamdhip64.so.7")
    assert hip.hipSetDevice(0) == 0
    rng = np.random.default_rng(4)
    a = rng.uniform(-1, 1, N).astype(np.float32)
    b = np.random.default_rng(5).uniform(-1, 1, N).astype(np.float32)
    p = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(4 * N)) == 0
    try:
        assert hip.hipMemcpy(p, ctypes.c_void_p(a.ctypes.data), ctypes.c_size_t(4 * N), 4) == 0
        handle = ctypes.create_string_buffer(64)
        rc = hip.hipIpcGetMemHandle(handle, p)
        if rc != 0:
            pytest.skip(f"hipIpcGetMemHandle unavailable on this box ({rc})")
        got_path = str(tmp_path / "got.npy")
        r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, n=N), handle.raw.hex(), got_path],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-3000:]
        res = json.loads(r.stdout.strip().splitlines()[-1])
        assert res == {"is_device": 1, "rc_into_ipc": 0, "rc_from_ipc": 0}, res
        # the imported buffer now holds a + b; the child's local buffer (a + b) + b
        want1 = a.copy()
        assert orc.reduce_local(b.copy(), want1, N, mpi.MPI_FLOAT, mpi.MPI_SUM) == 0
        got1 = np.empty(N, np.float32)
        assert hip.hipMemcpy(ctypes.c_void_p(got1.ctypes.data), p, ctypes.c_size_t(4 * N), 4) == 0
        assert np.array_equal(got1.view(np.uint32), want1.view(np.uint32))
        want2 = b.copy()
        assert orc.reduce_local(want1.copy(), want2, N, mpi.MPI_FLOAT, mpi.MPI_SUM) == 0
        got2 = np.load(got_path)
        assert np.array_equal(got2.view(np.uint32), want2.view(np.uint32))
    finally:
        hip.hipFree(p)

#!/usr/bin/env python3
"""Does a host-only MPI_Reduce_local start the GPU runtime?  

Run in a fresh process (no torch): loads the library, reports whether /dev/kfd
is open or mapped and what hsa_system_get_info answers (0x100b =
HSA_STATUS_ERROR_NOT_INITIALIZED), after each of: library load, a host-buffer
MPI_Reduce_local of 1 and of 4 Mi doubles, and finally hipGetDeviceCount.

    python3 tools/kfd_probe.py
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))


def kfd_state():
    maps = open("/proc/self/maps").read().count("/dev/kfd")
    fds = 0
    for fd in os.listdir("/proc/self/fd"):
        try:
            fds += os.readlink(f"/proc/self/fd/{fd}") == "/dev/kfd"
        except OSError:
            pass
    return maps, fds


def hsa_state():
    hsa = ctypes.CDLL("libhsa-runtime64.so.1")
    v = ctypes.c_uint16(0)
    return hex(hsa.hsa_system_get_info(0, ctypes.byref(v)))     # HSA_SYSTEM_INFO_VERSION_MAJOR


def report(tag):
    m, f = kfd_state()
    print(f"{tag:34s} kfd mappings {m:3d}  kfd fds {f}  hsa_system_get_info {hsa_state()}  "
          f"threads {len(os.listdir('/proc/self/task'))}", flush=True)


def main():
    import numpy as np
    report("start")
    import mpich_pip_amd as m
    lib = m.load()
    report("after library load")
    for n in (1, 4 << 20):
        a = np.ones(n)
        b = np.ones(n)
        rc = lib.MPI_Reduce_local(a.ctypes.data, b.ctypes.data, n, m.MPI_DOUBLE, m.MPI_SUM)
        assert rc == 0 and b[0] == 2.0 and b[-1] == 2.0
        report(f"after host-host reduce n={n}")
    print("MPIR_Hip_device_count", lib.MPIR_Hip_device_count())
    report("after hipGetDeviceCount")


if __name__ == "__main__":
    main()

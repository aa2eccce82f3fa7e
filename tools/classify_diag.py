"""Diagnostic: each buffer kind's HSA / HIP answers next to the library's
MPIR_Hip_is_device_ptr, in a process that has started HIP through torch, each
kind on a fresh thread (as tests/test_classify_kinds_gpu.py runs them).

    python tools/classify_diag.py
"""
import ctypes
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "mpich-pip_amd")]

import torch  # noqa: E402
import mpich_pip_amd as m  # noqa: E402
import test_classify_kinds_gpu as K  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so.7")     # the library's runtime (torch bundles another)
hsa = ctypes.CDLL("libhsa-runtime64.so.1")
lib = m.load()
torch.cuda.set_device(0)
torch.zeros(1, device="cuda")


def agent_kind(h):
    class Agent(ctypes.Structure):
        _fields_ = [("handle", ctypes.c_uint64)]
    t = ctypes.c_int(-1)
    rc = hsa.hsa_agent_get_info(Agent(h), 17, ctypes.byref(t))      # HSA_AGENT_INFO_DEVICE
    return {0: "cpu", 1: "gpu"}.get(t.value, f"?{rc}/{t.value}") if h else "none"


def row(name, p):
    info = K.HsaInfo()
    info.size = ctypes.sizeof(info)
    hrc = hsa.hsa_amd_pointer_info(ctypes.c_void_p(p), ctypes.byref(info), None, None, None)
    at = K.PtrAttr()
    rc = hip.hipPointerGetAttributes(ctypes.byref(at), ctypes.c_void_p(p))
    d1 = lib.MPIR_Hip_is_device_ptr(ctypes.c_void_p(p))
    d2 = lib.MPIR_Hip_is_device_ptr(ctypes.c_void_p(p))
    print(f"{name:18s} {p:#x} hsa rc {hrc} type {info.type} owner {agent_kind(info.agentOwner)} "
          f"flags {info.global_flags:#x} host_base {info.hostBaseAddress or 0:#x} | hip rc {rc} type {at.type} "
          f"dev {at.device} | is_device {d1} {d2} [{threading.current_thread().name}]", flush=True)


def run(maker, name):
    ks = K.Kinds(hip)
    try:
        x = getattr(ks, maker)()
        row(name, x)
    finally:
        ks.close()


# torch's own allocations (its bundled HIP runtime): a pinned tensor and a device tensor
pt = torch.ones(1 << 20).pin_memory()
dt_ = torch.ones(1 << 20, device="cuda")
row("torch pin_memory", pt.data_ptr())
row("torch cuda tensor", dt_.data_ptr())

for rnd in range(2):
    # an IPC export first, as tests/test_classify_ipc_gpu.py's parent does
    p = ctypes.c_void_p()
    hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 22))
    h = ctypes.create_string_buffer(64)
    print("ipc export rc", hip.hipIpcGetMemHandle(h, p))
    for label, maker, _ in K.KINDS:
        t = threading.Thread(target=run, args=(maker, label))
        t.start()
        t.join()
    for label, maker, _ in K.KINDS:
        run(maker, label + " (main)")
    hip.hipFree(p)

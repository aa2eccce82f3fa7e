"""Every kind of buffer a caller can hand MPI_Reduce_local, classified by the
HSA pointer query (hip_reduce.hip classify) and reduced
bit-exact against the oracle.  The reference runs no query at all: its loop
reads host memory (reduce_local.c:35-122, opsum.c:21-76).

Kinds: hipMalloc, hipMallocAsync (stream-ordered pool: HSA_VMEM), VMM
(hipMemCreate + hipMemAddressReserve + hipMemMap: HSA_VMEM), hipMallocManaged
(RESERVED_ADDR: asks HIP), hipHostMalloc (HSA, CPU-owned: pinned),
hipHostRegister'ed malloc memory (UNKNOWN to HSA: pageable path) and plain
pageable memory.  Each kind is paired with a hipMalloc buffer in both roles
(inbuf and inoutbuf) and with a buffer of its own kind; MPIR_Hip_is_device_ptr
reports the class.  Each case runs on a thread of its own: the library keeps
HIP's host verdicts per thread by page, and a fresh thread starts with none.

The buffers come from the HIP runtime the library itself links
(libamdhip64.so.7 from /opt/rocm), not from the copy torch bundles: a process
that imports torch holds two HIP runtimes (and two HSA runtimes), and one does
not know the other's managed or pinned allocations (it sees them through the
kernel driver only: another runtime's hipHostMalloc memory reads as device
memory, its managed memory as unregistered host memory -- both still combined
correctly, on the GPU or the host).  An MPI program has one runtime.
"""
import ctypes
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = (1 << 18) + 3                 # fp32 elements: ragged, ~1 MiB
NB = N * 4


class Loc(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("id", ctypes.c_int)]


class AllocFlags(ctypes.Structure):
    _fields_ = [("compressionType", ctypes.c_ubyte), ("gpuDirectRDMACapable", ctypes.c_ubyte),
                ("usage", ctypes.c_ushort)]


class Prop(ctypes.Structure):       # hipMemAllocationProp (hip_runtime_api.h:1748)
    _fields_ = [("type", ctypes.c_int), ("requestedHandleType", ctypes.c_int), ("location", Loc),
                ("win32HandleMetaData", ctypes.c_void_p), ("allocFlags", AllocFlags)]


class AccessDesc(ctypes.Structure):  # hipMemAccessDesc (hip_runtime_api.h:1201)
    _fields_ = [("location", Loc), ("flags", ctypes.c_int)]


def library_hip(mpi):
    """The HIP runtime the product library links (already loaded by it)."""
    mpi.load()
    return ctypes.CDLL("libamdhip64.so.7")


@pytest.fixture(scope="module")
def hip(mpi):
    if mpi.load().MPIR_Hip_device_count() <= 0:
        pytest.fail("gpu test requires a HIP device")
    h = library_hip(mpi)
    _ok(h.hipSetDevice(0), "hipSetDevice")
    return h


class PtrAttr(ctypes.Structure):     # hipPointerAttribute_t (hip_runtime_api.h:280)
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


class HsaInfo(ctypes.Structure):     # hsa_amd_pointer_info_t (hsa_ext_amd.h:2379)
    _fields_ = [("size", ctypes.c_uint32), ("type", ctypes.c_int), ("agentBaseAddress", ctypes.c_void_p),
                ("hostBaseAddress", ctypes.c_void_p), ("sizeInBytes", ctypes.c_size_t), ("userData", ctypes.c_void_p),
                ("agentOwner", ctypes.c_uint64), ("global_flags", ctypes.c_uint32), ("registered", ctypes.c_bool)]


def _diag(hip, p):
    """HIP's and HSA's own answers for p (for the failure message)."""
    at = PtrAttr()
    rc = hip.hipPointerGetAttributes(ctypes.byref(at), ctypes.c_void_p(p))
    hsa = ctypes.CDLL("libhsa-runtime64.so.1")     # the library's HSA runtime
    info = HsaInfo()
    info.size = ctypes.sizeof(info)
    hrc = hsa.hsa_amd_pointer_info(ctypes.c_void_p(p), ctypes.byref(info), None, None, None)
    class Agent(ctypes.Structure):
        _fields_ = [("handle", ctypes.c_uint64)]
    kind = ctypes.c_int(-1)
    if info.agentOwner:
        hsa.hsa_agent_get_info(Agent(info.agentOwner), 17, ctypes.byref(kind))     # HSA_AGENT_INFO_DEVICE
    return (f"ptr {p:#x}: hip rc {rc} type {at.type} device {at.device} managed {at.isManaged}; "
            f"hsa rc {hrc} type {info.type} owner {info.agentOwner:#x} ({ {0: 'cpu', 1: 'gpu'}.get(kind.value, '-') }) "
            f"flags {info.global_flags:#x}")


def _ok(rc, what):
    assert rc == 0, f"{what}: hip error {rc}"


class Kinds:
    """Allocations of each kind, freed at the end."""

    def __init__(self, hip):
        self.hip = hip
        self.frees = []
        self.keep = []

    def device(self):
        p = ctypes.c_void_p()
        _ok(self.hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(NB)), "hipMalloc")
        self.frees.append(("hipFree", p.value))
        return p.value

    def pool(self):
        p = ctypes.c_void_p()
        _ok(self.hip.hipMallocAsync(ctypes.byref(p), ctypes.c_size_t(NB), None), "hipMallocAsync")
        _ok(self.hip.hipStreamSynchronize(None), "sync")
        self.frees.append(("pool", p.value))
        return p.value

    def vmm(self):
        prop = Prop()
        prop.type = 1                   # hipMemAllocationTypePinned
        prop.location = Loc(1, 0)       # hipMemLocationTypeDevice, device 0
        gran = ctypes.c_size_t()
        _ok(self.hip.hipMemGetAllocationGranularity(ctypes.byref(gran), ctypes.byref(prop), 0), "granularity")
        size = (NB + gran.value - 1) // gran.value * gran.value
        h = ctypes.c_void_p()
        _ok(self.hip.hipMemCreate(ctypes.byref(h), ctypes.c_size_t(size), ctypes.byref(prop), ctypes.c_ulonglong(0)),
            "hipMemCreate")
        p = ctypes.c_void_p()
        _ok(self.hip.hipMemAddressReserve(ctypes.byref(p), ctypes.c_size_t(size), ctypes.c_size_t(0), None,
                                          ctypes.c_ulonglong(0)), "hipMemAddressReserve")
        _ok(self.hip.hipMemMap(p, ctypes.c_size_t(size), ctypes.c_size_t(0), h, ctypes.c_ulonglong(0)), "hipMemMap")
        acc = AccessDesc(Loc(1, 0), 3)  # hipMemAccessFlagsProtReadWrite
        _ok(self.hip.hipMemSetAccess(p, ctypes.c_size_t(size), ctypes.byref(acc), ctypes.c_size_t(1)),
            "hipMemSetAccess")
        self.frees.append(("vmm", (p.value, size, h.value)))
        return p.value

    def managed(self):
        p = ctypes.c_void_p()
        _ok(self.hip.hipMallocManaged(ctypes.byref(p), ctypes.c_size_t(NB), 1), "hipMallocManaged")
        self.frees.append(("hipFree", p.value))
        return p.value

    def pinned(self):
        p = ctypes.c_void_p()
        _ok(self.hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(NB), 0), "hipHostMalloc")
        self.frees.append(("hipHostFree", p.value))
        return p.value

    def registered(self):
        buf = np.zeros(NB + 8192, np.uint8)
        addr = (buf.ctypes.data + 4095) & ~4095
        _ok(self.hip.hipHostRegister(ctypes.c_void_p(addr), ctypes.c_size_t(NB), 0), "hipHostRegister")
        self.keep.append(buf)
        self.frees.append(("hipHostUnregister", addr))
        return addr

    def pageable(self):
        buf = np.zeros(NB + 64, np.uint8)
        self.keep.append(buf)
        return buf.ctypes.data

    def close(self):
        self.hip.hipDeviceSynchronize()
        for kind, v in reversed(self.frees):
            if kind == "pool":
                self.hip.hipFreeAsync(ctypes.c_void_p(v), None)
                self.hip.hipStreamSynchronize(None)
            elif kind == "vmm":
                p, size, h = v
                self.hip.hipMemUnmap(ctypes.c_void_p(p), ctypes.c_size_t(size))
                self.hip.hipMemRelease(ctypes.c_void_p(h))
                self.hip.hipMemAddressFree(ctypes.c_void_p(p), ctypes.c_size_t(size))
            else:
                getattr(self.hip, kind)(ctypes.c_void_p(v))


KINDS = [("hipMalloc", "device", 1), ("hipMallocAsync", "pool", 1), ("VMM", "vmm", 1),
         ("hipMallocManaged", "managed", 1), ("hipHostMalloc", "pinned", 0),
         ("hipHostRegister", "registered", 0), ("pageable", "pageable", 0)]
KIND_CLASS = {"device": 1, "pool": 1, "vmm": 1, "managed": 1, "pinned": 2, "registered": 2, "pageable": 0}


def _put(hip, dst, arr):
    _ok(hip.hipMemcpy(ctypes.c_void_p(dst), ctypes.c_void_p(arr.ctypes.data), ctypes.c_size_t(NB), 4), "H2X")


def _get(hip, src):
    out = np.empty(N, np.float32)
    _ok(hip.hipMemcpy(ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(src), ctypes.c_size_t(NB), 4), "X2H")
    return out


@pytest.mark.parametrize("name,maker,is_dev", KINDS, ids=[k[0] for k in KINDS])
def test_kind_classified_and_reduced(mpi, orc, hip, name, maker, is_dev):
    err = []

    def body():
        try:
            _case(mpi, orc, hip, name, maker, is_dev)
        except BaseException as e:      # noqa: BLE001
            err.append(e)
    t = threading.Thread(target=body)
    t.start()
    t.join(120)
    assert not t.is_alive(), "case hung"
    if err:
        raise err[0]


def _case(mpi, orc, hip, name, maker, is_dev):
    lib = mpi.load()
    ks = Kinds(hip)
    try:
        x = getattr(ks, maker)()
        y = getattr(ks, maker)()
        d = ks.device()
        pre = _diag(hip, x)
        got = lib.MPIR_Hip_is_device_ptr(ctypes.c_void_p(x))
        assert got == is_dev, (name, pre, _diag(hip, x), lib.MPIR_Hip_is_device_ptr(ctypes.c_void_p(x)))
        # the class a 1 MiB call sees: 0 pageable, 1 device, 2 pinned
        assert lib.MPIR_Hip_pointer_kind(ctypes.c_void_p(x), NB) == KIND_CLASS[maker], (name, pre)
        rng = np.random.default_rng(sum(map(ord, name)))
        a = rng.uniform(-1, 1, N).astype(np.float32)
        b = rng.uniform(-1, 1, N).astype(np.float32)
        want = a.copy()
        assert orc.reduce_local(b.copy(), want, N, mpi.MPI_FLOAT, mpi.MPI_SUM) == 0
        # (inbuf, inoutbuf): kind into device, device into kind, kind into kind
        for pin, pio in ((x, d), (d, x), (y, x)):
            _put(hip, pin, b)
            _put(hip, pio, a)
            rc = lib.MPI_Reduce_local(ctypes.c_void_p(pin), ctypes.c_void_p(pio), N, mpi.MPI_FLOAT, mpi.MPI_SUM)
            assert rc == 0, mpi.error_string(rc)
            got = _get(hip, pio)
            assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), (name, pin == x, pio == x)
    finally:
        ks.close()


def test_registration_after_kept_verdict(mpi, orc, hip):
    """One thread, one page: a pageable buffer reduced small (its verdict kept),
    then registered with hipHostRegister -- which HSA still reports as UNKNOWN --
    and reduced large: the large call asks HIP again and sees it pinned; after
    hipHostUnregister a large call sees it pageable again.  Every reduction
    bit-exact (hip_reduce.hip classify, `reuse`)."""
    lib = mpi.load()
    err = []

    def body():
        try:
            buf = np.zeros(NB + 8192, np.uint8)
            addr = (buf.ctypes.data + 4095) & ~4095
            x = np.frombuffer((ctypes.c_char * NB).from_address(addr), np.float32)
            d = Kinds(hip)
            dv = d.device()
            rng = np.random.default_rng(11)
            a = rng.uniform(-1, 1, N).astype(np.float32)
            b = rng.uniform(-1, 1, N).astype(np.float32)

            def check(n):
                # inbuf = the host page, inoutbuf = a device buffer
                x[:n] = b[:n]
                _put(hip, dv, a)
                rc = lib.MPI_Reduce_local(ctypes.c_void_p(addr), ctypes.c_void_p(dv), n, mpi.MPI_FLOAT, mpi.MPI_SUM)
                assert rc == 0, mpi.error_string(rc)
                want = a[:n].copy()
                assert orc.reduce_local(b[:n].copy(), want, n, mpi.MPI_FLOAT, mpi.MPI_SUM) == 0
                got = _get(hip, dv)[:n]
                assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), n

            try:
                check(16)
                assert lib.MPIR_Hip_pointer_kind(ctypes.c_void_p(addr), 64) == 0
                _ok(hip.hipHostRegister(ctypes.c_void_p(addr), ctypes.c_size_t(NB), 0), "hipHostRegister")
                try:
                    # a small call may keep the pageable verdict (only the null-stream ordering differs)
                    assert lib.MPIR_Hip_pointer_kind(ctypes.c_void_p(addr), 64) in (0, 2)
                    assert lib.MPIR_Hip_pointer_kind(ctypes.c_void_p(addr), NB) == 2, _diag(hip, addr)
                    assert lib.MPIR_Hip_pointer_kind(ctypes.c_void_p(addr), 64) == 2      # refreshed
                    check(N)
                    check(16)
                finally:
                    _ok(hip.hipHostUnregister(ctypes.c_void_p(addr)), "hipHostUnregister")
                assert lib.MPIR_Hip_pointer_kind(ctypes.c_void_p(addr), NB) == 0, _diag(hip, addr)
                check(N)
            finally:
                d.close()
        except BaseException as e:      # noqa: BLE001
            err.append(e)
    t = threading.Thread(target=body)
    t.start()
    t.join(120)
    assert not t.is_alive(), "case hung"
    if err:
        raise err[0]


def test_kept_pageable_verdict_orders_after_null_stream(mpi, orc, hip):
    """kept host verdicts are keyed by the 4 KiB page, and
    a registered buffer may start in the page of a pageable buffer classified
    earlier.  Here the thread first reduces a pageable buffer A (its verdict
    kept), then B = A + 2048 B is registered with hipHostRegister and filled
    by a null-stream hipMemcpyAsync queued behind a 512 MiB device copy, and a
    small host-host MPI_Reduce_local(C, B) follows at once.  B's page answers
    with A's kept pageable verdict; the call must still wait for the null
    stream before reading B (hip_reduce.hip classify `kept`), so B ends as
    copied + C, bit-exact against the oracle."""
    lib = mpi.load()
    err = []
    n = 16

    def body():
        ks = Kinds(hip)
        try:
            region = np.zeros(NB + 3 * 4096, np.uint8)
            base = (region.ctypes.data + 4095) & ~4095
            a_addr, b_addr = base, base + 2048
            va = np.frombuffer((ctypes.c_char * 64).from_address(a_addr), np.float32)
            vb = np.frombuffer((ctypes.c_char * 64).from_address(b_addr), np.float32)
            c = np.linspace(-1, 1, n).astype(np.float32)
            # A (pageable) reduced small: this page's pageable verdict is kept
            va[:] = 1.0
            rc = lib.MPI_Reduce_local(ctypes.c_void_p(c.ctypes.data), ctypes.c_void_p(a_addr), n,
                                      mpi.MPI_FLOAT, mpi.MPI_SUM)
            assert rc == 0, mpi.error_string(rc)
            assert lib.MPIR_Hip_pointer_kind(ctypes.c_void_p(b_addr), 64) == 0      # the kept verdict answers
            _ok(hip.hipHostRegister(ctypes.c_void_p(b_addr), ctypes.c_size_t(NB), 0), "hipHostRegister")
            try:
                big = 512 << 20
                s0, s1 = ctypes.c_void_p(), ctypes.c_void_p()
                _ok(hip.hipMalloc(ctypes.byref(s0), ctypes.c_size_t(big)), "hipMalloc")
                _ok(hip.hipMalloc(ctypes.byref(s1), ctypes.c_size_t(big)), "hipMalloc")
                ks.frees += [("hipFree", s0.value), ("hipFree", s1.value)]
                src = np.arange(n, dtype=np.float32) + 100.0
                dsrc = ks.device()
                _ok(hip.hipMemcpy(ctypes.c_void_p(dsrc), ctypes.c_void_p(src.ctypes.data), ctypes.c_size_t(64), 1),
                    "H2D")
                vb[:] = -7.0
                # null stream: a long device copy, then the D2H fill of B (registered: DMA, asynchronous)
                _ok(hip.hipMemcpyAsync(s1, s0, ctypes.c_size_t(big), 3, None), "D2D")
                _ok(hip.hipMemcpyAsync(ctypes.c_void_p(b_addr), ctypes.c_void_p(dsrc), ctypes.c_size_t(64), 2, None),
                    "D2H")
                rc = lib.MPI_Reduce_local(ctypes.c_void_p(c.ctypes.data), ctypes.c_void_p(b_addr), n,
                                          mpi.MPI_FLOAT, mpi.MPI_SUM)
                assert rc == 0, mpi.error_string(rc)
                _ok(hip.hipDeviceSynchronize(), "sync")
                want = src.copy()
                assert orc.reduce_local(c.copy(), want, n, mpi.MPI_FLOAT, mpi.MPI_SUM) == 0
                assert np.array_equal(vb.view(np.uint32), want.view(np.uint32)), (vb, want)
            finally:
                _ok(hip.hipHostUnregister(ctypes.c_void_p(b_addr)), "hipHostUnregister")
        except BaseException as e:      # noqa: BLE001
            err.append(e)
        finally:
            ks.close()
    t = threading.Thread(target=body)
    t.start()
    t.join(120)
    assert not t.is_alive(), "case hung"
    if err:
        raise err[0]

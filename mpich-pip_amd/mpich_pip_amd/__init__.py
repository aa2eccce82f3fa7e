"""ctypes binding of libmpich_reduce_local.so -- the MI355X MPI_Reduce_local.

This is host plumbing for tests, the benchmark and the smoke check; the
product is the C ABI declared in include/mpi_reduce_local.h (see
INTEGRATION.md for how MPICH links it).  Constants mirror that header, which
mirrors the reference's mpi.h.in / configure.ac values.

The library is loaded from mpich-pip_amd/lib/ (built by `make -C
mpich-pip_amd` or __graft_entry__.build()).  A missing library raises
immediately: there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib", "libmpich_reduce_local.so")

# ---- error classes (mpi.h.in:784-811)
MPI_SUCCESS = 0
MPI_ERR_BUFFER = 1
MPI_ERR_COUNT = 2
MPI_ERR_TYPE = 3
MPI_ERR_OP = 9
MPI_ERR_ARG = 12
MPI_ERR_OTHER = 15

MPI_ERRORS_ARE_FATAL = 0x54000000
MPI_ERRORS_RETURN = 0x54000001

# ---- ops (mpi.h.in:310-325)
MPI_OP_NULL = 0x18000000
MPI_MAX = 0x58000001
MPI_MIN = 0x58000002
MPI_SUM = 0x58000003
MPI_PROD = 0x58000004
MPI_LAND = 0x58000005
MPI_BAND = 0x58000006
MPI_LOR = 0x58000007
MPI_BOR = 0x58000008
MPI_LXOR = 0x58000009
MPI_BXOR = 0x5800000A
MPI_MINLOC = 0x5800000B
MPI_MAXLOC = 0x5800000C
MPI_REPLACE = 0x5800000D
MPI_NO_OP = 0x5800000E

OPS = {
    "MPI_MAX": MPI_MAX, "MPI_MIN": MPI_MIN, "MPI_SUM": MPI_SUM, "MPI_PROD": MPI_PROD,
    "MPI_LAND": MPI_LAND, "MPI_BAND": MPI_BAND, "MPI_LOR": MPI_LOR, "MPI_BOR": MPI_BOR,
    "MPI_LXOR": MPI_LXOR, "MPI_BXOR": MPI_BXOR, "MPI_MINLOC": MPI_MINLOC, "MPI_MAXLOC": MPI_MAXLOC,
}

# ---- datatypes, x86-64 values (configure.ac:3442-3705)
MPI_DATATYPE_NULL = 0x0C000000
DATATYPES = {
    "MPI_CHAR": 0x4C000101,
    "MPI_UNSIGNED_CHAR": 0x4C000102,
    "MPI_SHORT": 0x4C000203,
    "MPI_UNSIGNED_SHORT": 0x4C000204,
    "MPI_INT": 0x4C000405,
    "MPI_UNSIGNED": 0x4C000406,
    "MPI_LONG": 0x4C000807,
    "MPI_UNSIGNED_LONG": 0x4C000808,
    "MPI_LONG_LONG": 0x4C000809,
    "MPI_FLOAT": 0x4C00040A,
    "MPI_DOUBLE": 0x4C00080B,
    "MPI_LONG_DOUBLE": 0x4C00100C,
    "MPI_BYTE": 0x4C00010D,
    "MPI_WCHAR": 0x4C00040E,
    "MPI_2INT": 0x4C000816,
    "MPI_SIGNED_CHAR": 0x4C000118,
    "MPI_UNSIGNED_LONG_LONG": 0x4C000819,
    "MPI_FLOAT_INT": 0x8C000000,
    "MPI_DOUBLE_INT": 0x8C000001,
    "MPI_LONG_DOUBLE_INT": 0x8C000004,
    "MPI_LONG_INT": 0x8C000002,
    "MPI_SHORT_INT": 0x8C000003,
    "MPI_INT8_T": 0x4C000137,
    "MPI_INT16_T": 0x4C000238,
    "MPI_INT32_T": 0x4C000439,
    "MPI_INT64_T": 0x4C00083A,
    "MPI_UINT8_T": 0x4C00013B,
    "MPI_UINT16_T": 0x4C00023C,
    "MPI_UINT32_T": 0x4C00043D,
    "MPI_UINT64_T": 0x4C00083E,
    "MPI_C_BOOL": 0x4C00013F,
    "MPI_C_FLOAT_COMPLEX": 0x4C000840,
    "MPI_C_DOUBLE_COMPLEX": 0x4C001041,
    "MPI_C_LONG_DOUBLE_COMPLEX": 0x4C002042,
    "MPIX_C_FLOAT16": 0x4C000246,
    "MPI_AINT": 0x4C000843,
    "MPI_OFFSET": 0x4C000844,
    "MPI_COUNT": 0x4C000845,
}
globals().update(DATATYPES)

# Every symbol include/mpi_reduce_local.h declares (checked by the CPU tests).
EXPORTED_SYMBOLS = [
    "MPI_Reduce_local", "PMPI_Reduce_local", "MPIR_Reduce_local",
    "MPIR_MAXF", "MPIR_MINF", "MPIR_SUM", "MPIR_PROD", "MPIR_LAND", "MPIR_BAND", "MPIR_LOR",
    "MPIR_BOR", "MPIR_LXOR", "MPIR_BXOR", "MPIR_MAXLOC", "MPIR_MINLOC", "MPIR_REPLACE", "MPIR_NO_OP",
    "MPIR_MAXF_check_dtype", "MPIR_MINF_check_dtype", "MPIR_SUM_check_dtype", "MPIR_PROD_check_dtype",
    "MPIR_LAND_check_dtype", "MPIR_BAND_check_dtype", "MPIR_LOR_check_dtype", "MPIR_BOR_check_dtype",
    "MPIR_LXOR_check_dtype", "MPIR_BXOR_check_dtype", "MPIR_MAXLOC_check_dtype",
    "MPIR_MINLOC_check_dtype", "MPIR_REPLACE_check_dtype", "MPIR_NO_OP_check_dtype",
    "MPIR_Op_table", "MPIR_Op_check_dtype_table",
    "MPI_Op_create", "PMPI_Op_create", "MPI_Op_free", "PMPI_Op_free",
    "MPI_Op_commutative", "PMPI_Op_commutative", "MPIR_Op_is_commutative",
    "MPI_Error_class", "MPI_Error_string",
    "MPIX_Reduce_local_stream", "MPIX_Reduce_local_set_errhandler", "MPIX_Reduce_local_get_errhandler",
    "MPIX_Reduce_local_multi", "MPIR_Hip_combine",
    # device collectives (include/mpix_hip_coll.h)
    "MPIX_Hip_comm_get_unique_id", "MPIX_Hip_comm_create", "MPIX_Hip_comm_create_loopback",
    "MPIX_Hip_comm_free", "MPIX_Hip_comm_rank", "MPIX_Hip_comm_size",
    "MPIX_Allreduce_hip", "MPIX_Reduce_scatter_block_hip", "MPIX_Reduce_hip", "MPIX_Reduce_scatter_hip",
    "MPIX_Scan_hip", "MPIX_Exscan_hip",
    # the HIP shim (include/mpir_hip_reduce.h)
    "MPIR_Hip_reduce", "MPIR_Hip_elem_size", "MPIR_Hip_has_kernel", "MPIR_Hip_is_device_ptr",
    "MPIR_Hip_pointer_kind", "MPIR_Hip_memcpy", "MPIR_Hip_error_string", "MPIR_Hip_device_count", "MPIR_Hip_thread_contexts",
    "MPIR_Hip_host_max_bytes", "MPIR_Hip_set_host_max_bytes", "MPIR_Hip_mixed_max_bytes", "MPIR_Hip_direct_dispatches", "MPIR_Hip_direct_profile",
    "MPIR_Hip_direct_last_kernel_ns", "MPIR_Hip_direct_state", "MPIR_Hip_direct_busy_skips",
    "MPIR_Hip_direct_last_split", "MPIR_Hip_direct_kernarg_writes", "MPIR_Hip_direct_placement", "MPIR_Hip_build_id", "MPIR_Hip_combine_set_flags",
    "MPIR_Hip_direct_prepare", "MPIR_Hip_set_local_ranks", "MPIR_Hip_host_threads",
    "MPIR_Hip_default_rings_in_vram", "MPIR_Hip_direct_ring_location", "MPIR_Hip_set_keep_bytes",
    "MPIR_Hip_set_keep_min_bytes",
    # runtime subset for config 1 (include/mpi_pip.h)
    "MPI_Init", "MPI_Initialized", "MPI_Finalize", "MPI_Finalized", "MPI_Abort", "MPI_Comm_size",
    "MPI_Comm_rank", "MPI_Get_processor_name", "MPI_Wtime", "MPI_Wtick", "MPI_Barrier", "MPI_Bcast",
    "MPI_Reduce",
]

MPI_User_function = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int))

_lib = None


# what load()'s MPIR_Hip_default_rings_in_vram(1) returned: 1 set then, 0 the
# environment held a value, -1 the HSA runtime had started (None: not loaded)
RINGS_DEFAULT = None


def load(path: str | None = None) -> ctypes.CDLL:
    """Load the C-ABI library (raises if it was not built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(f"{p} missing: build it with `make -C mpich-pip_amd` "
                           "(no CPU fallback exists for MPI_Reduce_local)")
    lib = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
    vp, i32 = ctypes.c_void_p, ctypes.c_int
    for name in ("MPI_Reduce_local", "PMPI_Reduce_local", "MPIR_Reduce_local"):
        f = getattr(lib, name)
        f.argtypes = [vp, vp, i32, i32, i32]
        f.restype = i32
    lib.MPIX_Reduce_local_stream.argtypes = [vp, vp, i32, i32, i32, vp]
    lib.MPIX_Reduce_local_stream.restype = i32
    lib.MPIX_Reduce_local_multi.argtypes = [ctypes.POINTER(vp), i32, vp, i32, i32, i32, i32, vp]
    lib.MPIX_Reduce_local_multi.restype = i32
    lib.MPIX_Hip_comm_get_unique_id.argtypes = [vp]
    lib.MPIX_Hip_comm_get_unique_id.restype = i32
    lib.MPIX_Hip_comm_create.argtypes = [vp, i32, i32, ctypes.POINTER(vp)]
    lib.MPIX_Hip_comm_create.restype = i32
    lib.MPIX_Hip_comm_create_loopback.argtypes = [i32, ctypes.POINTER(vp)]
    lib.MPIX_Hip_comm_create_loopback.restype = i32
    lib.MPIX_Hip_comm_free.argtypes = [ctypes.POINTER(vp)]
    lib.MPIX_Hip_comm_free.restype = i32
    for name in ("MPIX_Allreduce_hip", "MPIX_Reduce_scatter_block_hip", "MPIX_Scan_hip", "MPIX_Exscan_hip"):
        f = getattr(lib, name)
        f.argtypes = [vp, vp, i32, i32, i32, vp, i32, vp]
        f.restype = i32
    lib.MPIX_Reduce_hip.argtypes = [vp, vp, i32, i32, i32, i32, vp, i32, vp]
    lib.MPIX_Reduce_hip.restype = i32
    lib.MPIX_Reduce_scatter_hip.argtypes = [vp, vp, ctypes.POINTER(i32), i32, i32, vp, i32, vp]
    lib.MPIX_Reduce_scatter_hip.restype = i32
    lib.MPIX_Reduce_local_set_errhandler.argtypes = [i32]
    lib.MPIX_Reduce_local_set_errhandler.restype = i32
    lib.MPI_Op_create.argtypes = [MPI_User_function, i32, ctypes.POINTER(i32)]
    lib.MPI_Op_create.restype = i32
    lib.MPI_Op_free.argtypes = [ctypes.POINTER(i32)]
    lib.MPI_Op_free.restype = i32
    lib.MPI_Op_commutative.argtypes = [i32, ctypes.POINTER(i32)]
    lib.MPI_Op_commutative.restype = i32
    lib.MPIR_Op_is_commutative.argtypes = [i32]
    lib.MPIR_Op_is_commutative.restype = i32
    lib.MPI_Error_string.argtypes = [i32, ctypes.c_char_p, ctypes.POINTER(i32)]
    lib.MPI_Error_string.restype = i32
    lib.MPIR_Hip_reduce.argtypes = [vp, vp, ctypes.c_uint64, i32, i32, vp, i32]
    lib.MPIR_Hip_reduce.restype = i32
    lib.MPIR_Hip_has_kernel.argtypes = [i32, i32]
    lib.MPIR_Hip_has_kernel.restype = i32
    lib.MPIR_Hip_elem_size.argtypes = [i32]
    lib.MPIR_Hip_elem_size.restype = ctypes.c_size_t
    lib.MPIR_Hip_device_count.restype = i32
    lib.MPIR_Hip_thread_contexts.restype = i32
    lib.MPIR_Hip_host_max_bytes.restype = ctypes.c_uint64
    lib.MPIR_Hip_set_host_max_bytes.argtypes = [ctypes.c_uint64]
    lib.MPIR_Hip_set_host_max_bytes.restype = ctypes.c_uint64
    lib.MPIR_Hip_mixed_max_bytes.restype = ctypes.c_uint64
    lib.MPIR_Hip_direct_dispatches.restype = ctypes.c_uint64
    lib.MPIR_Hip_direct_profile.argtypes = [i32]
    lib.MPIR_Hip_direct_profile.restype = None
    lib.MPIR_Hip_direct_last_kernel_ns.restype = ctypes.c_uint64
    lib.MPIR_Hip_direct_state.argtypes = [i32]
    lib.MPIR_Hip_direct_state.restype = i32
    lib.MPIR_Hip_direct_busy_skips.restype = ctypes.c_uint64
    lib.MPIR_Hip_direct_kernarg_writes.restype = ctypes.c_uint64
    lib.MPIR_Hip_direct_last_split.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    lib.MPIR_Hip_direct_last_split.restype = None
    lib.MPIR_Hip_direct_placement.argtypes = [i32, ctypes.POINTER(i32)]
    lib.MPIR_Hip_direct_placement.restype = None
    lib.MPIR_Hip_direct_prepare.argtypes = [i32]
    lib.MPIR_Hip_direct_prepare.restype = i32
    lib.MPIR_Hip_default_rings_in_vram.argtypes = [i32]
    lib.MPIR_Hip_default_rings_in_vram.restype = i32
    lib.MPIR_Hip_direct_ring_location.argtypes = [i32]
    lib.MPIR_Hip_direct_ring_location.restype = i32
    for name in ("MPIR_Hip_set_keep_bytes", "MPIR_Hip_set_keep_min_bytes"):
        getattr(lib, name).argtypes = [ctypes.c_uint64]
        getattr(lib, name).restype = ctypes.c_uint64
    lib.MPIR_Hip_set_local_ranks.argtypes = [i32]
    lib.MPIR_Hip_set_local_ranks.restype = i32
    lib.MPIR_Hip_host_threads.argtypes = []
    lib.MPIR_Hip_host_threads.restype = i32
    lib.MPIR_Hip_build_id.restype = ctypes.c_char_p
    lib.MPIR_Hip_combine_set_flags.argtypes = [i32]
    lib.MPIR_Hip_combine_set_flags.restype = i32
    lib.MPIR_Hip_error_string.restype = ctypes.c_char_p
    lib.MPIR_Hip_pointer_kind.argtypes = [vp, ctypes.c_uint64]
    lib.MPIR_Hip_pointer_kind.restype = i32
    for name in [n for n in EXPORTED_SYMBOLS if n.endswith("_check_dtype")]:
        f = getattr(lib, name)
        f.argtypes = [i32]
        f.restype = i32
    # AQL rings in VRAM (direct_dispatch.hip default_rings_in_vram): the load-time
    # constructor stands aside in a process that already runs threads, which an
    # interpreter that imported numpy or torch first does (their pools are
    # parked and leave the environment alone); load() applies the default then,
    # while the HSA runtime has not started and the job set no value.
    global RINGS_DEFAULT
    RINGS_DEFAULT = lib.MPIR_Hip_default_rings_in_vram(1)
    if RINGS_DEFAULT == 1:
        os.environ["HSA_ALLOCATE_QUEUE_DEV_MEM"] = "1"      # Python's view of the variable the library set
    elif RINGS_DEFAULT == -1 and path is None:
        import warnings
        warnings.warn("mpich_pip_amd loaded after the GPU runtime started: its AQL rings stay in host memory "
                      "(~1.7 us per synchronous call); load it before the first GPU call, or export "
                      "HSA_ALLOCATE_QUEUE_DEV_MEM=1 (INTEGRATION.md, 'Keep the AQL rings in VRAM')",
                      RuntimeWarning, stacklevel=2)
    if path is None:
        _lib = lib
    return lib


def build_id() -> str:
    """MPIR_Hip_build_id: the source hashes and commit the library was built from."""
    return load().MPIR_Hip_build_id().decode()


def placement(dev: int = 0) -> dict:
    """MPIR_Hip_direct_placement for the calling thread: its CPU and NUMA node,
    device `dev`'s node, and the nodes of this thread's completion signal and of
    the device's error word (-1 where unknown or not yet created); `ring_in_vram`:
    MPIR_Hip_direct_ring_location (1 device memory, 0 host memory, -1 no queue)."""
    lib = load()
    out = (ctypes.c_int * 5)()
    lib.MPIR_Hip_direct_placement(dev, out)
    return {"cpu": out[0], "cpu_node": out[1], "gpu_node": out[2], "signal_node": out[3], "error_word_node": out[4],
            "ring_in_vram": lib.MPIR_Hip_direct_ring_location(dev)}


def error_class(code: int) -> int:
    """MPI_Error_class: the class of an error code (codes carry an error-stack
    index above the class bits, as MPICH's do)."""
    c = ctypes.c_int(-1)
    load().MPI_Error_class(code, ctypes.byref(c))
    return c.value


def error_string(code: int) -> str:
    lib = load()
    buf = ctypes.create_string_buffer(512)
    n = ctypes.c_int(0)
    lib.MPI_Error_string(code, buf, ctypes.byref(n))
    return buf.value.decode(errors="replace")


def fast_reduce_local():
    """The compiled binding of MPI_Reduce_local (csrc/py/fastcall.c, METH_FASTCALL):
    f(inbuf, inoutbuf, count, datatype, op) -> error code, ~0.25 us of Python
    overhead per call against ~1.2 us through ctypes.  Same library instance as
    load() (it is loaded first, so the errhandler and per-thread state are shared).
    Raises if the extension was not built."""
    load()
    from . import _fastcall
    return _fastcall.reduce_local


def fast_reduce_local_loop():
    """f(arg_sets, start, k) -> error code: k MPI_Reduce_local calls in a C loop
    (csrc/py/fastcall.c), call i with arg_sets[(start + i) % len(arg_sets)], the
    way a C caller issues them.  Raises if the extension was not built."""
    load()
    from . import _fastcall
    return _fastcall.reduce_local_loop


def reduce_local(inbuf: int, inoutbuf: int, count: int, datatype: int, op: int) -> int:
    """MPI_Reduce_local on raw addresses (device or host)."""
    return load().MPI_Reduce_local(ctypes.c_void_p(inbuf), ctypes.c_void_p(inoutbuf), count, datatype, op)


MPIX_ORDER_TREE = 0
MPIX_ORDER_CHAIN = 1


def reduce_local_multi(inbufs, outbuf: int, count: int, datatype: int, op: int, order: int,
                       stream: int = 0) -> int:
    """MPIX_Reduce_local_multi: outbuf = tree/chain fold of device buffers (addresses)."""
    arr = (ctypes.c_void_p * len(inbufs))(*inbufs)
    return load().MPIX_Reduce_local_multi(arr, len(inbufs), ctypes.c_void_p(outbuf), count, datatype, op, order,
                                          ctypes.c_void_p(stream or None))


MPIX_HIP_ALG_AUTO = 0
MPIX_HIP_ALG_REFERENCE_ORDER = 1
MPIX_HIP_ALG_RCCL = 2
MPI_IN_PLACE = ctypes.c_void_p(-1 & 0xFFFFFFFFFFFFFFFF).value


def comm_create_loopback(size: int):
    """`size` in-process virtual ranks on the current device (one thread each)."""
    arr = (ctypes.c_void_p * size)()
    rc = load().MPIX_Hip_comm_create_loopback(size, arr)
    if rc:
        raise RuntimeError(error_string(rc))
    return [arr[i] for i in range(size)]


def comm_free(comm) -> int:
    c = ctypes.c_void_p(comm)
    return load().MPIX_Hip_comm_free(ctypes.byref(c))


def allreduce(sendbuf, recvbuf: int, count: int, datatype: int, op: int, comm, algorithm: int = 0,
              stream: int = 0) -> int:
    return load().MPIX_Allreduce_hip(ctypes.c_void_p(sendbuf), ctypes.c_void_p(recvbuf), count, datatype, op,
                                     ctypes.c_void_p(comm), algorithm, ctypes.c_void_p(stream or None))


def reduce(sendbuf, recvbuf, count: int, datatype: int, op: int, root: int, comm, algorithm: int = 0,
           stream: int = 0) -> int:
    """MPIX_Reduce_hip (recvbuf significant at the root only; may be 0 elsewhere)."""
    return load().MPIX_Reduce_hip(ctypes.c_void_p(sendbuf), ctypes.c_void_p(recvbuf), count, datatype, op, root,
                                  ctypes.c_void_p(comm), algorithm, ctypes.c_void_p(stream or None))


def scan(sendbuf, recvbuf: int, count: int, datatype: int, op: int, comm, algorithm: int = 0,
         stream: int = 0) -> int:
    return load().MPIX_Scan_hip(ctypes.c_void_p(sendbuf), ctypes.c_void_p(recvbuf), count, datatype, op,
                                ctypes.c_void_p(comm), algorithm, ctypes.c_void_p(stream or None))


def exscan(sendbuf, recvbuf: int, count: int, datatype: int, op: int, comm, algorithm: int = 0,
           stream: int = 0) -> int:
    return load().MPIX_Exscan_hip(ctypes.c_void_p(sendbuf), ctypes.c_void_p(recvbuf), count, datatype, op,
                                  ctypes.c_void_p(comm), algorithm, ctypes.c_void_p(stream or None))


def reduce_scatter(sendbuf, recvbuf: int, recvcounts, datatype: int, op: int, comm, algorithm: int = 0,
                   stream: int = 0) -> int:
    """MPIX_Reduce_scatter_hip (per-rank recvcounts)."""
    arr = (ctypes.c_int * len(recvcounts))(*recvcounts)
    return load().MPIX_Reduce_scatter_hip(ctypes.c_void_p(sendbuf), ctypes.c_void_p(recvbuf), arr, datatype, op,
                                          ctypes.c_void_p(comm), algorithm, ctypes.c_void_p(stream or None))


def reduce_scatter_block(sendbuf, recvbuf: int, recvcount: int, datatype: int, op: int, comm,
                         algorithm: int = 0, stream: int = 0) -> int:
    return load().MPIX_Reduce_scatter_block_hip(ctypes.c_void_p(sendbuf), ctypes.c_void_p(recvbuf), recvcount,
                                                datatype, op, ctypes.c_void_p(comm), algorithm,
                                                ctypes.c_void_p(stream or None))


def reduce_local_stream(inbuf: int, inoutbuf: int, count: int, datatype: int, op: int, stream: int = 0) -> int:
    """MPIX_Reduce_local_stream: enqueue on a HIP stream (0 = library stream), no wait."""
    return load().MPIX_Reduce_local_stream(ctypes.c_void_p(inbuf), ctypes.c_void_p(inoutbuf), count,
                                           datatype, op, ctypes.c_void_p(stream or None))

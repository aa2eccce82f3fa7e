"""ctypes binding of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker / CPU baseline, never by the
product library (mpich-pip_amd/).  See op_oracle.c for what it restates.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
CLANG_LIB_PATH = os.path.join(HERE, "liboracle_clang.so")   # same sources, clang -O2 (CPU baseline only)
_lib = None
_clang = None


def _open(path: str) -> ctypes.CDLL:
    if not os.path.exists(path):
        raise RuntimeError(f"{path} missing: run `make -C oracle`")
    lib = ctypes.CDLL(path)
    vp, i32 = ctypes.c_void_p, ctypes.c_int
    for name in ("oracle_reduce_local", "oracle_reduce_local_nocheck"):
        f = getattr(lib, name)
        f.argtypes = [vp, vp, i32, i32, i32]
        f.restype = i32
    lib.oracle_cpu_baseline_sum_f32.argtypes = [i32, ctypes.c_long, i32]
    lib.oracle_cpu_baseline_sum_f32.restype = ctypes.c_double
    lib.oracle_cpu_baseline_sum_f32_pinned.argtypes = [i32, ctypes.POINTER(i32), ctypes.c_long, i32,
                                                       ctypes.POINTER(ctypes.c_double)]
    lib.oracle_cpu_baseline_sum_f32_pinned.restype = ctypes.c_double
    return lib


def load_clang() -> ctypes.CDLL:
    """The clang -O2 build of the same sources: a second CPU baseline, never the checker."""
    global _clang
    if _clang is None:
        _clang = _open(CLANG_LIB_PATH)
    return _clang


def load() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        lib = _open(LIB_PATH)
        i32 = ctypes.c_int
        lib.oracle_check_dtype.argtypes = [i32, i32]
        lib.oracle_check_dtype.restype = i32
        lib.oracle_h2f.argtypes = [ctypes.c_uint16]
        lib.oracle_h2f.restype = ctypes.c_float
        lib.oracle_f2h.argtypes = [ctypes.c_float]
        lib.oracle_f2h.restype = ctypes.c_uint16
        _lib = lib
    return _lib


def reduce_local(inbuf, inoutbuf, count: int, datatype: int, op: int, check: bool = True) -> int:
    """Oracle MPI_Reduce_local on numpy arrays (or raw addresses); inoutbuf updated in place."""
    lib = load()
    pin = inbuf.ctypes.data if hasattr(inbuf, "ctypes") else inbuf
    pio = inoutbuf.ctypes.data if hasattr(inoutbuf, "ctypes") else inoutbuf
    fn = lib.oracle_reduce_local if check else lib.oracle_reduce_local_nocheck
    return fn(ctypes.c_void_p(pin), ctypes.c_void_p(pio), count, datatype, op)


def check_dtype(op: int, datatype: int) -> int:
    return load().oracle_check_dtype(op, datatype)


def cpu_baseline_sum_f32(nthreads: int, count: int, iters: int, compiler: str = "gcc") -> float:
    """Seconds taken by the slowest of `nthreads` threads doing `iters` fp32 SUM calls of `count`
    (compiler "gcc": liboracle.so, MPICH's default build; "clang": liboracle_clang.so)."""
    lib = load_clang() if compiler == "clang" else load()
    return lib.oracle_cpu_baseline_sum_f32(nthreads, count, iters)


def physical_cores() -> list[tuple[int, int]]:
    """(logical cpu, socket) for one logical CPU per physical core among the
    CPUs this process may run on (sysfs topology: physical_package_id,
    core_id), lowest sibling first."""
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except AttributeError:
        allowed = list(range(os.cpu_count() or 1))
    seen, out = set(), []
    for c in allowed:
        base = f"/sys/devices/system/cpu/cpu{c}/topology/"
        try:
            pkg = int(open(base + "physical_package_id").read())
            core = int(open(base + "core_id").read())
        except (OSError, ValueError):
            pkg, core = 0, c
        if (pkg, core) not in seen:
            seen.add((pkg, core))
            out.append((c, pkg))
    return out


def cpu_quota() -> float | None:
    """CPUs' worth of time the cgroup grants this process (cgroup v2 cpu.max or
    v1 cfs quota / period), None when unlimited or unknown."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def spread_over_sockets(cores: list[tuple[int, int]], n: int) -> list[tuple[int, int]]:
    """n of the (cpu, socket) pairs, dealt round-robin over the sockets."""
    by = {}
    for c in cores:
        by.setdefault(c[1], []).append(c)
    out, k = [], 0
    while len(out) < min(n, len(cores)):
        for pkg in sorted(by):
            if k < len(by[pkg]) and len(out) < n:
                out.append(by[pkg][k])
        k += 1
    return out


def cpu_baseline_pinned(cpus: list[int], count: int, iters: int, compiler: str = "gcc") -> list[float]:
    """One thread pinned per listed CPU, NUMA-local first touch, barrier start;
    per-thread seconds for `iters` fp32 SUM calls of `count` (negative on failure)."""
    lib = load_clang() if compiler == "clang" else load()
    n = len(cpus)
    arr = (ctypes.c_int * n)(*cpus)
    secs = (ctypes.c_double * n)()
    lib.oracle_cpu_baseline_sum_f32_pinned(n, arr, count, iters, secs)
    return list(secs)

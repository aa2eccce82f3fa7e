#!/usr/bin/env python3
"""Why is bench.py's host_resident rate lower for pinned host buffers than for
pageable ones (117-122 against 200-265 GiB/s in round 3's bench lines)?  Both
take the same host combine.  For 256 MiB fp32 operands allocated several ways
this times, in one process:
  - numpy's single-thread read of one operand (np.sum) and copy (np.copyto);
  - MPI_Reduce_local on the pair (default dispatch: the host combine over the
    library's host threads), median of R calls;
and reports the NUMA node of each buffer's first page (move_pages).
  python3 tools/pinned_read_probe.py [R = 7]
"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))
import mpich_pip_amd as m  # noqa: E402

MIB = 1 << 20
N = 256 * MIB
R = int(sys.argv[1]) if len(sys.argv) > 1 else 7

libc = ctypes.CDLL(None, use_errno=True)
libc.syscall.restype = ctypes.c_long


def numa_node(addr: int) -> int:
    """move_pages(0, 1, [page], NULL, status, 0): the node the page sits on."""
    pages = (ctypes.c_void_p * 1)(addr & ~4095)
    status = (ctypes.c_int * 1)(-1)
    rc = libc.syscall(279, 0, 1, pages, None, status, 0)   # SYS_move_pages on x86-64
    return status[0] if rc == 0 else -100 - ctypes.get_errno()


hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]


def host_malloc(flags: int) -> np.ndarray:
    p = ctypes.c_void_p()
    rc = hip.hipHostMalloc(ctypes.byref(p), N, flags)
    assert rc == 0, rc
    a = np.ctypeslib.as_array((ctypes.c_float * (N // 4)).from_address(p.value))
    return a


def registered() -> np.ndarray:
    a = np.empty(N // 4, np.float32)
    a[:] = 0
    rc = hip.hipHostRegister(a.ctypes.data, N, 0)
    assert rc == 0, rc
    return a


def main():
    lib = m.load()
    lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN)
    rng = np.random.default_rng(1)
    src_a = rng.uniform(-1, 1, N // 4).astype(np.float32)
    src_b = rng.uniform(-1, 1, N // 4).astype(np.float32)
    kinds = {
        "pageable (numpy)": lambda: np.empty(N // 4, np.float32),
        "hipHostMalloc default": lambda: host_malloc(0x0),
        "hipHostMalloc NonCoherent": lambda: host_malloc(0x80000000),
        "hipHostMalloc Coherent": lambda: host_malloc(0x40000000),
        "hipHostRegister (numpy)": registered,
    }
    try:
        import torch
        kinds["torch pin_memory"] = lambda: torch.empty(N // 4, dtype=torch.float32).pin_memory().numpy()
    except Exception as exc:   # noqa: BLE001
        print("torch unavailable:", exc)
    for name, make in kinds.items():
        a, b = make(), make()
        np.copyto(a, src_a)
        np.copyto(b, src_b)
        t = []
        for _ in range(3):
            t0 = time.perf_counter()
            float(np.sum(b))
            t.append(time.perf_counter() - t0)
        read = N / min(t) / 2**30
        t = []
        for _ in range(3):
            t0 = time.perf_counter()
            np.copyto(a, b)
            t.append(time.perf_counter() - t0)
        copy = 2 * N / min(t) / 2**30
        np.copyto(a, src_a)
        t = []
        for _ in range(R):
            t0 = time.perf_counter()
            rc = lib.MPI_Reduce_local(b.ctypes.data, a.ctypes.data, N // 4, m.MPI_FLOAT, m.MPI_SUM)
            t.append(time.perf_counter() - t0)
            assert rc == 0, m.error_string(rc)
        t.sort()
        red = 3 * N / t[len(t) // 2] / 2**30
        print(f"{name:28s} node(a) {numa_node(a.ctypes.data):3d} node(b) {numa_node(b.ctypes.data):3d}  "
              f"np.sum read {read:7.1f} GiB/s  np.copyto {copy:7.1f} GiB/s  MPI_Reduce_local {red:7.1f} GiB/s "
              f"(median {t[len(t) // 2] * 1e3:.2f} ms)", flush=True)


if __name__ == "__main__" and not os.environ.get("BENCH_SEQ") and not os.environ.get("NUMA_SEQ"):
    main()


def bench_sequence():
    """bench.py's host legs verbatim: pinned copies of a device pair, pageable
    numpy copies of those, then the default-dispatch calls on each, alternated."""
    import torch
    lib = m.load()
    g = torch.Generator(device="cuda").manual_seed(5)
    a = torch.rand(N // 4, device="cuda", generator=g)
    b = torch.rand(N // 4, device="cuda", generator=g)
    ha, hb = a.cpu().pin_memory(), b.cpu().pin_memory()
    pa, pb = ha.numpy().copy(), hb.numpy().copy()
    # one checked call per kind first: the result is a + b exactly (fp32 SUM)
    want = ha.numpy() + hb.numpy()
    assert lib.MPI_Reduce_local(hb.data_ptr(), ha.data_ptr(), N // 4, m.MPI_FLOAT, m.MPI_SUM) == 0
    assert lib.MPI_Reduce_local(pb.ctypes.data, pa.ctypes.data, N // 4, m.MPI_FLOAT, m.MPI_SUM) == 0
    assert np.array_equal(ha.numpy(), want) and np.array_equal(pa, want), "host combine result"
    print(f"MPIR_CVAR_REDUCE_LOCAL_HOST_NUMA={os.environ.get('MPIR_CVAR_REDUCE_LOCAL_HOST_NUMA', '(default 1)')}")
    print(f"bench sequence: node(ha) {numa_node(ha.data_ptr())} node(hb) {numa_node(hb.data_ptr())} "
          f"node(pa) {numa_node(pa.ctypes.data)} node(pb) {numa_node(pb.ctypes.data)} main thread cpu {os.sched_getcpu() if hasattr(os, 'sched_getcpu') else '?'}")
    for rnd in range(3):
        for name, (x, y) in (("pinned", (hb.data_ptr(), ha.data_ptr())), ("pageable", (pb.ctypes.data, pa.ctypes.data))):
            t = []
            for _ in range(R):
                t0 = time.perf_counter()
                assert lib.MPI_Reduce_local(x, y, N // 4, m.MPI_FLOAT, m.MPI_SUM) == 0
                t.append(time.perf_counter() - t0)
            t.sort()
            print(f"  round {rnd} {name:9s} median {t[len(t) // 2] * 1e3:6.2f} ms = {3 * N / t[len(t) // 2] / 2**30:6.1f} GiB/s", flush=True)


if __name__ == "__main__" and os.environ.get("BENCH_SEQ"):
    bench_sequence()


def numa_sequence():
    """One pageable pair first-touched on each NUMA node (the main thread
    pinned there while it writes them), then, with the thread's full mask
    back, the default-dispatch call on each pair, alternated -- the floating
    pool (MPIR_CVAR_REDUCE_LOCAL_HOST_NUMA=0) against the node pools."""
    lib = m.load()
    full = os.sched_getaffinity(0)
    nodes = []
    for k in range(8):
        try:
            with open(f"/sys/devices/system/node/node{k}/cpulist") as f:
                txt = f.read().strip()
        except OSError:
            break
        cpus = set()
        for part in txt.split(","):
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
        nodes.append(cpus & full)
    rng = np.random.default_rng(3)
    src_a = rng.uniform(-1, 1, N // 4).astype(np.float32)
    src_b = rng.uniform(-1, 1, N // 4).astype(np.float32)
    pairs = []
    for k, cpus in enumerate(nodes):
        if not cpus:
            continue
        os.sched_setaffinity(0, cpus)
        a = np.empty(N // 4, np.float32)
        b = np.empty(N // 4, np.float32)
        np.copyto(a, src_a)
        np.copyto(b, src_b)
        os.sched_setaffinity(0, full)
        pairs.append((k, a, b))
    print(f"MPIR_CVAR_REDUCE_LOCAL_HOST_NUMA={os.environ.get('MPIR_CVAR_REDUCE_LOCAL_HOST_NUMA', '(default 1)')} "
          f"main thread mask {len(full)} CPUs; pairs on nodes "
          + ", ".join(f"{k}: ({numa_node(a.ctypes.data)}, {numa_node(b.ctypes.data)})" for k, a, b in pairs))
    for k, a, b in pairs:
        want = a + b
        assert lib.MPI_Reduce_local(b.ctypes.data, a.ctypes.data, N // 4, m.MPI_FLOAT, m.MPI_SUM) == 0
        assert np.array_equal(a, want), "host combine result"
    for rnd in range(3):
        for k, a, b in pairs:
            t = []
            for _ in range(R):
                t0 = time.perf_counter()
                assert lib.MPI_Reduce_local(b.ctypes.data, a.ctypes.data, N // 4, m.MPI_FLOAT, m.MPI_SUM) == 0
                t.append(time.perf_counter() - t0)
            t.sort()
            print(f"  round {rnd} pair on node {k}: median {t[len(t) // 2] * 1e3:6.2f} ms = "
                  f"{3 * N / t[len(t) // 2] / 2**30:6.1f} GiB/s", flush=True)


if __name__ == "__main__" and os.environ.get("NUMA_SEQ"):
    numa_sequence()

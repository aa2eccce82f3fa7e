"""Device collectives over RCCL (one process per rank): MPI_Allreduce and
MPI_Reduce at small sizes, MPI_Reduce_scatter_block (config 5's collective)
at small sizes, and configs 4 and 5 at their full BASELINE sizes.

Needs one GPU per rank: RCCL refuses two ranks of a communicator on one
device.  With fewer visible GPUs the multi-rank cases skip; the reference-order
algorithm itself is covered on one GPU by test_coll_loopback_gpu.py (same code,
loopback transport).  A 1-rank RCCL communicator always runs here, which
exercises dlopen of librccl, ncclCommInitRank and both algorithms.
"""
import multiprocessing as mp
import os

import numpy as np
import pytest

import _types as T

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rank_main(rank, size, uid, q, cases):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes
    import torch
    import mpich_pip_amd as mpi
    import _types as T
    torch.cuda.set_device(rank)
    lib = mpi.load()
    lib.MPIX_Reduce_local_set_errhandler(mpi.MPI_ERRORS_RETURN)
    comm = ctypes.c_void_p()
    rc = lib.MPIX_Hip_comm_create(ctypes.c_char_p(uid), size, rank, ctypes.byref(comm))
    if rc:
        q.put((rank, "create", rc, mpi.error_string(rc)))
        return
    out = []
    for kind, t, op, count, alg in cases:
        rng = np.random.default_rng(1000 + rank)
        x = T.to_bytes(T.gen(t, count, rng, op, specials=False))
        send = torch.from_numpy(x.copy()).cuda()
        recv = torch.zeros_like(send)
        torch.cuda.synchronize()
        if kind == "rsb":   # count = recvcount; every rank sends count * size elements
            x = T.to_bytes(T.gen(t, count * size, rng, op, specials=False))
            send = torch.from_numpy(x.copy()).cuda()
            recv = torch.zeros(count * T.elem_size(t), dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            rc = mpi.reduce_scatter_block(send.data_ptr(), recv.data_ptr(), count, mpi.DATATYPES[t], mpi.OPS[op],
                                          comm.value, alg)
        elif kind == "allreduce":
            rc = mpi.allreduce(send.data_ptr(), recv.data_ptr(), count, mpi.DATATYPES[t], mpi.OPS[op], comm.value,
                               alg)
        else:   # reduce to the last rank; recvbuf NULL elsewhere
            root = size - 1
            rc = mpi.reduce(send.data_ptr(), recv.data_ptr() if rank == root else 0, count, mpi.DATATYPES[t],
                            mpi.OPS[op], root, comm.value, alg)
        torch.cuda.synchronize()
        out.append((rc, x, recv.cpu().numpy()))
    q.put((rank, "ok", 0, out))
    mpi.comm_free(comm.value)


def _run(size, cases):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))
    import ctypes
    import mpich_pip_amd as mpi
    uid = ctypes.create_string_buffer(128)
    assert mpi.load().MPIX_Hip_comm_get_unique_id(uid) == 0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, size, uid.raw, q, cases)) for r in range(size)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(size):
        r = q.get(timeout=300)
        res[r[0]] = r
    for p in procs:
        p.join(60)
    return res


def _ngpus():
    import torch
    return torch.cuda.device_count()


def _gamma(k, u):
    return k * u / (1 - k * u)


@pytest.mark.parametrize("size", [1, 2, 4, 8])
def test_allreduce_and_reduce_over_rccl(mpi, orc, cuda, size):
    from oracle import schedules as S
    if _ngpus() < size:
        pytest.skip(f"needs {size} GPUs, {_ngpus()} visible")
    REF, RCCL = mpi.MPIX_HIP_ALG_REFERENCE_ORDER, mpi.MPIX_HIP_ALG_RCCL
    cases = [("allreduce", "MPI_FLOAT", "MPI_SUM", (1 << 20) + 3, REF),
             ("allreduce", "MPI_FLOAT", "MPI_SUM", (1 << 20) + 3, RCCL),
             ("allreduce", "MPI_INT", "MPI_SUM", 4099, RCCL),
             ("allreduce", "MPIX_C_FLOAT16", "MPI_SUM", 4099, REF),
             ("allreduce", "MPI_DOUBLE", "MPI_MAX", 100, REF),
             ("reduce", "MPI_FLOAT", "MPI_SUM", (1 << 20) + 3, REF),
             ("reduce", "MPI_FLOAT", "MPI_SUM", (1 << 20) + 3, RCCL),
             ("reduce", "MPI_INT", "MPI_SUM", 77, RCCL),
             ("reduce", "MPI_DOUBLE", "MPI_SUM", 77, REF)]
    res = _run(size, cases)
    for r in range(size):
        assert res[r][1] == "ok", res[r]
    for k, (kind, t, op, count, alg) in enumerate(cases):
        xs = [res[r][3][k][1] for r in range(size)]
        esz = T.elem_size(t)
        if kind == "allreduce":
            want = S.allreduce_smp_auto(xs, count, esz, mpi.DATATYPES[t], mpi.OPS[op]) if size > 1 else xs[0]
            checked = range(size)
        else:
            want = S.reduce_auto(xs, count, esz, mpi.DATATYPES[t], mpi.OPS[op], size - 1)
            checked = [size - 1]
        for r in range(size):
            assert res[r][3][k][0] == 0, (kind, t, alg, r)
        for r in checked:
            rc, _, got = res[r][3][k]
            if alg == mpi.MPIX_HIP_ALG_REFERENCE_ORDER or t == "MPI_INT":
                assert np.array_equal(got, want), (t, alg, r)
            else:
                # RCCL's own order: |got - ref| <= gamma_{p-1} * sum|x_i|
                g = got.view(np.float32).astype(np.float64)
                w = want.view(np.float32).astype(np.float64)
                mag = np.sum([np.abs(x.view(np.float32).astype(np.float64)) for x in xs], axis=0)
                u = 2.0 ** -24
                gamma = (size - 1) * u / (1 - (size - 1) * u)
                assert np.all(np.abs(g - w) <= gamma * mag + 1e-45), (t, r)


@pytest.mark.parametrize("size", [1, 2, 4, 8])
def test_reduce_scatter_block_over_rccl(mpi, orc, cuda, size):
    """Config 5's collective (reduce_scatter_block_intra_pairwise.c:97-140) at
    N ranks, one per GPU: reference order bit-exact against the oracle's
    step-by-step schedule with MPICH's algorithm choice (pairwise from 512 KiB
    of sendbuf, recursive halving below: reduce_scatter_block.c:136-148);
    RCCL's ncclReduceScatter within 2 gamma_{p-1} of it for fp16 / fp32 (both
    chains round at every step), exact for int32."""
    from oracle import schedules as S
    if _ngpus() < size:
        pytest.skip(f"needs {size} GPUs, {_ngpus()} visible")
    REF, RCCL = mpi.MPIX_HIP_ALG_REFERENCE_ORDER, mpi.MPIX_HIP_ALG_RCCL
    big = (1 << 17) + 3            # size * big * 2 B >= 524288 at every N >= 2: pairwise
    cases = [("rsb", "MPIX_C_FLOAT16", "MPI_SUM", big, REF),
             ("rsb", "MPIX_C_FLOAT16", "MPI_SUM", big, RCCL),
             ("rsb", "MPIX_C_FLOAT16", "MPI_SUM", 1000, REF),          # recursive halving
             ("rsb", "MPI_FLOAT", "MPI_SUM", 4099, REF),
             ("rsb", "MPI_FLOAT", "MPI_SUM", 4099, RCCL),
             ("rsb", "MPI_INT", "MPI_SUM", 77777, RCCL),
             ("rsb", "MPI_DOUBLE", "MPI_MAX", 4099, REF)]
    res = _run(size, cases)
    for r in range(size):
        assert res[r][1] == "ok", res[r]
    for k, (kind, t, op, count, alg) in enumerate(cases):
        xs = [res[r][3][k][1] for r in range(size)]
        esz = T.elem_size(t)
        want = S.reduce_scatter_block_auto(xs, count, esz, mpi.DATATYPES[t], mpi.OPS[op])
        for r in range(size):
            rc, _, got = res[r][3][k]
            assert rc == 0, (t, alg, r)
            if alg == REF or t == "MPI_INT" or size == 1:
                assert np.array_equal(got, want[r]), (t, count, alg, r)
                continue
            ft, u = (np.float16, 2.0 ** -11) if t == "MPIX_C_FLOAT16" else (np.float32, 2.0 ** -24)
            g = got.view(ft).astype(np.float64)
            w = want[r].view(ft).astype(np.float64)
            blk = slice(r * count, (r + 1) * count)
            mag = np.sum([np.abs(x.view(ft)[blk].astype(np.float64)) for x in xs], axis=0)
            tiny = 2.0 ** -24 if ft == np.float16 else 1e-45
            assert np.all(np.abs(g - w) <= 2 * _gamma(size - 1, u) * mag + tiny), (t, r)


def _config_rank_main(rank, size, uid, q, alg):
    """One rank of the config-size cases.  Every rank derives every rank's
    input from seeds -- allreduce: rank j's 256 MiB fp32 buffer is 8 chunks
    seeded (j, c); reduce-scatter: rank j's 1 GiB fp16 sendbuf is `size`
    blocks seeded (j, b) -- so it can check its own result without receiving
    anyone's data.  Expected values (numpy; fp32 / fp16 adds round like the
    reference's, pinned by tests/test_bench_selfcheck_cpu.py): allreduce in
    reduce_intra_reduce_scatter_gather.c's tree order per block (pof2 N), the
    pairwise chain per output block; RCCL against the exact (float64) sum
    within gamma_{p-1} (fp32) / 2 gamma_{p-1} (fp16, both chains round)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "mpich-pip_amd"))
    sys.path.insert(0, ROOT)
    import ctypes
    import torch
    import mpich_pip_amd as mpi
    from bench_coll import expect_allreduce
    torch.cuda.set_device(rank)
    lib = mpi.load()
    lib.MPIX_Reduce_local_set_errhandler(mpi.MPI_ERRORS_RETURN)
    comm = ctypes.c_void_p()
    rc = lib.MPIX_Hip_comm_create(ctypes.c_char_p(uid), size, rank, ctypes.byref(comm))
    if rc:
        q.put((rank, "create", rc, mpi.error_string(rc)))
        return
    out = {}
    # ---- config 4: MPI_Allreduce fp32 SUM, 256 MiB per rank
    n = 64 << 20
    chunks = 8

    def ar_input(j):
        return np.concatenate([np.random.default_rng((j, c, 4)).uniform(-1, 1, n // chunks).astype(np.float32)
                               for c in range(chunks)])
    xs = [ar_input(j) for j in range(size)]
    send = torch.from_numpy(xs[rank]).cuda()
    recv = torch.empty_like(send)
    torch.cuda.synchronize()
    rc = mpi.allreduce(send.data_ptr(), recv.data_ptr(), n, mpi.MPI_FLOAT, mpi.MPI_SUM, comm.value, alg)
    torch.cuda.synchronize()
    got = recv.cpu().numpy()
    del send, recv
    pof2 = size & (size - 1) == 0
    if alg == mpi.MPIX_HIP_ALG_REFERENCE_ORDER and pof2:
        out["allreduce"] = (rc, bool(np.array_equal(got.view(np.uint32), expect_allreduce(xs).view(np.uint32))))
    else:
        exact = np.sum([x.astype(np.float64) for x in xs], axis=0)
        mag = np.sum([np.abs(x.astype(np.float64)) for x in xs], axis=0)
        ok = np.all(np.abs(got.astype(np.float64) - exact) <= _gamma(max(size - 1, 1), 2.0 ** -24) * mag + 1e-45)
        out["allreduce"] = (rc, bool(ok))
    del xs, got
    # ---- config 5: MPI_Reduce_scatter_block fp16 SUM, 1 GiB sendbuf per rank
    total = 1 << 29
    rcnt = total // size

    def rs_block(j, b):
        return np.random.default_rng((j, b, 5)).uniform(-4, 4, rcnt).astype(np.float16)
    send = torch.from_numpy(np.concatenate([rs_block(rank, b) for b in range(size)])).cuda()
    recv = torch.empty(rcnt, dtype=torch.float16, device="cuda")
    torch.cuda.synchronize()
    rc = mpi.reduce_scatter_block(send.data_ptr(), recv.data_ptr(), rcnt, mpi.MPIX_C_FLOAT16, mpi.MPI_SUM,
                                  comm.value, alg)
    torch.cuda.synchronize()
    got = recv.cpu().numpy()
    del send, recv
    mine = [rs_block(j, rank) for j in range(size)]
    acc = mine[rank].copy()                      # ((x_r + x_{r-1}) + x_{r-2}) + ...
    for i in range(1, size):
        acc = acc + mine[(rank - i) % size]
    if alg == mpi.MPIX_HIP_ALG_REFERENCE_ORDER:
        out["reduce_scatter_block"] = (rc, bool(np.array_equal(got.view(np.uint16), acc.view(np.uint16))))
    else:
        mag = np.sum([np.abs(x.astype(np.float64)) for x in mine], axis=0)
        ok = np.all(np.abs(got.astype(np.float64) - acc.astype(np.float64)) <=
                    2 * _gamma(max(size - 1, 1), 2.0 ** -11) * mag + 2.0 ** -24)
        out["reduce_scatter_block"] = (rc, bool(ok))
    q.put((rank, "ok", 0, out))
    mpi.comm_free(comm.value)


@pytest.mark.parametrize("alg", ["reference_order", "rccl"])
@pytest.mark.parametrize("size", [1, 2, 4, 8])
def test_config_size_collectives_over_rccl(mpi, cuda, size, alg):
    """BASELINE configs 4 and 5 at full size: MPI_Allreduce fp32 SUM of 256 MiB
    per rank and MPI_Reduce_scatter_block fp16 SUM of a 1 GiB sendbuf per rank
    (recvcount 2^29 / N), one rank per GPU, both algorithms."""
    if _ngpus() < size:
        pytest.skip(f"needs {size} GPUs, {_ngpus()} visible")
    import ctypes
    a = mpi.MPIX_HIP_ALG_REFERENCE_ORDER if alg == "reference_order" else mpi.MPIX_HIP_ALG_RCCL
    uid = ctypes.create_string_buffer(128)
    assert mpi.load().MPIX_Hip_comm_get_unique_id(uid) == 0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_config_rank_main, args=(r, size, uid.raw, q, a)) for r in range(size)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(size):
        r = q.get(timeout=600)
        res[r[0]] = r
    for p in procs:
        p.join(60)
    for r in range(size):
        assert res[r][1] == "ok", res[r]
        for name, (rc, ok) in res[r][3].items():
            assert rc == 0 and ok, (name, alg, r)

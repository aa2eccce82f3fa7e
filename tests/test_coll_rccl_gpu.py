"""Device collectives over RCCL (one process per rank).

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
        if kind == "allreduce":
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

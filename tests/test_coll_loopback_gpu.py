"""Device collectives (MPIX_Allreduce_hip, MPIX_Reduce_scatter_block_hip) on one GPU.

The loopback communicator runs p virtual ranks in this process (one host
thread each, transfers are device copies), so the complete reference-order
algorithm -- pre-fold, all-to-all of blocks, fused tree/chain combine,
allgather -- runs end to end on one MI355X.  The RCCL communicator differs
only in its transport (grouped ncclSend/ncclRecv) and needs one GPU per rank.
Expected bytes: oracle/schedules.py, the reference schedules run step by step
on the CPU oracle.  Bit-exact (complex NaN payloads excepted).
"""
import threading

import numpy as np
import pytest

import _types as T
from test_parity_gpu import same

pytestmark = pytest.mark.gpu


def run_ranks(fn, p, timeout=120):
    errs = [None] * p

    def wrap(r):
        try:
            fn(r)
        except BaseException as e:  # noqa: BLE001
            errs[r] = e

    ths = [threading.Thread(target=wrap, args=(r,), daemon=True) for r in range(p)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout)
        if t.is_alive():
            pytest.fail("collective did not complete (deadlock?)")
    for e in errs:
        if e is not None:
            raise e


CASES = [("MPI_FLOAT", "MPI_SUM"), ("MPIX_C_FLOAT16", "MPI_SUM"), ("MPI_INT", "MPI_SUM"),
         ("MPI_DOUBLE", "MPI_MAX"), ("MPI_UNSIGNED_CHAR", "MPI_BXOR"), ("MPI_C_DOUBLE_COMPLEX", "MPI_SUM"),
         ("MPI_DOUBLE_INT", "MPI_MAXLOC"), ("MPI_LONG_DOUBLE", "MPI_SUM"), ("MPI_C_LONG_DOUBLE_COMPLEX", "MPI_PROD")]


@pytest.mark.parametrize("t,op", CASES, ids=[f"{t}-{o}" for t, o in CASES])
@pytest.mark.parametrize("p", [1, 2, 3, 4, 5, 8])
@pytest.mark.parametrize("inplace", [False, True])
def test_allreduce_reference_order(mpi, orc, cuda, t, op, p, inplace):
    from oracle import schedules as S
    torch = cuda
    esz = T.elem_size(t)
    comms = mpi.comm_create_loopback(p)
    try:
        for count, seed in ((1003, p), (3, 11), ((1 << 19) + 3, 5 * p)):
            rng = np.random.default_rng(seed)
            xs = [T.to_bytes(T.gen(t, count, rng, op)) for _ in range(p)]
            if p > 1:
                want = S.allreduce_smp_auto(xs, count, esz, mpi.DATATYPES[t], mpi.OPS[op])
            else:
                want = xs[0]
            send = [torch.from_numpy(x.copy()).cuda() for x in xs]
            recv = [s.clone() if inplace else torch.zeros_like(s) for s in send]
            torch.cuda.synchronize()

            def rank(r):
                sb = mpi.MPI_IN_PLACE if inplace else send[r].data_ptr()
                rc = mpi.allreduce(sb, recv[r].data_ptr(), count, mpi.DATATYPES[t], mpi.OPS[op], comms[r],
                                   mpi.MPIX_HIP_ALG_REFERENCE_ORDER)
                assert rc == 0, mpi.error_string(rc)

            run_ranks(rank, p)
            torch.cuda.synchronize()
            for r in range(p):
                got = recv[r].cpu().numpy()
                assert same(got, want, t), f"rank {r} count {count}: {np.count_nonzero(got != want)} bytes differ"
    finally:
        for c in comms:
            mpi.comm_free(c)


@pytest.mark.parametrize("t,op", [("MPIX_C_FLOAT16", "MPI_SUM"), ("MPI_FLOAT", "MPI_SUM"), ("MPI_INT64_T", "MPI_PROD"),
                                  ("MPI_UNSIGNED", "MPI_BAND"), ("MPI_FLOAT", "MPI_MIN"),
                                  ("MPI_LONG_DOUBLE_INT", "MPI_MINLOC")])
@pytest.mark.parametrize("p", [1, 2, 3, 5, 6, 8])
@pytest.mark.parametrize("inplace", [False, True])
def test_reduce_scatter_block_reference_order(mpi, orc, cuda, t, op, p, inplace):
    from oracle import schedules as S
    torch = cuda
    esz = T.elem_size(t)
    comms = mpi.comm_create_loopback(p)
    try:
        for recvcount, seed in ((2053, p), ((1 << 18) + 1, 3 * p)):
            rng = np.random.default_rng(seed)
            xs = [T.to_bytes(T.gen(t, recvcount * p, rng, op)) for _ in range(p)]
            want = S.reduce_scatter_block_auto(xs, recvcount, esz, mpi.DATATYPES[t], mpi.OPS[op])
            send = [torch.from_numpy(x.copy()).cuda() for x in xs]
            recv = [s.clone() if inplace else torch.zeros(recvcount * esz, dtype=torch.uint8, device="cuda")
                    for s in send]
            torch.cuda.synchronize()

            def rank(r):
                sb = mpi.MPI_IN_PLACE if inplace else send[r].data_ptr()
                rc = mpi.reduce_scatter_block(sb, recv[r].data_ptr(), recvcount, mpi.DATATYPES[t], mpi.OPS[op],
                                              comms[r], mpi.MPIX_HIP_ALG_REFERENCE_ORDER)
                assert rc == 0, mpi.error_string(rc)

            run_ranks(rank, p)
            torch.cuda.synchronize()
            for r in range(p):
                got = recv[r][:recvcount * esz].cpu().numpy()
                assert same(got, want[r], t), f"rank {r}"
    finally:
        for c in comms:
            mpi.comm_free(c)


SWITCH = [("MPI_FLOAT", "MPI_SUM"), ("MPI_DOUBLE", "MPI_MAX"), ("MPIX_C_FLOAT16", "MPI_MIN")]


@pytest.mark.parametrize("t,op", SWITCH, ids=[f"{t}-{o}" for t, o in SWITCH])
@pytest.mark.parametrize("p", [6, 8])
def test_algorithm_switch_points(mpi, orc, cuda, t, op, p):
    """Both sides of MPICH's size thresholds: Allreduce binomial <= 2048 B <
    reduce-scatter-gather (reduce.c:214); Reduce_scatter_block recursive halving
    < 524288 total bytes <= pairwise (reduce_scatter_block.c:136-141)."""
    from oracle import schedules as S
    torch = cuda
    esz = T.elem_size(t)
    dt, o = mpi.DATATYPES[t], mpi.OPS[op]
    comms = mpi.comm_create_loopback(p)
    try:
        for count in (2048 // esz, 2048 // esz + 1):
            rng = np.random.default_rng(count + p)
            xs = [T.to_bytes(T.gen(t, count, rng, op)) for _ in range(p)]
            want = S.allreduce_smp_auto(xs, count, esz, dt, o)
            send = [torch.from_numpy(x.copy()).cuda() for x in xs]
            recv = [torch.zeros_like(x) for x in send]
            torch.cuda.synchronize()
            run_ranks(lambda r: _ok(mpi, mpi.allreduce(send[r].data_ptr(), recv[r].data_ptr(), count, dt, o,
                                                       comms[r], mpi.MPIX_HIP_ALG_REFERENCE_ORDER)), p)
            torch.cuda.synchronize()
            for r in range(p):
                assert same(recv[r].cpu().numpy(), want, t), f"allreduce count {count} rank {r}"
        first_long = -(-S.RSB_COMMUTATIVE_LONG_MSG_SIZE // (p * esz))
        for rc in (first_long - 1, first_long):
            rng = np.random.default_rng(rc + p)
            xs = [T.to_bytes(T.gen(t, rc * p, rng, op)) for _ in range(p)]
            want = S.reduce_scatter_block_auto(xs, rc, esz, dt, o)
            send = [torch.from_numpy(x.copy()).cuda() for x in xs]
            recv = [torch.zeros(rc * esz, dtype=torch.uint8, device="cuda") for _ in range(p)]
            torch.cuda.synchronize()
            run_ranks(lambda r: _ok(mpi, mpi.reduce_scatter_block(send[r].data_ptr(), recv[r].data_ptr(), rc, dt,
                                                                  o, comms[r], mpi.MPIX_HIP_ALG_REFERENCE_ORDER)), p)
            torch.cuda.synchronize()
            for r in range(p):
                assert same(recv[r].cpu().numpy(), want[r], t), f"reduce_scatter_block recvcount {rc} rank {r}"
    finally:
        for c in comms:
            mpi.comm_free(c)


RCASES = [("MPI_FLOAT", "MPI_SUM"), ("MPIX_C_FLOAT16", "MPI_SUM"), ("MPI_DOUBLE", "MPI_MAX"),
          ("MPI_INT64_T", "MPI_PROD"), ("MPI_DOUBLE_INT", "MPI_MINLOC")]


@pytest.mark.parametrize("t,op", RCASES, ids=[f"{t}-{o}" for t, o in RCASES])
@pytest.mark.parametrize("p", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("inplace", [False, True])
def test_reduce_reference_order(mpi, orc, cuda, t, op, p, inplace):
    """MPIX_Reduce_hip at every root: binomial (short) and reduce-scatter + gather
    (long) vs the step-by-step schedules; non-root recvbufs are NULL and the
    root's recvbuf is the only buffer written."""
    from oracle import schedules as S
    torch = cuda
    esz = T.elem_size(t)
    dt, o = mpi.DATATYPES[t], mpi.OPS[op]
    comms = mpi.comm_create_loopback(p)
    try:
        for count, seed in ((3, 7 * p), (2048 // esz, p), ((1 << 16) + 5, 3 * p)):
            rng = np.random.default_rng(seed)
            xs = [T.to_bytes(T.gen(t, count, rng, op)) for _ in range(p)]
            send = [torch.from_numpy(x.copy()).cuda() for x in xs]
            for root in range(p):
                want = S.reduce_auto(xs, count, esz, dt, o, root)
                rbuf = send[root].clone() if inplace else torch.zeros_like(send[root])
                keep = [s.clone() for s in send]
                torch.cuda.synchronize()

                def rank(r):
                    sb = mpi.MPI_IN_PLACE if (inplace and r == root) else send[r].data_ptr()
                    rb = rbuf.data_ptr() if r == root else 0
                    _ok(mpi, mpi.reduce(sb, rb, count, dt, o, root, comms[r], mpi.MPIX_HIP_ALG_REFERENCE_ORDER))

                run_ranks(rank, p)
                torch.cuda.synchronize()
                got = rbuf.cpu().numpy()
                bad = np.nonzero((got != want).reshape(-1, esz).any(axis=1))[0][:4]
                assert same(got, want, t), f"count {count} root {root}: elements {bad} got " \
                    f"{[bytes(got[i * esz:(i + 1) * esz]).hex() for i in bad]} want " \
                    f"{[bytes(want[i * esz:(i + 1) * esz]).hex() for i in bad]}"
                for r in range(p):      # sendbufs are read-only
                    assert torch.equal(send[r], keep[r]), f"rank {r} sendbuf modified"
    finally:
        for c in comms:
            mpi.comm_free(c)


RSCASES = [("MPI_FLOAT", "MPI_SUM"), ("MPIX_C_FLOAT16", "MPI_SUM"), ("MPI_DOUBLE", "MPI_MIN"),
           ("MPI_INT", "MPI_BXOR"), ("MPI_FLOAT_INT", "MPI_MAXLOC")]


@pytest.mark.parametrize("t,op", RSCASES, ids=[f"{t}-{o}" for t, o in RSCASES])
@pytest.mark.parametrize("p", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("inplace", [False, True])
def test_reduce_scatter_reference_order(mpi, orc, cuda, t, op, p, inplace):
    """MPIX_Reduce_scatter_hip with per-rank counts (zeros and a count larger
    than its displacement included, so the in-place output overlaps the
    rank's own block): recursive halving (short) and pairwise (long) vs the
    step-by-step schedules."""
    from oracle import schedules as S
    torch = cuda
    esz = T.elem_size(t)
    dt, o = mpi.DATATYPES[t], mpi.OPS[op]
    comms = mpi.comm_create_loopback(p)
    try:
        for scale, seed in ((1, p), (4096, 3 * p)):
            rng = np.random.default_rng(seed)
            counts = [int(c) * scale + int(rng.integers(0, 3)) for c in rng.integers(0, 9, p)]
            if p > 2:
                counts[1] = 0
            if p > 1:
                counts[-1] = sum(counts[:-1]) + 5
            total = sum(counts)
            xs = [T.to_bytes(T.gen(t, total, rng, op)) for _ in range(p)]
            want = S.reduce_scatter_auto(xs, counts, esz, dt, o)
            send = [torch.from_numpy(x.copy()).cuda() for x in xs]
            recv = [s.clone() if inplace else torch.zeros(max(1, c) * esz, dtype=torch.uint8, device="cuda")
                    for s, c in zip(send, counts)]
            torch.cuda.synchronize()

            def rank(r):
                sb = mpi.MPI_IN_PLACE if inplace else send[r].data_ptr()
                _ok(mpi, mpi.reduce_scatter(sb, recv[r].data_ptr(), counts, dt, o, comms[r],
                                            mpi.MPIX_HIP_ALG_REFERENCE_ORDER))

            run_ranks(rank, p)
            torch.cuda.synchronize()
            for r in range(p):
                got = recv[r][:counts[r] * esz].cpu().numpy()
                assert same(got, want[r], t), f"counts {counts} rank {r}"
    finally:
        for c in comms:
            mpi.comm_free(c)


SCASES = [("MPI_FLOAT", "MPI_SUM"), ("MPIX_C_FLOAT16", "MPI_SUM"), ("MPI_DOUBLE", "MPI_MAX"),
          ("MPI_LONG", "MPI_PROD"), ("MPI_2INT", "MPI_MINLOC"), ("MPI_C_FLOAT_COMPLEX", "MPI_SUM")]


@pytest.mark.parametrize("t,op", SCASES, ids=[f"{t}-{o}" for t, o in SCASES])
@pytest.mark.parametrize("p", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("inplace", [False, True])
@pytest.mark.parametrize("exclusive", [False, True])
def test_scan_reference_order(mpi, orc, cuda, t, op, p, inplace, exclusive):
    """MPIX_Scan_hip / MPIX_Exscan_hip vs the step-by-step recursive doubling;
    the exscan leaves rank 0's recvbuf untouched."""
    from oracle import schedules as S
    torch = cuda
    esz = T.elem_size(t)
    dt, o = mpi.DATATYPES[t], mpi.OPS[op]
    fn = mpi.exscan if exclusive else mpi.scan
    sim = S.exscan_recursive_doubling if exclusive else S.scan_recursive_doubling
    comms = mpi.comm_create_loopback(p)
    try:
        for count, seed in ((5, p), ((1 << 17) + 3, 3 * p)):
            rng = np.random.default_rng(seed)
            xs = [T.to_bytes(T.gen(t, count, rng, op)) for _ in range(p)]
            want = sim(xs, count, esz, dt, o)
            send = [torch.from_numpy(x.copy()).cuda() for x in xs]
            recv = [s.clone() if inplace else torch.full_like(s, 0xA5) for s in send]
            before0 = recv[0].clone()
            torch.cuda.synchronize()

            def rank(r):
                sb = mpi.MPI_IN_PLACE if inplace else send[r].data_ptr()
                _ok(mpi, fn(sb, recv[r].data_ptr(), count, dt, o, comms[r], mpi.MPIX_HIP_ALG_REFERENCE_ORDER))

            run_ranks(rank, p)
            torch.cuda.synchronize()
            for r in range(p):
                got = recv[r].cpu().numpy()
                if exclusive and r == 0:
                    assert torch.equal(recv[0], before0), "exscan wrote rank 0's recvbuf"
                    continue
                assert same(got, want[r], t), f"count {count} rank {r}"
    finally:
        for c in comms:
            mpi.comm_free(c)


FLAT = [("MPI_FLOAT", "MPI_SUM"), ("MPI_DOUBLE", "MPI_MAX"), ("MPIX_C_FLOAT16", "MPI_SUM"), ("MPI_2INT", "MPI_MAXLOC")]


@pytest.mark.parametrize("t,op", FLAT, ids=[f"{t}-{o}" for t, o in FLAT])
@pytest.mark.parametrize("p", [2, 3, 5, 8])
@pytest.mark.parametrize("cvars", ["smp_off", "max_smp_1"])
def test_allreduce_flat_branch(mpi, orc, cuda, t, op, p, cvars, monkeypatch):
    """MPIR_Allreduce_intra_auto's flat branch, selected by the reference's CVARs:
    MPIR_CVAR_ENABLE_SMP_COLLECTIVES=0 (recursive doubling at every size: nbytes
    is 0 while MAX_SMP_ALLREDUCE_MSG_SIZE is 0) and
    MPIR_CVAR_MAX_SMP_ALLREDUCE_MSG_SIZE=1 (recursive doubling short,
    Rabenseifner long).  Per-rank results vs the step-by-step schedules."""
    from oracle import schedules as S
    torch = cuda
    esz = T.elem_size(t)
    dt, o = mpi.DATATYPES[t], mpi.OPS[op]
    if cvars == "smp_off":
        monkeypatch.setenv("MPIR_CVAR_ENABLE_SMP_COLLECTIVES", "0")
        kw = dict(smp=False)
    else:
        monkeypatch.setenv("MPIR_CVAR_MAX_SMP_ALLREDUCE_MSG_SIZE", "1")
        kw = dict(smp=True, max_smp=1)
    comms = mpi.comm_create_loopback(p)
    try:
        for count, seed in ((3, p), (2048 // esz + 1, 2 * p), ((1 << 17) + 7, 3 * p)):
            rng = np.random.default_rng(seed)
            xs = [T.to_bytes(T.gen(t, count, rng, op)) for _ in range(p)]
            want = S.allreduce_auto(xs, count, esz, dt, o, **kw)
            send = [torch.from_numpy(x.copy()).cuda() for x in xs]
            recv = [torch.zeros_like(x) for x in send]
            torch.cuda.synchronize()
            run_ranks(lambda r: _ok(mpi, mpi.allreduce(send[r].data_ptr(), recv[r].data_ptr(), count, dt, o,
                                                       comms[r], mpi.MPIX_HIP_ALG_REFERENCE_ORDER)), p)
            torch.cuda.synchronize()
            for r in range(p):
                assert same(recv[r].cpu().numpy(), want[r], t), f"count {count} rank {r}"
    finally:
        for c in comms:
            mpi.comm_free(c)


def test_reduce_validation(mpi, cuda):
    torch = cuda
    comms = mpi.comm_create_loopback(2)
    try:
        a = torch.ones(4, device="cuda")
        b = torch.zeros(4, device="cuda")
        REF = mpi.MPIX_HIP_ALG_REFERENCE_ORDER
        # invalid root -> MPI_ERR_ROOT (class 7)
        assert mpi.reduce(a.data_ptr(), b.data_ptr(), 4, mpi.MPI_FLOAT, mpi.MPI_SUM, 2, comms[0], REF) & 0x7f == 7
        assert mpi.reduce(a.data_ptr(), b.data_ptr(), 4, mpi.MPI_FLOAT, mpi.MPI_SUM, -1, comms[0], REF) & 0x7f == 7
        # MPI_IN_PLACE at a non-root -> MPI_ERR_BUFFER
        assert mpi.reduce(mpi.MPI_IN_PLACE, 0, 4, mpi.MPI_FLOAT, mpi.MPI_SUM, 0, comms[1], REF) & 0x7f == 1
        # aliased buffers at the root -> MPI_ERR_BUFFER
        assert mpi.reduce(a.data_ptr(), a.data_ptr(), 4, mpi.MPI_FLOAT, mpi.MPI_SUM, 0, comms[0], REF) & 0x7f == 1
        # MPI_REPLACE is not a reduction op
        assert mpi.reduce(a.data_ptr(), b.data_ptr(), 4, mpi.MPI_FLOAT, mpi.MPI_REPLACE, 0, comms[0], REF) \
            & 0x7f == 9
        # count 0 is a no-op
        assert mpi.reduce(a.data_ptr(), b.data_ptr(), 0, mpi.MPI_FLOAT, mpi.MPI_SUM, 0, comms[0], REF) == 0
    finally:
        for c in comms:
            mpi.comm_free(c)


def _ok(mpi, rc):
    assert rc == 0, mpi.error_string(rc)


def test_collective_validation(mpi, cuda):
    torch = cuda
    comms = mpi.comm_create_loopback(1)
    a = torch.zeros(16, device="cuda")
    b = torch.zeros(16, device="cuda")
    try:
        ec = mpi.error_class
        assert ec(mpi.allreduce(a.data_ptr(), b.data_ptr(), 16, mpi.MPI_FLOAT, mpi.MPI_LAND, comms[0])) == mpi.MPI_ERR_OP
        assert ec(mpi.allreduce(a.data_ptr(), a.data_ptr(), 16, mpi.MPI_FLOAT, mpi.MPI_SUM, comms[0])) == \
            mpi.MPI_ERR_BUFFER
        assert ec(mpi.allreduce(a.data_ptr(), b.data_ptr(), -1, mpi.MPI_FLOAT, mpi.MPI_SUM, comms[0])) == \
            mpi.MPI_ERR_COUNT
        assert ec(mpi.allreduce(a.data_ptr(), b.data_ptr(), 16, mpi.MPI_FLOAT, mpi.MPI_REPLACE, comms[0])) == \
            mpi.MPI_ERR_OP
        assert ec(mpi.reduce_scatter_block(a.data_ptr(), b.data_ptr(), 16, mpi.MPI_BYTE, mpi.MPI_SUM,
                                           comms[0])) == mpi.MPI_ERR_OP
        assert mpi.allreduce(a.data_ptr(), b.data_ptr(), 0, mpi.MPI_FLOAT, mpi.MPI_SUM, comms[0]) == 0
    finally:
        mpi.comm_free(comms[0])


@pytest.mark.parametrize("p", [3, 8])
def test_large_blocks_skewed_staging(mpi, orc, cuda, p):
    """Messages whose staging slots are >= 1 MiB, where the slots sit at a
    skewed (non-power-of-two) stride (coll_hip.c stage_stride): Allreduce and
    Reduce (root 0 and p-1) through the reduce-scatter phase, Reduce_scatter_block
    pairwise, Scan and Exscan -- fp32 SUM, bit-exact vs the step-by-step schedules."""
    from oracle import schedules as S
    torch = cuda
    esz, dt, o = 4, mpi.MPI_FLOAT, mpi.MPI_SUM
    REF = mpi.MPIX_HIP_ALG_REFERENCE_ORDER
    comms = mpi.comm_create_loopback(p)
    try:
        count = (1 << 21) + 5                      # 8 MiB per rank: blocks >= 1 MiB at p = 8
        rng = np.random.default_rng(p)
        xs = [rng.uniform(-1, 1, count).astype(np.float32).view(np.uint8) for _ in range(p)]
        send = [torch.from_numpy(x.copy()).cuda() for x in xs]
        recv = [torch.zeros_like(s) for s in send]
        torch.cuda.synchronize()
        run_ranks(lambda r: _ok(mpi, mpi.allreduce(send[r].data_ptr(), recv[r].data_ptr(), count, dt, o,
                                                   comms[r], REF)), p)
        torch.cuda.synchronize()
        want = S.allreduce_smp_auto(xs, count, esz, dt, o)
        for r in range(p):
            assert np.array_equal(recv[r].cpu().numpy(), want), f"allreduce rank {r}"
        for root in (0, p - 1):
            rbuf = torch.zeros_like(send[root])
            torch.cuda.synchronize()
            run_ranks(lambda r: _ok(mpi, mpi.reduce(send[r].data_ptr(), rbuf.data_ptr() if r == root else 0,
                                                    count, dt, o, root, comms[r], REF)), p)
            torch.cuda.synchronize()
            assert np.array_equal(rbuf.cpu().numpy(), S.reduce_auto(xs, count, esz, dt, o, root)), f"reduce {root}"
        rcount = (1 << 18) + 1                     # 1 MiB + 4 B per block: pairwise, skewed slots
        ys = [rng.uniform(-1, 1, rcount * p).astype(np.float32).view(np.uint8) for _ in range(p)]
        ysend = [torch.from_numpy(y.copy()).cuda() for y in ys]
        yrecv = [torch.zeros(rcount * esz, dtype=torch.uint8, device="cuda") for _ in range(p)]
        torch.cuda.synchronize()
        run_ranks(lambda r: _ok(mpi, mpi.reduce_scatter_block(ysend[r].data_ptr(), yrecv[r].data_ptr(), rcount, dt,
                                                              o, comms[r], REF)), p)
        torch.cuda.synchronize()
        want = S.reduce_scatter_block_auto(ys, rcount, esz, dt, o)
        for r in range(p):
            assert np.array_equal(yrecv[r].cpu().numpy(), want[r]), f"reduce_scatter_block rank {r}"
        scount = (1 << 18) + 3
        zs = [rng.uniform(-1, 1, scount).astype(np.float32).view(np.uint8) for _ in range(p)]
        zsend = [torch.from_numpy(z.copy()).cuda() for z in zs]
        for fn, sim in ((mpi.scan, S.scan_recursive_doubling), (mpi.exscan, S.exscan_recursive_doubling)):
            zrecv = [torch.zeros_like(z) for z in zsend]
            torch.cuda.synchronize()
            run_ranks(lambda r: _ok(mpi, fn(zsend[r].data_ptr(), zrecv[r].data_ptr(), scount, dt, o, comms[r],
                                            REF)), p)
            torch.cuda.synchronize()
            want = sim(zs, scount, esz, dt, o)
            for r in range(1 if fn is mpi.exscan else 0, p):
                assert np.array_equal(zrecv[r].cpu().numpy(), want[r]), f"{fn.__name__} rank {r}"
    finally:
        for c in comms:
            mpi.comm_free(c)


PIPE = [("MPI_FLOAT", "MPI_SUM"), ("MPIX_C_FLOAT16", "MPI_SUM"), ("MPI_DOUBLE", "MPI_MAX"), ("MPI_INT", "MPI_BXOR")]


@pytest.mark.parametrize("t,op", PIPE, ids=[f"{t}-{o}" for t, o in PIPE])
@pytest.mark.parametrize("p", [2, 3, 5, 8])
@pytest.mark.parametrize("kind", ["allreduce", "reduce_scatter_block", "reduce"])
def test_pipelined_reference_order(mpi, orc, cuda, t, op, p, kind, monkeypatch):
    """The reference-order schedules with the exchange cut into chunks and each
    chunk's fold overlapping the next chunk's transfer (coll_hip.c
    exchange_fold_pipelined; MPIR_CVAR_DEVICE_COLL_PIPELINE_KB = 64 here so
    that test-sized blocks span many chunks, ragged last chunks included):
    bit-exact against the oracle's step-by-step schedules, every rank."""
    from oracle import schedules as S
    monkeypatch.setenv("MPIR_CVAR_DEVICE_COLL_PIPELINE_KB", "64")
    torch = cuda
    esz = T.elem_size(t)
    comms = mpi.comm_create_loopback(p)
    try:
        count = (1 << 19) + 7 if kind != "reduce_scatter_block" else (1 << 17) + 5
        rng = np.random.default_rng(17 * p + len(kind))
        n = count * p if kind == "reduce_scatter_block" else count
        xs = [T.to_bytes(T.gen(t, n, rng, op)) for _ in range(p)]
        root = p - 1
        if kind == "allreduce":
            want = [S.allreduce_smp_auto(xs, count, esz, mpi.DATATYPES[t], mpi.OPS[op])] * p
        elif kind == "reduce_scatter_block":
            want = S.reduce_scatter_block_auto(xs, count, esz, mpi.DATATYPES[t], mpi.OPS[op])
        else:
            want = {root: S.reduce_auto(xs, count, esz, mpi.DATATYPES[t], mpi.OPS[op], root)}
        send = [torch.from_numpy(x.copy()).cuda() for x in xs]
        recv = [torch.zeros(count * esz, dtype=torch.uint8, device="cuda") for _ in range(p)]
        torch.cuda.synchronize()

        def rank(r):
            if kind == "allreduce":
                rc = mpi.allreduce(send[r].data_ptr(), recv[r].data_ptr(), count, mpi.DATATYPES[t], mpi.OPS[op],
                                   comms[r], mpi.MPIX_HIP_ALG_REFERENCE_ORDER)
            elif kind == "reduce_scatter_block":
                rc = mpi.reduce_scatter_block(send[r].data_ptr(), recv[r].data_ptr(), count, mpi.DATATYPES[t],
                                              mpi.OPS[op], comms[r], mpi.MPIX_HIP_ALG_REFERENCE_ORDER)
            else:
                rc = mpi.reduce(send[r].data_ptr(), recv[r].data_ptr() if r == root else 0, count,
                                mpi.DATATYPES[t], mpi.OPS[op], root, comms[r], mpi.MPIX_HIP_ALG_REFERENCE_ORDER)
            assert rc == 0, mpi.error_string(rc)

        run_ranks(rank, p)
        torch.cuda.synchronize()
        for r in range(p):
            if kind == "reduce" and r != root:
                continue
            got = recv[r].cpu().numpy()
            assert same(got, want[r], t), f"rank {r}: {np.count_nonzero(got != want[r])} bytes differ"
    finally:
        for c in comms:
            mpi.comm_free(c)

"""Fused schedule combines (MPIX_Reduce_local_multi) vs the reference schedules, on one GPU.

The reference's Allreduce on one node (allreduce_intra_smp.c -> MPIR_Reduce via
reduce_intra_reduce_scatter_gather.c) and its Reduce_scatter_block
(reduce_scatter_block_intra_pairwise.c) call MPIR_Reduce_local log2(p) resp.
p-1 times per element.  The MI355X design gathers every rank's copy of a block
in HBM (all-to-all) and folds them in ONE pass with the schedule's exact
association and operand order.  Here p ranks' buffers live on one GPU; the
expected bytes come from oracle/schedules.py, which runs the reference
schedules step by step through the C oracle.  Bit-exact (complex NaN payloads
excepted, see test_parity_gpu.same).
"""
import numpy as np
import pytest

import _types as T
from test_parity_gpu import same

pytestmark = pytest.mark.gpu


def _pof2(p):
    q = 1
    while q * 2 <= p:
        q *= 2
    return q


def _cnts_disps(count, pof2):
    cnts = [count // pof2 + (1 if i < count % pof2 else 0) for i in range(pof2)]
    disps = [sum(cnts[:i]) for i in range(pof2)]
    return cnts, disps


def _bitrev(n, bits):
    return int(format(n, f"0{bits}b")[::-1], 2) if bits else 0


def fused_allreduce(mpi, torch, xs_dev, count, esz, dt, op):
    """The MI355X reference-order Allreduce on p virtual ranks (one GPU):
    pre-fold (p not a power of two), then per block b the owner newrank
    k = bitrev(b) folds y_j = x_{k ^ j}[b] with MPIX_ORDER_TREE."""
    p = len(xs_dev)
    pof2 = _pof2(p)
    rem = p - pof2
    leaves = []
    for r in range(p):                     # reduce_intra_reduce_scatter_gather.c:138-170
        if r < 2 * rem:
            if r % 2 == 0:
                acc = xs_dev[r].clone()
                torch.cuda.synchronize()
                assert mpi.reduce_local(xs_dev[r + 1].data_ptr(), acc.data_ptr(), count, dt, op) == 0
                leaves.append(acc)
        else:
            leaves.append(xs_dev[r])
    assert len(leaves) == pof2
    cnts, disps = _cnts_disps(count, pof2)
    out = torch.empty(count * esz, dtype=torch.uint8, device="cuda")
    bits = pof2.bit_length() - 1
    for b in range(pof2):
        k = _bitrev(b, bits)
        ys = [leaves[k ^ j].data_ptr() + disps[b] * esz for j in range(pof2)]
        rc = mpi.reduce_local_multi(ys, out.data_ptr() + disps[b] * esz, cnts[b], dt, op, mpi.MPIX_ORDER_TREE)
        assert rc == 0, mpi.error_string(rc)
    torch.cuda.synchronize()
    return out.cpu().numpy()


CASES = [("MPI_FLOAT", "MPI_SUM"), ("MPI_DOUBLE", "MPI_SUM"), ("MPIX_C_FLOAT16", "MPI_SUM"),
         ("MPI_INT", "MPI_SUM"), ("MPI_INT64_T", "MPI_PROD"), ("MPI_FLOAT", "MPI_MAX"),
         ("MPI_DOUBLE", "MPI_MIN"), ("MPI_C_FLOAT_COMPLEX", "MPI_SUM"), ("MPI_FLOAT", "MPI_PROD"),
         ("MPI_UNSIGNED_CHAR", "MPI_BXOR"), ("MPI_INT", "MPI_LAND")]


@pytest.mark.parametrize("t,op", CASES, ids=[f"{t}-{o}" for t, o in CASES])
@pytest.mark.parametrize("p", [2, 3, 4, 6, 8])
def test_fused_allreduce_matches_reference_schedule(mpi, orc, cuda, t, op, p):
    from oracle import schedules as S
    torch = cuda
    esz = T.elem_size(t)
    for count, seed in ((1003, p), ((1 << 18) + 5, 7 * p)):
        rng = np.random.default_rng(seed)
        xs = [T.to_bytes(T.gen(t, count, rng, op)) for _ in range(p)]
        want = S.allreduce_smp(xs, count, esz, mpi.DATATYPES[t], mpi.OPS[op])
        xs_dev = [torch.from_numpy(x.copy()).cuda() for x in xs]
        got = fused_allreduce(mpi, torch, xs_dev, count, esz, mpi.DATATYPES[t], mpi.OPS[op])
        assert same(got, want, t), f"p={p} count={count}: {np.count_nonzero(got != want)} bytes differ"


@pytest.mark.parametrize("t,op", [("MPIX_C_FLOAT16", "MPI_SUM"), ("MPI_FLOAT", "MPI_SUM"), ("MPI_INT", "MPI_SUM"),
                                  ("MPI_DOUBLE", "MPI_MAX"), ("MPI_UNSIGNED", "MPI_BOR")])
@pytest.mark.parametrize("p", [2, 3, 5, 8, 11])
def test_fused_reduce_scatter_block_matches_pairwise(mpi, orc, cuda, t, op, p):
    """Config 5's schedule: rank r's block = ((x_r + x_{r-1}) + x_{r-2}) + ... (fp16: per-step rounding)."""
    from oracle import schedules as S
    torch = cuda
    esz = T.elem_size(t)
    recvcount = 4099
    rng = np.random.default_rng(p)
    xs = [T.to_bytes(T.gen(t, recvcount * p, rng, op)) for _ in range(p)]
    want = S.reduce_scatter_block_pairwise(xs, recvcount, esz, mpi.DATATYPES[t], mpi.OPS[op])
    xs_dev = [torch.from_numpy(x.copy()).cuda() for x in xs]
    nb = recvcount * esz
    for r in range(p):
        out = torch.empty(nb, dtype=torch.uint8, device="cuda")
        ys = [xs_dev[(r - i) % p].data_ptr() + r * nb for i in range(p)]
        rc = mpi.reduce_local_multi(ys, out.data_ptr(), recvcount, mpi.DATATYPES[t], mpi.OPS[op],
                                    mpi.MPIX_ORDER_CHAIN)
        assert rc == 0, mpi.error_string(rc)
        got = out.cpu().numpy()
        assert same(got, want[r], t), f"rank {r}"


def test_multi_validation(mpi, cuda):
    torch = cuda
    a = torch.zeros(64, device="cuda")
    b = torch.zeros(64, device="cuda")
    ptrs = [a.data_ptr(), b.data_ptr(), a.data_ptr()]
    # tree needs a power of two
    ec = mpi.error_class
    assert ec(mpi.reduce_local_multi(ptrs, b.data_ptr(), 64, mpi.MPI_FLOAT, mpi.MPI_SUM,
                                     mpi.MPIX_ORDER_TREE)) == mpi.MPI_ERR_ARG
    # op/type check like MPI_Reduce_local
    assert ec(mpi.reduce_local_multi(ptrs[:2], b.data_ptr(), 64, mpi.MPI_FLOAT, mpi.MPI_BAND,
                                     mpi.MPIX_ORDER_CHAIN)) == mpi.MPI_ERR_OP
    h = np.zeros(64, np.float32)
    assert ec(mpi.reduce_local_multi([h.ctypes.data, a.data_ptr()], b.data_ptr(), 64, mpi.MPI_FLOAT, mpi.MPI_SUM,
                                     mpi.MPIX_ORDER_CHAIN)) == mpi.MPI_ERR_BUFFER


def test_multi_overlap_refused(mpi, cuda):
    """outbuf may be inbufs[0] exactly; any other overlap is MPI_ERR_BUFFER,
    whatever MPIR_CVAR_COLL_ALIAS_CHECK says (the CHAIN path for n > 8 writes
    outbuf between passes)."""
    torch = cuda
    ec = mpi.error_class
    bufs = [torch.full((4096,), float(j + 1), device="cuda") for j in range(12)]
    p = [b.data_ptr() for b in bufs]
    F, S, C, T = mpi.MPI_FLOAT, mpi.MPI_SUM, mpi.MPIX_ORDER_CHAIN, mpi.MPIX_ORDER_TREE
    # exactly a later operand, on the multi-pass CHAIN shape and on a fused TREE
    assert ec(mpi.reduce_local_multi(p, p[9], 4096, F, S, C)) == mpi.MPI_ERR_BUFFER
    assert ec(mpi.reduce_local_multi(p[:4], p[2], 4096, F, S, T)) == mpi.MPI_ERR_BUFFER
    # partial overlaps: with operand 0, and a later operand's tail
    assert ec(mpi.reduce_local_multi(p[:4], p[0] + 16, 4096, F, S, T)) == mpi.MPI_ERR_BUFFER
    assert ec(mpi.reduce_local_multi(p[:3], p[2] - 64, 4096, F, S, C)) == mpi.MPI_ERR_BUFFER
    assert "overlaps outbuf" in mpi.error_string(mpi.reduce_local_multi(p[:3], p[1] + 4, 4096, F, S, C))
    # adjacent (touching, not overlapping) and exactly operand 0 are fine
    big = torch.ones(2 * 4096, device="cuda")
    assert mpi.reduce_local_multi([big.data_ptr(), p[1]], big.data_ptr() + 4 * 4096, 4096, F, S, C) == 0
    assert mpi.reduce_local_multi(p, p[0], 4096, F, S, C) == 0
    torch.cuda.synchronize()
    assert torch.equal(bufs[0], torch.full((4096,), float(sum(range(1, 13))), device="cuda"))
    assert torch.equal(big[4096:], torch.full((4096,), 3.0, device="cuda"))


ANY = [("MPI_DOUBLE_INT", "MPI_MINLOC"), ("MPI_2INT", "MPI_MAXLOC"), ("MPI_INT", "MPI_LAND"),
       ("MPI_UNSIGNED_SHORT", "MPI_BOR"), ("MPI_C_DOUBLE_COMPLEX", "MPI_PROD"), ("MPI_LONG_DOUBLE", "MPI_SUM"),
       ("MPI_LONG_DOUBLE_INT", "MPI_MAXLOC"), ("MPI_FLOAT", "MPI_SUM"), ("MPIX_C_FLOAT16", "MPI_MAX")]


@pytest.mark.parametrize("t,op", ANY, ids=[f"{t}-{o}" for t, o in ANY])
@pytest.mark.parametrize("n,order", [(2, "TREE"), (4, "TREE"), (16, "TREE"), (64, "TREE"), (3, "CHAIN"),
                                     (13, "CHAIN")])
def test_one_pass_combine_matches_stepwise_fold(mpi, orc, cuda, t, op, n, order):
    """MPIR_Hip_combine's general one-pass path (k_combine_any: any op/type, any n,
    no device temporaries) and the fused kernels agree bit for bit with the
    same fold done one MPIR_Reduce_local step at a time by the oracle.  The
    output aliases operand 0 on the CHAIN cases."""
    torch = cuda
    esz = T.elem_size(t)
    count = 1000 + n
    rng = np.random.default_rng(n)
    xs = [T.to_bytes(T.gen(t, count, rng, op)) for _ in range(n)]
    dt, o = mpi.DATATYPES[t], mpi.OPS[op]
    acc = [x.copy() for x in xs]
    if order == "TREE":
        step = 1
        while step < n:
            for j in range(0, n, 2 * step):
                assert orc.reduce_local(acc[j + step], acc[j], count, dt, o, check=False) == 0
            step *= 2
    else:
        for j in range(1, n):
            assert orc.reduce_local(acc[j], acc[0], count, dt, o, check=False) == 0
    want = acc[0]
    dev = [torch.from_numpy(x.copy()).cuda() for x in xs]
    out = dev[0] if order == "CHAIN" else torch.zeros(count * esz, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    rc = mpi.reduce_local_multi([d.data_ptr() for d in dev], out.data_ptr(), count, dt, o,
                                mpi.MPIX_ORDER_TREE if order == "TREE" else mpi.MPIX_ORDER_CHAIN)
    assert rc == 0, mpi.error_string(rc)
    torch.cuda.synchronize()
    assert same(out.cpu().numpy(), want, t)


def test_concurrent_threads_minloc_tree16_regression(mpi, orc, cuda):
    """Regression for the corruption removed in e7b5d60: several host threads
    folding MPI_MINLOC (no fused kernel: the general path) at once, each on its
    own library stream.  The removed path took its temporaries with
    hipMallocAsync / hipFreeAsync, and the default memory pool handed a block
    freed on one stream to another stream while the first stream's kernels
    still read it (tools/mempool_race.hip: 3 of 1200 results corrupted at 4
    threads, 14 of 2400 at 8; profiles/archive/r02/mempool_race.log).  The product takes
    no stream-ordered allocations (tests/test_no_stream_ordered_alloc_cpu.py);
    this checks the concurrent folds stay bit-exact."""
    import threading
    torch = cuda
    t, op, n, count, iters, nthreads = "MPI_DOUBLE_INT", "MPI_MINLOC", 16, 1 << 16, 12, 4
    dt, o = mpi.DATATYPES[t], mpi.OPS[op]
    esz = T.elem_size(t)
    cases = []
    for k in range(nthreads):
        rng = np.random.default_rng(100 + k)
        xs = [T.to_bytes(T.gen(t, count, rng, op)) for _ in range(n)]
        acc = [x.copy() for x in xs]
        step = 1
        while step < n:
            for j in range(0, n, 2 * step):
                assert orc.reduce_local(acc[j + step], acc[j], count, dt, o, check=False) == 0
            step *= 2
        dev = [torch.from_numpy(x).cuda() for x in xs]
        outs = [torch.zeros(count * esz, dtype=torch.uint8, device="cuda") for _ in range(iters)]
        cases.append((acc[0], dev, outs))
    torch.cuda.synchronize()
    errors = []

    def run(k):
        want, dev, outs = cases[k]
        for out in outs:
            rc = mpi.reduce_local_multi([d.data_ptr() for d in dev], out.data_ptr(), count, dt, o,
                                        mpi.MPIX_ORDER_TREE)
            if rc:
                errors.append(mpi.error_string(rc))
    th = [threading.Thread(target=run, args=(k,)) for k in range(nthreads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    torch.cuda.synchronize()
    for k, (want, _, outs) in enumerate(cases):
        for i, out in enumerate(outs):
            assert same(out.cpu().numpy(), want, t), (k, i)


EVERY = [(op, t) for op in T.OPS for t in T.ALL_TYPES if T.compute_ok(op, t)]


@pytest.mark.parametrize("op,t", EVERY, ids=[f"{o}-{t}" for o, t in EVERY])
def test_every_pair_fused_matches_stepwise_fold(mpi, orc, cuda, op, t):
    """Every (op, type) the reference computes, through MPIX_Reduce_local_multi:
    TREE of 8 (one fused pass), CHAIN of 3, 5, 6, 7 and 8 (one pass each: the
    pairwise chain of every rank count up to 8) and CHAIN of 11 (a pass of 8,
    then one of 4 reading the first's output) against the same fold done one
    oracle MPIR_Reduce_local step at a time.  Operands with
    specials (NaN, +-0, inf, denormals, extremes); the second round starts
    every buffer one element past 256 B alignment so the fused kernel's head
    and tail elements run too."""
    torch = cuda
    esz = T.elem_size(t)
    dt, o = mpi.DATATYPES[t], mpi.OPS[op]
    for k, (n, order) in enumerate(((8, "TREE"), (8, "CHAIN"), (5, "CHAIN"), (3, "CHAIN"), (6, "CHAIN"),
                                    (7, "CHAIN"), (11, "CHAIN"))):
        for off in (0, esz):
            count = 3000 + 7 * n + k
            rng = np.random.default_rng(1000 * n + k + off)
            xs = [T.to_bytes(T.gen(t, count, rng, op)) for _ in range(n)]
            acc = [x.copy() for x in xs]
            if order == "TREE":
                step = 1
                while step < n:
                    for j in range(0, n, 2 * step):
                        assert orc.reduce_local(acc[j + step], acc[j], count, dt, o, check=False) == 0
                    step *= 2
            else:
                for j in range(1, n):
                    assert orc.reduce_local(acc[j], acc[0], count, dt, o, check=False) == 0
            nb = count * esz
            dev = []
            for x in xs:
                d = torch.zeros(nb + off + 64, dtype=torch.uint8, device="cuda")
                d[off:off + nb].copy_(torch.from_numpy(x))
                dev.append(d)
            out = torch.zeros(nb + off + 64, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            rc = mpi.reduce_local_multi([d.data_ptr() + off for d in dev], out.data_ptr() + off, count, dt, o,
                                        mpi.MPIX_ORDER_TREE if order == "TREE" else mpi.MPIX_ORDER_CHAIN)
            assert rc == 0, mpi.error_string(rc)
            torch.cuda.synchronize()
            got = out[off:off + nb].cpu().numpy()
            assert same(got, acc[0], t), f"n={n} {order} off={off}: {np.count_nonzero(got != acc[0])} bytes differ"
            assert not out[:off].any() and not out[off + nb:].any(), "wrote outside the output"


@pytest.mark.parametrize("t,order,block_mib", [("MPI_FLOAT", "TREE", 32), ("MPIX_C_FLOAT16", "CHAIN", 128)],
                         ids=["config4-tree8-fp32-32MiB", "config5-chain8-fp16-128MiB"])
def test_fused_full_size_blocks(mpi, orc, cuda, t, order, block_mib):
    """The fused combines at the block sizes of BASELINE configs 4-5 at N = 8
    (Allreduce 256 MiB -> 8 x 32 MiB blocks, TREE; Reduce_scatter_block 1 GiB
    fp16 -> 8 x 128 MiB blocks, CHAIN), bit-exact against the oracle's
    step-by-step fold over the whole block."""
    torch = cuda
    esz = T.elem_size(t)
    n = (block_mib << 20) // esz
    dt, o = mpi.DATATYPES[t], mpi.OPS["MPI_SUM"]
    g = torch.Generator(device="cuda").manual_seed(block_mib)
    if t == "MPI_FLOAT":
        dev = [torch.rand(n, device="cuda", generator=g) * 2 - 1 for _ in range(8)]
    else:
        dev = [(torch.rand(n, device="cuda", generator=g) * 8 - 4).half() for _ in range(8)]
    out = torch.empty_like(dev[0])
    torch.cuda.synchronize()
    rc = mpi.reduce_local_multi([d.data_ptr() for d in dev], out.data_ptr(), n, dt, o,
                                mpi.MPIX_ORDER_TREE if order == "TREE" else mpi.MPIX_ORDER_CHAIN)
    assert rc == 0, mpi.error_string(rc)
    torch.cuda.synchronize()
    acc = [d.cpu().numpy().view(np.uint8).copy() for d in dev]
    del dev
    if order == "TREE":
        step = 1
        while step < 8:
            for j in range(0, 8, 2 * step):
                assert orc.reduce_local(acc[j + step], acc[j], n, dt, o, check=False) == 0
            step *= 2
    else:
        for j in range(1, 8):
            assert orc.reduce_local(acc[j], acc[0], n, dt, o, check=False) == 0
    got = out.cpu().numpy().view(np.uint8)
    assert np.array_equal(got, acc[0]), f"{np.count_nonzero(got != acc[0])} bytes differ"


@pytest.mark.parametrize("t,order,nbytes", [("MPI_FLOAT", "TREE", (256 << 20) + 20), ("MPIX_C_FLOAT16", "CHAIN", (512 << 20) + 6)],
                         ids=["tree2-fp32-256MiB", "chain2-fp16-512MiB"])
def test_two_operand_fold_large_blocks(mpi, orc, cuda, t, order, nbytes):
    """Two-operand folds over blocks of 256 MiB and more run on the 1024 x 1
    shape (launch_combine_p; config 5's 2 x 512 MiB at 2 ranks), with the
    operands one element past 16 B alignment so the head and tail run too;
    bit-exact against the oracle's MPIR_Reduce_local step."""
    torch = cuda
    esz = T.elem_size(t)
    n = nbytes // esz
    dt, o = mpi.DATATYPES[t], mpi.OPS["MPI_SUM"]
    g = torch.Generator(device="cuda").manual_seed(n)
    if t == "MPI_FLOAT":
        dev = [torch.rand(n + 1, device="cuda", generator=g) * 2 - 1 for _ in range(2)]
    else:
        dev = [(torch.rand(n + 1, device="cuda", generator=g) * 8 - 4).half() for _ in range(2)]
    out = torch.zeros_like(dev[0])
    torch.cuda.synchronize()
    ptrs = [d.data_ptr() + esz for d in dev]
    rc = mpi.reduce_local_multi(ptrs, out.data_ptr() + esz, n, dt, o,
                                mpi.MPIX_ORDER_TREE if order == "TREE" else mpi.MPIX_ORDER_CHAIN)
    assert rc == 0, mpi.error_string(rc)
    torch.cuda.synchronize()
    acc = [d.cpu().numpy().view(np.uint8)[esz:].copy() for d in dev]
    del dev
    assert orc.reduce_local(acc[1], acc[0], n, dt, o, check=False) == 0
    got = out.cpu().numpy().view(np.uint8)
    assert not got[:esz].any(), "wrote before the output"
    assert np.array_equal(got[esz:], acc[0]), f"{np.count_nonzero(got[esz:] != acc[0])} bytes differ"

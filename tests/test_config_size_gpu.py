"""BASELINE configs 2, 4 and 5 at their full sizes on one GPU, against the
oracle (config 2 at full size was a property check, and
configs 4 / 5 ran only at size 1 without a second GPU).

  * config 2: MPI_Reduce_local fp32 SUM, 64 MiB per operand -- aligned (the
    lean tile kernel), ragged (tile + head / tail) and with inbuf 4 B off
    inoutbuf's alignment (the shift kernel), random operands with the edge
    values of tests/_types.py, bit-exact against oracle_reduce_local;
  * config 4's combine: the fused TREE8 fold MPIX_Reduce_local_multi runs for
    MPI_Allreduce fp32 256 MiB at 8 ranks (one 32 MiB block per owner,
    reduce_intra_reduce_scatter_gather.c:186-249: ((y0+y1)+(y2+y3))+
    ((y4+y5)+(y6+y7))), operands at the collective's skewed staging stride;
  * config 5's combine: the fused CHAIN8 fp16 fold of MPI_Reduce_scatter_block
    (1 GiB sendbuf, 8 ranks: 8 blocks of 128 MiB,
    reduce_scatter_block_intra_pairwise.c:97-134: (((x0+x1)+x2)+...)+x7).
The folds' expected bytes are the oracle's step-by-step MPIR_Reduce_local calls
in the schedule's association (oracle/op_oracle.c, gcc -O2).  What these do not
cover is the xGMI transport at 8 ranks (tests/test_coll_rccl_gpu.py, N > 1).
"""
import numpy as np
import pytest

import _types as T

pytestmark = pytest.mark.gpu

MIB = 1 << 20


def _dev(torch, arr, slack=0):
    t = torch.zeros(arr.nbytes + slack, dtype=torch.uint8, device="cuda")
    t[:arr.nbytes] = torch.from_numpy(arr.view(np.uint8))
    return t


@pytest.mark.parametrize("extra,off", [(0, 0), (3, 0), (1, 4)], ids=["aligned", "ragged", "inbuf+4B"])
def test_config2_64mib_vs_oracle(mpi, orc, cuda, extra, off):
    torch = cuda
    n = (64 * MIB) // 4 + extra
    rng = np.random.default_rng(64 + extra + off)
    a = T.gen("MPI_FLOAT", n, rng, "MPI_SUM").view(np.float32)
    b = T.gen("MPI_FLOAT", n, rng, "MPI_SUM").view(np.float32)
    want = a.copy()
    assert orc.reduce_local(b.copy(), want, n, mpi.MPI_FLOAT, mpi.MPI_SUM) == 0
    tio = _dev(torch, a)
    tin = torch.zeros(b.nbytes + 64, dtype=torch.uint8, device="cuda")
    tin[off:off + b.nbytes] = torch.from_numpy(b.view(np.uint8))
    torch.cuda.synchronize()
    assert mpi.reduce_local(tin.data_ptr() + off, tio.data_ptr(), n, mpi.MPI_FLOAT, mpi.MPI_SUM) == 0
    got = tio.cpu().numpy().view(np.uint32)
    assert np.array_equal(got, want.view(np.uint32)), int(np.count_nonzero(got != want.view(np.uint32)))


def _staged(torch, blocks):
    """The blocks at coll_hip.c's staging stride (slot rounded to 256 B, + 4352 B
    from 1 MiB up, + 6400 B for slots of 96-192 MiB), as the all-to-all leaves them."""
    nb = blocks[0].nbytes
    st = (nb + 255) & ~255
    stride = st + (6400 if 96 * MIB <= st < 192 * MIB else (4352 if st >= MIB else 0))
    buf = torch.zeros(stride * len(blocks), dtype=torch.uint8, device="cuda")
    for j, blk in enumerate(blocks):
        buf[j * stride:j * stride + nb] = torch.from_numpy(blk.view(np.uint8))
    return buf, [buf.data_ptr() + j * stride for j in range(len(blocks))]


def test_config4_tree8_fp32_32mib_blocks_vs_oracle(mpi, orc, cuda):
    torch = cuda
    n = (32 * MIB) // 4
    rng = np.random.default_rng(4)
    ys = [rng.uniform(-1, 1, n).astype(np.float32) for _ in range(8)]
    buf, ptrs = _staged(torch, ys)
    out = torch.empty(n * 4, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    rc = mpi.reduce_local_multi(ptrs, out.data_ptr(), n, mpi.MPI_FLOAT, mpi.MPI_SUM, mpi.MPIX_ORDER_TREE)
    assert rc == 0, mpi.error_string(rc)
    torch.cuda.synchronize()
    # ((y0+y1)+(y2+y3))+((y4+y5)+(y6+y7)), each + an MPIR_Reduce_local(in, inout)
    # with inout the left operand
    lvl = [y.copy() for y in ys]
    while len(lvl) > 1:
        nxt = []
        for i in range(0, len(lvl), 2):
            acc = lvl[i].copy()
            assert orc.reduce_local(lvl[i + 1], acc, n, mpi.MPI_FLOAT, mpi.MPI_SUM) == 0
            nxt.append(acc)
        lvl = nxt
    got = out.cpu().numpy().view(np.uint32)
    assert np.array_equal(got, lvl[0].view(np.uint32)), int(np.count_nonzero(got != lvl[0].view(np.uint32)))


def test_config5_chain8_fp16_128mib_blocks_vs_oracle(mpi, orc, cuda):
    torch = cuda
    n = (128 * MIB) // 2
    rng = np.random.default_rng(5)
    xs = [rng.uniform(-1, 1, n).astype(np.float16) for _ in range(8)]
    buf, ptrs = _staged(torch, xs)
    out = torch.empty(n * 2, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    rc = mpi.reduce_local_multi(ptrs, out.data_ptr(), n, mpi.MPIX_C_FLOAT16, mpi.MPI_SUM, mpi.MPIX_ORDER_CHAIN)
    assert rc == 0, mpi.error_string(rc)
    torch.cuda.synchronize()
    acc = xs[0].copy()
    for j in range(1, 8):     # rounding to fp16 at every step, as the reference's loop does
        assert orc.reduce_local(xs[j], acc, n, mpi.MPIX_C_FLOAT16, mpi.MPI_SUM) == 0
    got = out.cpu().numpy().view(np.uint16)
    assert np.array_equal(got, acc.view(np.uint16)), int(np.count_nonzero(got != acc.view(np.uint16)))


# ---- configs 4 and 5 end to end at 8 ranks and full size, on one GPU: the
# ---- loopback communicator (8 virtual ranks, one host thread each, transfers
# ---- are device copies) runs the complete reference-order collective -- the
# ---- all-to-all of blocks into the skewed staging slots, the fused combine,
# ---- the allgather -- on the BASELINE workload.  Only the transport differs
# ---- from the 8-GPU run (grouped ncclSend / ncclRecv over xGMI,
# ---- tests/test_coll_rccl_gpu.py).

def test_config4_allreduce_fp32_256mib_8_ranks_loopback_vs_oracle(mpi, orc, cuda):
    """MPI_Allreduce fp32 SUM, 256 MiB per rank, 8 ranks: MPICH's choice on one
    node (allreduce_intra_smp.c -> reduce_intra_reduce_scatter_gather.c:186-249,
    then the bcast), oracle/schedules.py allreduce_smp_auto step by step."""
    from oracle import schedules as S
    from test_coll_loopback_gpu import run_ranks
    torch = cuda
    p, count = 8, (256 * MIB) // 4
    xs = [np.random.default_rng(400 + r).uniform(-1, 1, count).astype(np.float32) for r in range(p)]
    want = S.allreduce_smp_auto(xs, count, 4, mpi.MPI_FLOAT, mpi.MPI_SUM).view(np.uint32)
    comms = mpi.comm_create_loopback(p)
    try:
        send = [torch.from_numpy(x).cuda() for x in xs]
        del xs
        recv = [torch.empty_like(s) for s in send]
        torch.cuda.synchronize()

        def rank(r):
            rc = mpi.allreduce(send[r].data_ptr(), recv[r].data_ptr(), count, mpi.MPI_FLOAT, mpi.MPI_SUM, comms[r],
                               mpi.MPIX_HIP_ALG_REFERENCE_ORDER)
            assert rc == 0, mpi.error_string(rc)

        run_ranks(rank, p)
        torch.cuda.synchronize()
        for r in range(p):
            got = recv[r].cpu().numpy().view(np.uint32)
            assert np.array_equal(got, want), f"rank {r}: {int(np.count_nonzero(got != want))} elements differ"
    finally:
        for c in comms:
            mpi.comm_free(c)


def test_config5_reduce_scatter_block_fp16_1gib_8_ranks_loopback_vs_oracle(mpi, orc, cuda):
    """MPI_Reduce_scatter_block fp16 SUM, 1 GiB sendbuf per rank (recvcount
    2^29 / 8), 8 ranks: pairwise (reduce_scatter_block.c:136-148,
    reduce_scatter_block_intra_pairwise.c:97-134), oracle/schedules.py
    reduce_scatter_block_auto's chain per rank, rounded to fp16 at every step.
    Operands: random fp16 bit patterns of magnitude < 2 (subnormals and zeros
    included), so the 8-term sums stay finite."""
    from oracle import schedules as S
    from test_coll_loopback_gpu import run_ranks
    torch = cuda
    p = 8
    total = (1024 * MIB) // 2
    rcount = total // p
    xs = [np.random.default_rng(500 + r).integers(0, 1 << 16, total, dtype=np.uint16) & np.uint16(0xBFFF)
          for r in range(p)]
    assert p * rcount * 2 >= S.RSB_COMMUTATIVE_LONG_MSG_SIZE      # the pairwise algorithm
    want = S.reduce_scatter_block_pairwise(xs, rcount, 2, mpi.MPIX_C_FLOAT16, mpi.MPI_SUM, workers=p)
    comms = mpi.comm_create_loopback(p)
    try:
        send = [torch.from_numpy(x.view(np.int16)).cuda() for x in xs]
        del xs
        recv = [torch.empty(rcount, dtype=torch.int16, device="cuda") for _ in range(p)]
        torch.cuda.synchronize()

        def rank(r):
            rc = mpi.reduce_scatter_block(send[r].data_ptr(), recv[r].data_ptr(), rcount, mpi.MPIX_C_FLOAT16,
                                          mpi.MPI_SUM, comms[r], mpi.MPIX_HIP_ALG_REFERENCE_ORDER)
            assert rc == 0, mpi.error_string(rc)

        run_ranks(rank, p)
        torch.cuda.synchronize()
        for r in range(p):
            got = recv[r].cpu().numpy().view(np.uint16)
            w = want[r].view(np.uint16)
            assert np.array_equal(got, w), f"rank {r}: {int(np.count_nonzero(got != w))} elements differ"
    finally:
        for c in comms:
            mpi.comm_free(c)

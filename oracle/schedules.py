"""CPU simulation of MPICH's reduction schedules -- TEST INFRASTRUCTURE ONLY.

Step-by-step restatements of the reference's blocking collective algorithms
for p ranks held in one process: every MPIC_Sendrecv becomes a copy between
the ranks' numpy buffers (all sends of a step read the state before that
step's reductions), every MPIR_Reduce_local becomes a call into the C oracle
(oracle/op_oracle.c, `oracle_reduce_local_nocheck`).  They define the
summation order the GPU's fused schedule combines must reproduce bit for bit.

  reduce_scatter_gather   src/mpi/coll/reduce/reduce_intra_reduce_scatter_gather.c:130-250
                          (reduce-scatter phase; the gather to the root and the
                          SMP allreduce's MPIR_Bcast only move data)
  allreduce_smp           src/mpi/coll/allreduce/allreduce_intra_smp.c: MPIR_Reduce to
                          node root 0 (reduce.c:170-205 picks reduce_scatter_gather for
                          nbytes > 2048, builtin op, count >= pof2) + MPIR_Bcast
  allreduce_rsag          src/mpi/coll/allreduce/allreduce_intra_reduce_scatter_allgather.c:72-290
  reduce_scatter_block_pairwise
                          src/mpi/coll/reduce_scatter_block/reduce_scatter_block_intra_pairwise.c:75-134
"""
from __future__ import annotations

import numpy as np

from . import reduce_local


def _pof2(p: int) -> int:
    q = 1
    while q * 2 <= p:
        q *= 2
    return q


def _cnts_disps(count: int, pof2: int):
    cnts = [count // pof2 + (1 if i < count % pof2 else 0) for i in range(pof2)]
    disps = [0] * pof2
    for i in range(1, pof2):
        disps[i] = disps[i - 1] + cnts[i - 1]
    return cnts, disps


def _red(tmp: np.ndarray, acc: np.ndarray, n: int, dt: int, op: int):
    """MPIR_Reduce_local(tmp, acc, n): acc = op(acc, tmp) elementwise, in place."""
    if n:
        rc = reduce_local(tmp, acc, n, dt, op, check=False)
        assert rc == 0, rc


def reduce_scatter_gather_phase(bufs: list[np.ndarray], count: int, esz: int, dt: int, op: int,
                                even_keeps: bool = True):
    """The pre-fold + recursive-halving reduce-scatter shared by the reduce and the
    Rabenseifner allreduce.  `bufs[r]` are byte arrays (count*esz), updated in place.
    even_keeps=True: reduce_scatter_gather (odd ranks < 2*rem send to rank-1,
    reduce.c:138-170); False: Rabenseifner (even ranks send to rank+1, :85-125).
    Returns (newrank per rank, cnts, disps, pof2, final block index per rank)."""
    p = len(bufs)
    pof2 = _pof2(p)
    rem = p - pof2
    newrank = [0] * p
    # non-power-of-two pre-fold
    for r in range(p):
        if r < 2 * rem:
            keeper = (r % 2 == 0) if even_keeps else (r % 2 == 1)
            if keeper:
                src = r + 1 if even_keeps else r - 1
                tmp = bufs[src].copy()
                _red(tmp, bufs[r], count, dt, op)
                newrank[r] = r // 2
            else:
                newrank[r] = -1
        else:
            newrank[r] = r - rem
    cnts, disps = _cnts_disps(count, pof2)
    real = {}
    for r in range(p):
        if newrank[r] >= 0:
            real[newrank[r]] = r
    st = {r: {"send_idx": 0, "recv_idx": 0, "last_idx": pof2} for r in real.values()}
    mask = 1
    while mask < pof2:
        sends = {}
        plans = {}
        for nr, r in real.items():
            s = st[r]
            nd = nr ^ mask
            if nr < nd:
                s["send_idx"] = s["recv_idx"] + pof2 // (mask * 2)
                send_lo, send_hi = s["send_idx"], s["last_idx"]
                recv_lo, recv_hi = s["recv_idx"], s["send_idx"]
            else:
                s["recv_idx"] = s["send_idx"] + pof2 // (mask * 2)
                send_lo, send_hi = s["send_idx"], s["recv_idx"]
                recv_lo, recv_hi = s["recv_idx"], s["last_idx"]
            lo = disps[send_lo] * esz if send_hi > send_lo else 0
            sends[r] = (real[nd], bufs[r][lo:lo + sum(cnts[send_lo:send_hi]) * esz].copy())
            plans[r] = (recv_lo, recv_hi)
        for nr, r in real.items():
            peer = real[nr ^ mask]
            recv_lo, recv_hi = plans[r]
            if recv_hi > recv_lo:
                data = sends[peer][1]
                lo = disps[recv_lo] * esz
                n = sum(cnts[recv_lo:recv_hi])
                _red(data, bufs[r][lo:lo + n * esz], n, dt, op)
            s = st[r]
            s["send_idx"] = s["recv_idx"]
        mask <<= 1
        if mask < pof2:
            for r in st:
                s = st[r]
                s["last_idx"] = s["recv_idx"] + pof2 // mask
    final_block = {r: st[r]["send_idx"] for r in st}
    return newrank, cnts, disps, pof2, final_block


def bitrev(n: int, bits: int) -> int:
    return int(format(n, f"0{bits}b")[::-1], 2) if bits else 0


def _gather(bufs, newrank, cnts, disps, pof2, final_block, count, esz):
    """The data movement after the reduce-scatter (gather to root + bcast, or the
    allgather): every element comes from the rank that owns its block."""
    out = np.empty(count * esz, dtype=np.uint8)
    bits = pof2.bit_length() - 1
    for r, nr in enumerate(newrank):
        if nr < 0:
            continue
        b = final_block[r]
        assert b == bitrev(nr, bits)          # newrank n ends owning block bitrev(n)
        lo = disps[b] * esz
        out[lo:lo + cnts[b] * esz] = bufs[r][lo:lo + cnts[b] * esz]
    return out


def allreduce_smp(rank_bufs: list[np.ndarray], count: int, esz: int, dt: int, op: int) -> np.ndarray:
    """MPI_Allreduce result on one node (every rank ends with the same bytes)."""
    bufs = [b.view(np.uint8).reshape(-1).copy() for b in rank_bufs]
    res = reduce_scatter_gather_phase(bufs, count, esz, dt, op, even_keeps=True)
    return _gather(bufs, *res, count, esz)


def allreduce_rsag(rank_bufs: list[np.ndarray], count: int, esz: int, dt: int, op: int) -> np.ndarray:
    """Rabenseifner (the flat-communicator algorithm); same block ownership."""
    bufs = [b.view(np.uint8).reshape(-1).copy() for b in rank_bufs]
    res = reduce_scatter_gather_phase(bufs, count, esz, dt, op, even_keeps=False)
    return _gather(bufs, *res, count, esz)


def reduce_scatter_block_pairwise(rank_sendbufs: list[np.ndarray], recvcount: int, esz: int, dt: int,
                                  op: int) -> list[np.ndarray]:
    """Each rank's recvbuf after MPI_Reduce_scatter_block (pairwise exchanges)."""
    p = len(rank_sendbufs)
    send = [b.view(np.uint8).reshape(-1) for b in rank_sendbufs]
    nb = recvcount * esz
    recv = [send[r][r * nb:(r + 1) * nb].copy() for r in range(p)]
    for i in range(1, p):
        for r in range(p):
            src = (r - i + p) % p
            tmp = send[src][r * nb:(r + 1) * nb].copy()
            _red(tmp, recv[r], recvcount, dt, op)
    return recv

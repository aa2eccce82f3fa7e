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
  reduce_binomial         src/mpi/coll/reduce/reduce_intra_binomial.c:93-140 (commutative op:
                          lroot = root)
  allreduce_smp_auto      allreduce_intra_smp.c with MPIR_Reduce_intra_auto's choice
                          (reduce.c:214-225): reduce_scatter_gather when nbytes > 2048
                          (MPIR_CVAR_REDUCE_SHORT_MSG_SIZE), builtin op and count >= pof2,
                          else the binomial tree; then MPIR_Bcast
  reduce_scatter_block_recursive_halving
                          src/mpi/coll/reduce_scatter_block/
                          reduce_scatter_block_intra_recursive_halving.c:143-300
  reduce_scatter_block_auto
                          MPIR_Reduce_scatter_block_intra_auto (reduce_scatter_block.c:136-148):
                          builtin ops are commutative, so recursive halving below 524288
                          total bytes (MPIR_CVAR_REDUCE_SCATTER_COMMUTATIVE_LONG_MSG_SIZE),
                          pairwise from there on
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
                                  op: int, workers: int = 1) -> list[np.ndarray]:
    """Each rank's recvbuf after MPI_Reduce_scatter_block (pairwise exchanges).
    Rank r's block is its own chain ((x_r + x_{r-1}) + x_{r-2}) + ..., independent
    of the other ranks', so `workers` > 1 runs the ranks' chains on that many
    threads (the oracle's C calls release the GIL); each chain keeps its order."""
    p = len(rank_sendbufs)
    send = [b.view(np.uint8).reshape(-1) for b in rank_sendbufs]
    nb = recvcount * esz
    recv = [send[r][r * nb:(r + 1) * nb].copy() for r in range(p)]

    def chain(r):
        for i in range(1, p):
            src = (r - i + p) % p
            _red(send[src][r * nb:(r + 1) * nb].copy(), recv[r], recvcount, dt, op)
    if workers > 1:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(workers) as ex:
            list(ex.map(chain, range(p)))
    else:
        for r in range(p):
            chain(r)
    return recv


REDUCE_SHORT_MSG_SIZE = 2048            # reduce.c:14-17 (MPIR_CVAR_REDUCE_SHORT_MSG_SIZE)
RSB_COMMUTATIVE_LONG_MSG_SIZE = 524288  # reduce_scatter.c:14-17


def reduce_binomial(rank_bufs: list[np.ndarray], count: int, esz: int, dt: int, op: int,
                    root: int = 0) -> np.ndarray:
    """MPI_Reduce's binomial tree (reduce_intra_binomial.c:93-140), commutative op:
    relrank r with bit `mask` clear receives the accumulation of relrank r|mask
    and folds it in as the SECOND operand (MPIR_Reduce_local(tmp_buf, recvbuf)),
    so recvbuf = recvbuf (+) tmp.  Returns the root's recvbuf."""
    p = len(rank_bufs)
    acc = [b.view(np.uint8).reshape(-1).copy() for b in rank_bufs]   # indexed by real rank
    mask = 1
    while mask < p:
        for rel in range(0, p, 2 * mask):            # the ranks still receiving at this mask
            src_rel = rel | mask
            if src_rel < p:
                r, src = (rel + root) % p, (src_rel + root) % p
                tmp = acc[src].copy()                # src sent its finished accumulation
                _red(tmp, acc[r], count, dt, op)
        mask <<= 1
    return acc[root]


def allreduce_smp_auto(rank_bufs: list[np.ndarray], count: int, esz: int, dt: int, op: int) -> np.ndarray:
    """MPI_Allreduce on one node with MPICH's algorithm choice: MPIR_Reduce to node
    root 0 (reduce.c:214: reduce_scatter_gather if count*size > 2048 and
    count >= pof2 for a builtin op, else binomial) followed by MPIR_Bcast."""
    p = len(rank_bufs)
    if p == 1:
        return rank_bufs[0].view(np.uint8).reshape(-1).copy()
    if count * esz > REDUCE_SHORT_MSG_SIZE and count >= _pof2(p):
        return allreduce_smp(rank_bufs, count, esz, dt, op)
    return reduce_binomial(rank_bufs, count, esz, dt, op, root=0)


def reduce_scatter_recursive_halving(rank_sendbufs: list[np.ndarray], recvcounts: list[int], esz: int,
                                     dt: int, op: int) -> list[np.ndarray]:
    """Each rank's recvbuf after MPI_Reduce_scatter's recursive halving
    (reduce_scatter_intra_recursive_halving.c; the _block variant,
    reduce_scatter_block_intra_recursive_halving.c:143-300, is this with equal
    counts), step by step:
      pre-fold   even r < 2*rem sends everything to r+1, which computes
                 tmp_results = x_r (+) x_{r-1} (its own data first)
      halving    newrank n, mask = pof2/2 .. 1, partner n ^ mask; the lower
                 newrank keeps the low half of [send_idx, last_idx); received
                 data is folded in as the second operand; newcnts[i] covers
                 old ranks 2i and 2i+1 for i < rem
      final      every participant copies its block; odd r < 2*rem sends
                 block r-1 back to r-1."""
    p = len(rank_sendbufs)
    total = sum(recvcounts)
    disps = [sum(recvcounts[:i]) for i in range(p)]
    res = [b.view(np.uint8).reshape(-1)[:total * esz].copy() for b in rank_sendbufs]   # tmp_results
    pof2 = _pof2(p)
    rem = p - pof2
    newrank = [0] * p
    for r in range(p):
        if r < 2 * rem:
            if r % 2 == 0:
                newrank[r] = -1
            else:
                tmp = res[r - 1].copy()
                _red(tmp, res[r], total, dt, op)
                newrank[r] = r // 2
        else:
            newrank[r] = r - rem
    newcnts = []
    for i in range(pof2):
        old_i = i * 2 + 1 if i < rem else i + rem
        newcnts.append(recvcounts[old_i] + recvcounts[old_i - 1] if old_i < 2 * rem else recvcounts[old_i])
    newdisps = [0] * pof2
    for i in range(1, pof2):
        newdisps[i] = newdisps[i - 1] + newcnts[i - 1]
    real = {newrank[r]: r for r in range(p) if newrank[r] >= 0}
    st = {r: [0, 0, pof2] for r in real.values()}     # send_idx, recv_idx, last_idx
    mask = pof2 >> 1
    while mask > 0:
        plans = {}
        for n, r in real.items():
            s = st[r]
            nd = n ^ mask
            if n < nd:
                s[0] = s[1] + mask
                send_lo, send_hi, recv_lo, recv_hi = s[0], s[2], s[1], s[0]
            else:
                s[1] = s[0] + mask
                send_lo, send_hi, recv_lo, recv_hi = s[0], s[1], s[1], s[2]
            scnt = sum(newcnts[send_lo:send_hi])
            lo = newdisps[send_lo] * esz if send_hi > send_lo else 0
            plans[r] = (real[nd], res[r][lo:lo + scnt * esz].copy(), recv_lo, recv_hi)
        for n, r in real.items():
            peer, _, recv_lo, recv_hi = plans[r]
            rcnt = sum(newcnts[recv_lo:recv_hi])
            if rcnt:
                lo = newdisps[recv_lo] * esz
                data = plans[peer][1]
                assert data.size == rcnt * esz
                _red(data, res[r][lo:lo + rcnt * esz], rcnt, dt, op)
            s = st[r]
            s[0] = s[1]
            s[2] = s[1] + mask
        mask >>= 1
    out = [None] * p
    for r in range(p):
        if newrank[r] >= 0:
            out[r] = res[r][disps[r] * esz:(disps[r] + recvcounts[r]) * esz].copy()
    for r in range(0, 2 * rem, 2):
        out[r] = res[r + 1][disps[r] * esz:(disps[r] + recvcounts[r]) * esz].copy()
    return out


def reduce_scatter_block_recursive_halving(rank_sendbufs: list[np.ndarray], recvcount: int, esz: int,
                                           dt: int, op: int) -> list[np.ndarray]:
    """reduce_scatter_block_intra_recursive_halving.c:143-300 (equal counts)."""
    return reduce_scatter_recursive_halving(rank_sendbufs, [recvcount] * len(rank_sendbufs), esz, dt, op)


def reduce_scatter_pairwise(rank_sendbufs: list[np.ndarray], recvcounts: list[int], esz: int, dt: int,
                            op: int) -> list[np.ndarray]:
    """reduce_scatter_intra_pairwise.c: rank r's block = ((x_r + x_{r-1}) + x_{r-2}) + ..."""
    p = len(rank_sendbufs)
    disps = [sum(recvcounts[:i]) for i in range(p)]
    send = [b.view(np.uint8).reshape(-1) for b in rank_sendbufs]
    recv = [send[r][disps[r] * esz:(disps[r] + recvcounts[r]) * esz].copy() for r in range(p)]
    for i in range(1, p):
        for r in range(p):
            src = (r - i + p) % p
            tmp = send[src][disps[r] * esz:(disps[r] + recvcounts[r]) * esz].copy()
            _red(tmp, recv[r], recvcounts[r], dt, op)
    return recv


def reduce_scatter_auto(rank_sendbufs: list[np.ndarray], recvcounts: list[int], esz: int, dt: int,
                        op: int) -> list[np.ndarray]:
    """MPI_Reduce_scatter with MPICH's choice for a builtin (commutative) op
    (MPIR_Reduce_scatter_intra_auto, reduce_scatter.c)."""
    if sum(recvcounts) * esz < RSB_COMMUTATIVE_LONG_MSG_SIZE:
        return reduce_scatter_recursive_halving(rank_sendbufs, recvcounts, esz, dt, op)
    return reduce_scatter_pairwise(rank_sendbufs, recvcounts, esz, dt, op)


def reduce_scatter_block_auto(rank_sendbufs: list[np.ndarray], recvcount: int, esz: int, dt: int,
                              op: int) -> list[np.ndarray]:
    """MPI_Reduce_scatter_block with MPICH's algorithm choice for a builtin
    (commutative) op (reduce_scatter_block.c:136-148)."""
    if len(rank_sendbufs) * recvcount * esz < RSB_COMMUTATIVE_LONG_MSG_SIZE:
        return reduce_scatter_block_recursive_halving(rank_sendbufs, recvcount, esz, dt, op)
    return reduce_scatter_block_pairwise(rank_sendbufs, recvcount, esz, dt, op)


def reduce_auto(rank_bufs: list[np.ndarray], count: int, esz: int, dt: int, op: int, root: int) -> np.ndarray:
    """MPI_Reduce's result at `root` on one node: reduce_intra_smp.c runs
    MPIR_Reduce_intra_auto over node_comm with the real root (reduce.c:214):
    binomial tree rooted at `root` for short messages, else
    reduce_scatter_gather, whose block values do not depend on the root."""
    p = len(rank_bufs)
    if p == 1:
        return rank_bufs[0].view(np.uint8).reshape(-1).copy()
    if count * esz > REDUCE_SHORT_MSG_SIZE and count >= _pof2(p):
        return allreduce_smp(rank_bufs, count, esz, dt, op)
    return reduce_binomial(rank_bufs, count, esz, dt, op, root=root)


def _scan_rd(rank_sendbufs: list[np.ndarray], count: int, dt: int, op: int, exclusive: bool):
    """The recursive-doubling prefix reductions, step by step.
    scan_intra_recursive_doubling.c:94-147 (inclusive) and
    exscan_intra_recursive_doubling.c:105-170 (exclusive), commutative op:
    partial_scan starts as x_r; at mask m, r exchanges partial_scan with
    r ^ m (< p) and folds the received one in as the SECOND operand; when
    r > r ^ m it also folds it into recvbuf (exclusive: the first one is
    copied).  Returns recvbuf per rank (None for rank 0 of an exscan)."""
    p = len(rank_sendbufs)
    ps = [b.view(np.uint8).reshape(-1).copy() for b in rank_sendbufs]
    rb = [b.copy() if not exclusive else None for b in ps]
    mask = 1
    while mask < p:
        sent = [x.copy() for x in ps]                  # MPIC_Sendrecv reads before this step's folds
        for r in range(p):
            dst = r ^ mask
            if dst >= p:
                continue
            tmp = sent[dst]
            _red(tmp.copy(), ps[r], count, dt, op)
            if r > dst:
                if exclusive and rb[r] is None:
                    rb[r] = tmp.copy()
                else:
                    _red(tmp.copy(), rb[r], count, dt, op)
        mask <<= 1
    return rb


def scan_recursive_doubling(rank_sendbufs: list[np.ndarray], count: int, esz: int, dt: int,
                            op: int) -> list[np.ndarray]:
    """MPI_Scan on one node: MPIR_Scan_intra_auto -> MPIR_Scan_intra_smp (node-
    consecutive), whose single-node case is MPIR_Scan over node_comm, i.e. this
    recursive doubling (scan.c, scan_intra_smp.c)."""
    return _scan_rd(rank_sendbufs, count, dt, op, exclusive=False)


def exscan_recursive_doubling(rank_sendbufs: list[np.ndarray], count: int, esz: int, dt: int,
                              op: int) -> list[np.ndarray]:
    """MPI_Exscan (MPIR_Exscan_intra_auto -> recursive doubling); rank 0 -> None."""
    return _scan_rd(rank_sendbufs, count, dt, op, exclusive=True)


def allreduce_recursive_doubling(rank_bufs: list[np.ndarray], count: int, esz: int, dt: int,
                                 op: int) -> list[np.ndarray]:
    """MPI_Allreduce's flat-branch recursive doubling, step by step
    (allreduce_intra_recursive_doubling.c): even r < 2*rem sends to r+1, which
    folds it in second (x_r (+) x_{r-1}); then at mask 1, 2, 4, ... every newrank
    exchanges its accumulation with newrank ^ mask and folds the received one in
    second; odd r < 2*rem finally hands its result to r-1.  Per-rank results
    (they can differ in operand order, e.g. MAX of +0 / -0)."""
    p = len(rank_bufs)
    pof2 = _pof2(p)
    rem = p - pof2
    acc = [b.view(np.uint8).reshape(-1).copy() for b in rank_bufs]
    real = {}
    for r in range(p):
        if r < 2 * rem:
            if r % 2:
                _red(acc[r - 1].copy(), acc[r], count, dt, op)
                real[r // 2] = r
        else:
            real[r - rem] = r
    mask = 1
    while mask < pof2:
        sent = {r: acc[r].copy() for r in real.values()}
        for n, r in real.items():
            _red(sent[real[n ^ mask]].copy(), acc[r], count, dt, op)
        mask <<= 1
    for r in range(0, 2 * rem, 2):
        acc[r] = acc[r + 1].copy()
    return acc


def allreduce_auto(rank_bufs: list[np.ndarray], count: int, esz: int, dt: int, op: int, smp: bool = True,
                   max_smp: int = 0, short: int = 2048) -> list[np.ndarray]:
    """MPIR_Allreduce_intra_auto (allreduce.c:145-217) for a builtin op on one node,
    per rank.  nbytes is 0 unless MPIR_CVAR_MAX_SMP_ALLREDUCE_MSG_SIZE is set
    (:159), so the SMP branch is taken whenever the SMP CVARs are on, and the flat
    branch then picks recursive doubling; Rabenseifner needs max_smp > 0 and a
    message above `short` with count >= pof2."""
    p = len(rank_bufs)
    nbytes = count * esz if max_smp else 0
    if smp and nbytes <= max_smp:
        res = allreduce_smp_auto(rank_bufs, count, esz, dt, op)
        return [res.copy() for _ in range(p)]
    if p == 1:
        return [rank_bufs[0].view(np.uint8).reshape(-1).copy()]
    if nbytes <= short or count < _pof2(p):
        return allreduce_recursive_doubling(rank_bufs, count, esz, dt, op)
    res = allreduce_rsag(rank_bufs, count, esz, dt, op)
    return [res.copy() for _ in range(p)]

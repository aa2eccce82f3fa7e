"""Short-message reference schedules: the closed forms the device collectives run
agree bit for bit with the step-by-step simulations in oracle/schedules.py.  CPU only.

MPICH switches algorithm on message size:
  MPI_Allreduce (one node) -> MPIR_Reduce to root 0: binomial tree when
      count*size <= 2048 or count < pof2 (reduce.c:214), then MPIR_Bcast;
  MPI_Reduce_scatter_block -> recursive halving when p*recvcount*size < 524288
      (reduce_scatter_block.c:136-141), pairwise above.
The device implementations (csrc/host/coll_hip.c) do not replay those rounds:
they gather the operands a rank needs in one exchange and fold them in the
schedule's association.  These tests pin that fold plan -- restated here in
numpy-free index form and evaluated through the C oracle -- against the
simulations, with MAX over signed zeros and NaN payloads so operand order
(not just association) is checked.
"""
import numpy as np
import pytest

import _types as T
from mpich_pip_amd import DATATYPES, OPS


def _red(orc, tmp, acc, n, t, op):
    assert orc.reduce_local(tmp, acc, n, DATATYPES[t], OPS[op], check=False) == 0


def _pof2(p):
    q = 1
    while q * 2 <= p:
        q *= 2
    return q


def _bitrev(n, bits):
    r = 0
    for i in range(bits):
        if n & (1 << i):
            r |= 1 << (bits - 1 - i)
    return r


def binomial_plan(p):
    """(dst, src) steps: slot dst = slot dst (+) slot src; slots are ranks 0..p-1."""
    steps, mask = [], 1
    while mask < p:
        for r in range(0, p, 2 * mask):
            if r + mask < p:
                steps.append((r, r + mask))
        mask <<= 1
    return steps


def halving_plan(p, rank):
    """RSB recursive halving for block `rank`: (pre-fold steps, tree operand slots)."""
    pof2 = _pof2(p)
    rem = p - pof2
    bits = pof2.bit_length() - 1
    n = rank // 2 if rank < 2 * rem else rank - rem
    real = [2 * m + 1 if m < rem else m + rem for m in range(pof2)]
    pre = [(2 * m + 1, 2 * m) for m in range(rem)]
    tree = [real[n ^ _bitrev(k, bits)] for k in range(pof2)]
    return pre, tree


def tree_fold(orc, slots, count, t, op):
    n, step = len(slots), 1
    while step < n:
        for j in range(0, n, 2 * step):
            _red(orc, slots[j + step], slots[j], count, t, op)
        step *= 2
    return slots[0]


def _inputs(t, op, n, p, seed):
    rng = np.random.default_rng(seed)
    return [T.to_bytes(T.gen(t, n, rng, op)) for _ in range(p)]


CASES = [("MPI_FLOAT", "MPI_SUM"), ("MPIX_C_FLOAT16", "MPI_SUM"), ("MPI_DOUBLE", "MPI_MAX"),
         ("MPI_FLOAT", "MPI_MIN"), ("MPI_DOUBLE_INT", "MPI_MAXLOC")]


@pytest.mark.parametrize("t,op", CASES)
@pytest.mark.parametrize("p", [2, 3, 4, 5, 6, 7, 8, 11, 16])
def test_allreduce_short_binomial_plan(orc, t, op, p):
    from oracle import schedules as S
    esz = T.elem_size(t)
    for count in (1, 3, 2048 // esz):
        xs = _inputs(t, op, count, p, 1000 * p + count)
        want = S.allreduce_smp_auto(xs, count, esz, DATATYPES[t], OPS[op])
        assert np.array_equal(want, S.reduce_binomial(xs, count, esz, DATATYPES[t], OPS[op]))
        slots = [x.copy() for x in xs]
        for dst, src in binomial_plan(p):
            _red(orc, slots[src], slots[dst], count, t, op)
        assert np.array_equal(slots[0], want), f"count {count}"


@pytest.mark.parametrize("t,op", CASES)
@pytest.mark.parametrize("p", [2, 3, 4, 5, 6, 7, 8, 11, 16])
def test_reduce_scatter_block_short_halving_plan(orc, t, op, p):
    from oracle import schedules as S
    esz = T.elem_size(t)
    for rc in (1, 7, 513):
        xs = _inputs(t, op, rc * p, p, 77 * p + rc)
        want = S.reduce_scatter_block_auto(xs, rc, esz, DATATYPES[t], OPS[op])
        nb = rc * esz
        for r in range(p):
            pre, tree = halving_plan(p, r)
            slots = [x[r * nb:(r + 1) * nb].copy() for x in xs]
            for dst, src in pre:
                _red(orc, slots[src], slots[dst], rc, t, op)
            got = tree_fold(orc, [slots[i] for i in tree], rc, t, op)
            assert np.array_equal(got, want[r]), f"p {p} rank {r} recvcount {rc}"


def test_algorithm_switch_points(orc):
    """The size thresholds pick the algorithms MPICH picks (fp32 SUM, p = 8)."""
    from oracle import schedules as S
    p = 8
    for count, small in ((512, True), (513, False), (4, True)):
        xs = _inputs("MPI_FLOAT", "MPI_SUM", count, p, count)
        got = S.allreduce_smp_auto(xs, count, 4, DATATYPES["MPI_FLOAT"], OPS["MPI_SUM"])
        ref = (S.reduce_binomial if small else S.allreduce_smp)(xs, count, 4, DATATYPES["MPI_FLOAT"],
                                                                OPS["MPI_SUM"])
        assert np.array_equal(got, ref)
    # reduce_scatter_block: 524288 total bytes is already "long" (strict <)
    for rc, small in ((16383, True), (16384, False)):
        xs = _inputs("MPI_FLOAT", "MPI_SUM", rc * p, p, rc)
        got = S.reduce_scatter_block_auto(xs, rc, 4, DATATYPES["MPI_FLOAT"], OPS["MPI_SUM"])
        fn = S.reduce_scatter_block_recursive_halving if small else S.reduce_scatter_block_pairwise
        ref = fn(xs, rc, 4, DATATYPES["MPI_FLOAT"], OPS["MPI_SUM"])
        assert all(np.array_equal(a, b) for a, b in zip(got, ref))


@pytest.mark.parametrize("t,op", CASES)
@pytest.mark.parametrize("p", [2, 3, 5, 6, 8])
def test_reduce_short_binomial_plan_any_root(orc, t, op, p):
    """MPI_Reduce, short messages: the binomial tree rooted at `root`
    (relrank = rank - root) is the binomial fold over slots in relrank order."""
    from oracle import schedules as S
    esz = T.elem_size(t)
    count = 5
    xs = _inputs(t, op, count, p, 31 * p)
    for root in range(p):
        want = S.reduce_auto(xs, count, esz, DATATYPES[t], OPS[op], root)
        slots = [xs[(rel + root) % p].copy() for rel in range(p)]
        for dst, src in binomial_plan(p):
            _red(orc, slots[src], slots[dst], count, t, op)
        assert np.array_equal(slots[0], want), f"root {root}"


@pytest.mark.parametrize("t,op", CASES)
@pytest.mark.parametrize("p", [2, 3, 5, 6, 8])
def test_reduce_scatter_irregular_halving_plan(orc, t, op, p):
    """MPI_Reduce_scatter (per-rank counts, zeros included) short path: the
    same fold plan per block as the _block variant, over the simulation."""
    from oracle import schedules as S
    esz = T.elem_size(t)
    rng = np.random.default_rng(p)
    counts = [int(c) for c in rng.integers(0, 40, p)]
    counts[p // 2] = 0
    total = sum(counts)
    disps = [sum(counts[:i]) for i in range(p)]
    xs = _inputs(t, op, total, p, 5 * p)
    want = S.reduce_scatter_auto(xs, counts, esz, DATATYPES[t], OPS[op])
    for r in range(p):
        pre, tree = halving_plan(p, r)
        lo, hi = disps[r] * esz, (disps[r] + counts[r]) * esz
        slots = [x[lo:hi].copy() for x in xs]
        if counts[r]:
            for dst, src in pre:
                _red(orc, slots[src], slots[dst], counts[r], t, op)
            got = tree_fold(orc, [slots[i] for i in tree], counts[r], t, op)
        else:
            got = slots[0]
        assert np.array_equal(got, want[r]), f"p {p} rank {r} counts {counts}"


def test_reduce_scatter_regular_counts_match_block_schedules(orc):
    from oracle import schedules as S
    p, rc = 5, 70000
    xs = _inputs("MPI_FLOAT", "MPI_SUM", rc * p, p, 3)
    a = S.reduce_scatter_pairwise(xs, [rc] * p, 4, DATATYPES["MPI_FLOAT"], OPS["MPI_SUM"])
    b = S.reduce_scatter_block_pairwise(xs, rc, 4, DATATYPES["MPI_FLOAT"], OPS["MPI_SUM"])
    assert all(np.array_equal(x, y) for x, y in zip(a, b))


def scan_plan(r):
    """Device plan for rank r's scan: the partial scans r receives in the
    recursive doubling are, per set bit m of r (increasing), the full tree
    T(d) over z_j = x_{d ^ j}, j < m, with d = r ^ m; the result is the chain
    x_r (+) T(d_1) (+) T(d_2) ... (exscan: the chain without x_r)."""
    out, m = [], 1
    while m <= r:
        if r & m:
            d = r ^ m
            out.append([d ^ j for j in range(m)])
        m <<= 1
    return out


@pytest.mark.parametrize("t,op", CASES)
@pytest.mark.parametrize("p", [1, 2, 3, 5, 6, 8, 13])
@pytest.mark.parametrize("exclusive", [False, True])
def test_scan_plan(orc, t, op, p, exclusive):
    from oracle import schedules as S
    esz = T.elem_size(t)
    count = 7
    xs = _inputs(t, op, count, p, 11 * p)
    fn = S.exscan_recursive_doubling if exclusive else S.scan_recursive_doubling
    want = fn(xs, count, esz, DATATYPES[t], OPS[op])
    for r in range(p):
        parts = [tree_fold(orc, [xs[i].copy() for i in blk], count, t, op) for blk in scan_plan(r)]
        chain = parts if exclusive else [xs[r].copy()] + parts
        if not chain:
            assert r == 0 and want[0] is None
            continue
        acc = chain[0].copy()
        for x in chain[1:]:
            _red(orc, x, acc, count, t, op)
        assert np.array_equal(acc, want[r]), f"rank {r}"


@pytest.mark.parametrize("t,op", CASES)
@pytest.mark.parametrize("p", [2, 3, 5, 6, 8, 11])
def test_allreduce_flat_recursive_doubling_plan(orc, t, op, p):
    """Flat-branch Allreduce (SMP CVARs off): rank r's result is the tree over
    z_j = Y_{n ^ j}, Y_m = x_{2m+1} (+) x_{2m} for m < rem, n = r's newrank
    (an excluded even rank takes its odd neighbour's)."""
    from oracle import schedules as S
    esz = T.elem_size(t)
    count = 9
    xs = _inputs(t, op, count, p, 13 * p)
    want = S.allreduce_auto(xs, count, esz, DATATYPES[t], OPS[op], smp=False)
    pof2 = _pof2(p)
    rem = p - pof2
    for r in range(p):
        slots = [x.copy() for x in xs]
        for m in range(rem):
            _red(orc, slots[2 * m], slots[2 * m + 1], count, t, op)
        n = r // 2 if r < 2 * rem else r - rem
        real = [2 * m + 1 if m < rem else m + rem for m in range(pof2)]
        got = tree_fold(orc, [slots[real[n ^ j]] for j in range(pof2)], count, t, op)
        assert np.array_equal(got, want[r]), f"rank {r}"


def test_allreduce_flat_branch_choice(orc):
    """nbytes is 0 unless MAX_SMP_ALLREDUCE_MSG_SIZE is set: with the SMP CVARs
    off the flat branch is recursive doubling at every size; Rabenseifner only
    with a nonzero MAX_SMP_ALLREDUCE_MSG_SIZE and a long message."""
    from oracle import schedules as S
    p, count = 6, 4099
    xs = _inputs("MPI_DOUBLE", "MPI_SUM", count, p, 1)
    dt, o = DATATYPES["MPI_DOUBLE"], OPS["MPI_SUM"]
    rd = S.allreduce_recursive_doubling(xs, count, 8, dt, o)
    assert all(np.array_equal(a, b) for a, b in zip(S.allreduce_auto(xs, count, 8, dt, o, smp=False), rd))
    rab = S.allreduce_rsag(xs, count, 8, dt, o)
    got = S.allreduce_auto(xs, count, 8, dt, o, smp=True, max_smp=1)
    assert all(np.array_equal(a, rab) for a in got)

"""bench_coll.py's on-transport self-check (numpy, same association) agrees
bit for bit with the oracle's step-by-step reference schedules
(oracle/schedules.py), so a "bitexact: true" in the N > 1 bench line means
parity with the reference order.  CPU only."""
import numpy as np
import pytest

import bench_coll as B
from mpich_pip_amd import MPI_FLOAT, MPIX_C_FLOAT16, MPI_SUM


@pytest.mark.parametrize("p", [2, 4, 8])
def test_allreduce_expectation_matches_schedule(orc, p):
    from oracle import schedules as S
    n = 4099 + p
    xs = [np.random.default_rng(77 + r).uniform(-1, 1, n).astype(np.float32) for r in range(p)]
    want = S.allreduce_smp([x.view(np.uint8) for x in xs], n, 4, MPI_FLOAT, MPI_SUM)
    assert np.array_equal(B.expect_allreduce(xs).view(np.uint8), want)


@pytest.mark.parametrize("p", [2, 3, 4, 8])
def test_reduce_scatter_expectation_matches_schedule(orc, p):
    from oracle import schedules as S
    rc = 1031
    hs = [np.random.default_rng(91 + r).uniform(-4, 4, rc * p).astype(np.float16) for r in range(p)]
    want = S.reduce_scatter_block_pairwise([h.view(np.uint8) for h in hs], rc, 2, MPIX_C_FLOAT16, MPI_SUM)
    for r in range(p):
        assert np.array_equal(B.expect_reduce_scatter_block(hs, r, rc).view(np.uint8), want[r][:rc * 2])


@pytest.mark.parametrize("p", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("exclusive", [False, True])
def test_scan_expectation_matches_schedule(orc, p, exclusive):
    from oracle import schedules as S
    n = 1031
    xs = [np.random.default_rng(5 + r).uniform(-1, 1, n).astype(np.float32) for r in range(p)]
    fn = S.exscan_recursive_doubling if exclusive else S.scan_recursive_doubling
    want = fn([x.view(np.uint8) for x in xs], n, 4, MPI_FLOAT, MPI_SUM)
    for r in range(p):
        got = B.expect_scan(xs, r, exclusive)
        if want[r] is None:
            assert got is None
        else:
            assert np.array_equal(got.view(np.uint8), want[r])


@pytest.mark.parametrize("p", [2, 4, 8])
def test_reduce_expectation_matches_schedule(orc, p):
    """The bench's Reduce check (root p-1, long message) reuses the allreduce closed form."""
    from oracle import schedules as S
    n = (1 << 16) + 3
    xs = [np.random.default_rng(77 + r).uniform(-1, 1, n).astype(np.float32) for r in range(p)]
    want = S.reduce_auto([x.view(np.uint8) for x in xs], n, 4, MPI_FLOAT, MPI_SUM, p - 1)
    assert np.array_equal(B.expect_allreduce(xs).view(np.uint8), want)

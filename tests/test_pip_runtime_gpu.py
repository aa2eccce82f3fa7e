"""Config 1 with a GPU visible: `mpiexec -n N examples/cpi`
and builtin MPI_Reduce through the runtime subset, every combine step running
MPIR_Reduce_local on host operands (the host combine by default).

Expected values:
  * cpi, np = 2: the reference's golden line;
  * cpi, other np: the same arithmetic in Python (IEEE double, same order) and
    the binomial combine order of reduce_intra_binomial.c:100-160;
  * MPI_Reduce of 4099 doubles (> 2048 B, so reduce-scatter + gather,
    reduce.c:214-216): oracle/schedules.py's step-by-step
    reduce_intra_reduce_scatter_gather on the CPU oracle -- bit for bit.
"""
import os
import struct

import numpy as np
import pytest

from test_pip_runtime_cpu import MPIEXEC, ROOT, build_prog, parse, run

pytestmark = pytest.mark.gpu
CPI = os.path.join(ROOT, "examples", "cpi")


def cpi_partial(rank, nprocs, n=10000):
    h = 1.0 / n
    s = 0.0
    for k in range(rank + 1, n + 1, nprocs):
        x = h * (float(k) - 0.5)
        s += 4.0 / (1.0 + x * x)
    return h * s


def binomial_sum(xs, root=0):
    p, acc, mask = len(xs), list(xs), 1
    while mask < p:
        for rel in range(0, p, 2 * mask):
            if rel | mask < p:
                a, b = (rel + root) % p, ((rel | mask) + root) % p
                acc[a] = acc[a] + acc[b]
        mask <<= 1
    return acc[root]


def test_cpi_np2_golden(cuda):
    r = run(2, CPI, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "pi is approximately 3.1415926544231318, Error is 0.0000000008333387" in r.stdout


@pytest.mark.parametrize("n", [1, 3, 4, 8])
def test_cpi_other_sizes(cuda, n):
    r = run(n, CPI, timeout=300)
    assert r.returncode == 0, r.stderr
    want = binomial_sum([cpi_partial(q, n) for q in range(n)])
    assert f"pi is approximately {want:.16f}," in r.stdout


@pytest.fixture(scope="module")
def prog(tmp_path_factory, mpi):
    return build_prog(tmp_path_factory)


def fnv(b: bytes) -> str:
    h = 1469598103934665603
    for c in b:
        h = ((h ^ c) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return f"{h:016x}"


def inputs(rank, n):
    return np.array([((rank + 1) * 0.1 + i * 1e-3) + 1.0 / (3.0 + rank + i) for i in range(n)], dtype=np.float64)


@pytest.mark.parametrize("p", [2, 3, 5, 8])
def test_builtin_reduce_schedules(cuda, orc, mpi, prog, p):
    r = run(p, prog, "gpu", timeout=400)
    assert r.returncode == 0, r.stderr
    check_builtin_reduce_rows(parse(r.stdout), p, mpi)


def check_builtin_reduce_rows(rows, p, mpi):
    """pip_plumbing's `dreduce` rows against the oracle (binomial for count 1,
    reduce-scatter + gather for count 4099)."""
    from oracle import schedules as S
    assert rows["errs"][0] == ["7", "5", "2", "9"]
    got = {(int(n), int(root)): (int(rc), h) for n, root, rc, h, _ in rows["dreduce"]}
    assert len(got) == 2 * p
    for root in range(p):
        # count 1: binomial
        want1 = binomial_sum([inputs(q, 1)[0] for q in range(p)], root)
        assert got[(1, root)] == (0, fnv(struct.pack("<d", want1))), root
        # count 4099: reduce-scatter + gather in the reference's order
        xs = [inputs(q, 4099).view(np.uint8) for q in range(p)]
        want = S.allreduce_smp(xs, 4099, 8, mpi.MPI_DOUBLE, mpi.MPI_SUM)
        assert got[(4099, root)] == (0, fnv(want.tobytes())), root

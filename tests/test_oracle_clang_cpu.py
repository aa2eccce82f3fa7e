"""The clang -O2 build of the oracle (oracle/liboracle_clang.so) computes what the
gcc -O2 build computes on finite inputs, so bench.py's second CPU-baseline line
("also report clang -O2") times the same arithmetic.  NaN
operands are excluded: there the two compilers' vectorized loops differ
(DESIGN.md §(c), "Documented build dependence"), and the gcc build is the checker.
"""
import ctypes

import numpy as np
import pytest

import oracle

MPI_INT, MPI_LONG, MPI_FLOAT, MPI_DOUBLE = 0x4c000405, 0x4c000807, 0x4c00040a, 0x4c00080b
OPS = {"MAX": 0x58000001, "MIN": 0x58000002, "SUM": 0x58000003, "PROD": 0x58000004}
TYPES = {MPI_INT: np.int32, MPI_LONG: np.int64, MPI_FLOAT: np.float32, MPI_DOUBLE: np.float64}


def _inputs(npt, n, seed):
    rng = np.random.default_rng(seed)
    if np.issubdtype(npt, np.integer):
        info = np.iinfo(npt)
        return (rng.integers(info.min, info.max, n, dtype=npt, endpoint=True),
                rng.integers(info.min, info.max, n, dtype=npt, endpoint=True))
    a = rng.uniform(-4, 4, n).astype(npt)
    b = rng.uniform(-4, 4, n).astype(npt)
    a[:6] = [0.0, -0.0, np.inf, -np.inf, np.finfo(npt).tiny / 4, np.finfo(npt).max]
    b[:6] = [-0.0, 0.0, 1.0, -np.inf, np.finfo(npt).tiny / 2, np.finfo(npt).max]
    return a, b


@pytest.mark.parametrize("op", sorted(OPS))
@pytest.mark.parametrize("dt", sorted(TYPES))
def test_clang_build_matches_gcc_build(op, dt):
    npt = TYPES[dt]
    n = 10007
    a, b = _inputs(npt, n, 0xC1A6 + dt % 97)
    want, got = a.copy(), a.copy()
    with np.errstate(all="ignore"):
        assert oracle.reduce_local(b, want, n, dt, OPS[op]) == 0
        clang = oracle.load_clang()
        assert clang.oracle_reduce_local(ctypes.c_void_p(b.ctypes.data), ctypes.c_void_p(got.ctypes.data),
                                         n, dt, OPS[op]) == 0
    assert np.array_equal(want.view(f"u{npt().itemsize}"), got.view(f"u{npt().itemsize}"))


def test_clang_cpu_baseline_runs():
    assert oracle.cpu_baseline_sum_f32(2, 1 << 16, 2, "clang") > 0

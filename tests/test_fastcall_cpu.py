"""The compiled binding's C loop (csrc/py/fastcall.c reduce_local_loop), which
bench.py times the headline with: call i uses arg_sets[(start + i) % len], the
loop stops at the first error and returns its code.  Host buffers (the host
combine), so it runs without a GPU."""
import numpy as np

import pytest


def test_loop_order_and_counts(mpi):
    f = mpi.fast_reduce_local_loop()
    a = np.zeros(8 * 5)
    b = np.ones(8 * 5)
    sets = tuple((b.ctypes.data + 64 * j, a.ctypes.data + 64 * j, 8, mpi.MPI_DOUBLE, mpi.MPI_SUM) for j in range(5))
    assert f(sets, 3, 12) == 0          # sets 3 4 0 1 2 3 4 0 1 2 3 4
    assert a.reshape(5, 8).tolist() == [[2.0] * 8, [2.0] * 8, [2.0] * 8, [3.0] * 8, [3.0] * 8]
    assert f(sets, 0, 0) == 0
    assert f(sets[:2], 1, 3) == 0       # fewer sets than calls: 1 0 1
    assert a[0] == 3.0 and a[8] == 4.0


def test_loop_stops_at_first_error(mpi):
    f = mpi.fast_reduce_local_loop()
    a = np.zeros(4)
    b = np.ones(4)
    good = (b.ctypes.data, a.ctypes.data, 4, mpi.MPI_DOUBLE, mpi.MPI_SUM)
    bad = (b.ctypes.data, a.ctypes.data, 4, mpi.MPI_DOUBLE, mpi.MPI_OP_NULL)
    rc = f((good, bad, good), 0, 3)
    assert mpi.error_class(rc) == mpi.MPI_ERR_OP
    assert a[0] == 1.0                  # the third call never ran


def test_loop_rejects_bad_arguments(mpi):
    f = mpi.fast_reduce_local_loop()
    with pytest.raises(TypeError):
        f([(0, 0, 0, 0, 0)], 0, 1)
    with pytest.raises(ValueError):
        f((), 0, 1)
    with pytest.raises(TypeError):
        f(((1, 2, 3),), 0, 1)

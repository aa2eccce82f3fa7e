"""The host combine on a rank with no visible GPU (CPU tests).

Both operands in host memory take the library's host combine -- the kernels'
own functors (reduce_ops.hpp, __host__ __device__) compiled by hipcc for the
host, split over the library's host threads from 512 KiB.  It is product code,
not the oracle, and needs no device: a CPU-only rank of a job reduces host
buffers as the reference's loop does anywhere (opsum.c:21).  Every (op, type)
pair the reference accepts, edge values included, aligned and misaligned, plus
the thread-split sizes -- bit-exact against the oracle (the same checker as
test_parity_gpu.py::test_host_path_matrix_vs_oracle, which runs it with a GPU
visible).  This container has no GPU, so MPIR_Hip_device_count() is 0 here.
"""
import pytest

from test_parity_gpu import MATRIX, run_pair_host
import _types as T


@pytest.fixture(scope="module")
def no_gpu(mpi):
    if mpi.load().MPIR_Hip_device_count() != 0:
        pytest.skip("a GPU is visible: test_parity_gpu.py covers the host combine there")


@pytest.mark.parametrize("op,t", MATRIX, ids=[f"{o}-{t}" for o, t in MATRIX])
def test_host_combine_matrix_no_device(mpi, orc, no_gpu, op, t):
    for n, seed, off in ((1, 11, 0), (7, 12, 3), (1000, 13, 0), (4099, 14, 1)):
        run_pair_host(mpi, orc, op, t, n, seed, off)


@pytest.mark.parametrize("op,t", [("MPI_SUM", "MPI_FLOAT"), ("MPI_PROD", "MPI_C_DOUBLE_COMPLEX"),
                                  ("MPI_MAXLOC", "MPI_DOUBLE_INT"), ("MPI_BXOR", "MPI_UNSIGNED_CHAR"),
                                  ("MPI_SUM", "MPI_LONG_DOUBLE"), ("MPI_SUM", "MPIX_C_FLOAT16")])
def test_host_combine_thread_split_no_device(mpi, orc, no_gpu, op, t):
    """From 512 KiB per operand the combine is split over the host threads
    (parts on 64-byte boundaries): ragged and misaligned element counts."""
    esz = T.elem_size(t)
    for n, off in (((600 << 10) // esz + 3, 0), ((600 << 10) // esz + 1, 3), ((4 << 20) // esz + 5, 0)):
        run_pair_host(mpi, orc, op, t, n, 21 + n, off)


def test_host_limit_zero_still_combines_without_device(mpi, orc, no_gpu):
    """A host limit of 0 sends both-host calls to GPU staging when a device
    exists; with none, the host combine takes them (no MPI_ERR_OTHER)."""
    from test_parity_gpu import host_max
    with host_max(mpi, 0):
        run_pair_host(mpi, orc, "MPI_SUM", "MPI_DOUBLE", 4099, 5, 0)

"""pytest configuration: the `gpu` marker, import paths, shared fixtures.

`-m "not gpu"` tests run anywhere (oracle vs golden vectors, host logic,
C-ABI exports); `-m gpu` tests need an MI355X and call the HIP path through
the C ABI, checking it against the oracle.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "mpich-pip_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP GPU (MI355X); runs the gfx950 kernels")


@pytest.fixture(scope="session")
def mpi():
    """The product C-ABI library (ctypes), errors returned instead of fatal."""
    import mpich_pip_amd as m
    lib = m.load()
    assert lib.MPIX_Reduce_local_set_errhandler(m.MPI_ERRORS_RETURN) == 0
    return m


@pytest.fixture(scope="session")
def orc():
    import oracle
    oracle.load()
    return oracle


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test requires a HIP device (torch.cuda.is_available() is False)")
    return torch

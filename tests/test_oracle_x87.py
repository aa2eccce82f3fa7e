"""long double (x87 80-bit) on the CPU: the software x87 the gfx950 kernels run
(mpich-pip_amd/csrc/hip/x87.hpp, compiled for the host) against the host's
x87 unit over every encoding class, and the oracle's long double loops
against the reference's codegen facts (10-byte stores: padding untouched;
unordered compares keep / select exactly as MPL_MAX and the MAXLOC branches
do).  The gfx950 kernels themselves are compared with the oracle in
test_parity_gpu.py.
"""
import os
import subprocess

import numpy as np
import pytest

import _types as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def x87_check(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("x87") / "x87_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "mpich-pip_amd", "csrc", "hip"),
                    os.path.join(ROOT, "tests", "progs", "x87_check.cpp"), "-o", exe], check=True)
    return exe


@pytest.mark.parametrize("seed", [1, 2])
def test_soft_x87_matches_host_x87(x87_check, seed):
    r = subprocess.run([x87_check, "1000000", str(seed)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 6 and all(ln.endswith(" 0 mismatches") for ln in lines), r.stdout


def enc(m, se, pad=b"\xaa" * 6):
    x = np.zeros(1, dtype=T.X80)
    x["m"], x["se"], x["pad"] = m, se, np.frombuffer(pad, dtype="V6")
    return x


@pytest.mark.parametrize("op", ["MPI_SUM", "MPI_PROD", "MPI_MAX", "MPI_MIN", "MPI_LXOR"])
def test_oracle_long_double_keeps_padding(orc, mpi, op):
    a = enc(0xC000000000000000, 0x3FFF, b"\x11" * 6)        # 1.5, inout
    b = enc(0x8000000000000000, 0x4000, b"\x22" * 6)        # 2.0, in
    io = T.to_bytes(a).copy()
    assert orc.reduce_local(T.to_bytes(b).copy(), io, 1, mpi.MPI_LONG_DOUBLE, mpi.OPS[op]) == 0
    assert bytes(io[10:16]) == b"\x11" * 6


def test_oracle_long_double_nan_rules(orc, mpi):
    """x87 (SDM vol. 1 Table 4-7): larger-significand NaN wins, SNaN quieted,
    SNaN + QNaN -> the QNaN, invalid encodings -> real indefinite."""
    cases = [
        ((0xC000000000000001, 0x7FFF), (0xC000000000000002, 0x7FFF), (0xC000000000000002, 0x7FFF)),
        ((0xC000000000000005, 0xFFFF), (0xC000000000000005, 0x7FFF), (0xC000000000000005, 0x7FFF)),
        ((0x8000000000000009, 0x7FFF), (0xC000000000000001, 0x7FFF), (0xC000000000000001, 0x7FFF)),
        ((0x8000000000000002, 0x7FFF), (0x8000000000000001, 0x7FFF), (0xC000000000000002, 0x7FFF)),
        ((0x4000000000000000, 0x3FFF), (0xC000000000000007, 0x7FFF), (0xC000000000000000, 0xFFFF)),
        ((0x8000000000000000, 0x7FFF), (0x8000000000000000, 0xFFFF), (0xC000000000000000, 0xFFFF)),
    ]
    for (am, ase), (bm, bse), (wm, wse) in cases:
        io = T.to_bytes(enc(am, ase)).copy()
        assert orc.reduce_local(T.to_bytes(enc(bm, bse)).copy(), io, 1, mpi.MPI_LONG_DOUBLE, mpi.MPI_SUM) == 0
        got = io.view(T.X80)[0]
        assert (int(got["m"]), int(got["se"])) == (wm, wse), (hex(am), hex(bm))

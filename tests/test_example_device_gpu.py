"""examples/reduce_local_device.c: MPI_Reduce_local from a plain C program
with one HIP runtime (no Python, no torch): device + device (the kernel in
place), pinned host + device, pageable host + host, each bit-exact against a
sequential fp32 loop over the same inputs (the reference's opsum.c:21-76
order), and the synchronous call's time in a loop."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "reduce_local_device")


@pytest.mark.gpu
@pytest.mark.parametrize("count", [(1 << 22) + 5, 1, 67108864])
def test_plain_c_device_program(count):
    assert os.path.exists(EXE), "build it first: make -C mpich-pip_amd examples"
    r = subprocess.run([EXE, str(count), "20"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "reduce_local_device ok" in r.stdout, r.stdout
    assert r.stdout.count("bit-exact") == 3, r.stdout

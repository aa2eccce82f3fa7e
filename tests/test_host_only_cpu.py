"""Host-buffer MPI_Reduce_local behaves like MPICH's loop inside a process
(reference opsum.c:21-76 via reduce_local.c:35-122, a
single-threaded scalar loop that touches no device and starts no thread).

Each case runs in a fresh child process pinned with `taskset`, so the
library's thread pool is sized from that affinity mask the first time it is
needed:
  * one usable CPU: a 4 MiB combine (above the 512 KiB split threshold)
    starts no thread -- /proc/self/task is unchanged -- and is bit-exact
    against the oracle;
  * two usable CPUs: at most one worker beside the caller.
The GPU-side half (no /dev/kfd opened by host-only calls on a GPU box) is
tests/test_host_only_gpu.py.
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, sys
sys.path[:0] = [{root!r}, os.path.join({root!r}, "mpich-pip_amd")]
import numpy as np
import mpich_pip_amd as m
import oracle
lib = m.load()
oracle.load()
tasks = lambda: len(os.listdir("/proc/self/task"))
rng = np.random.default_rng(7)
n = (4 << 20) // 8 + 3                       # 4 MiB of doubles, ragged
a = rng.uniform(-1, 1, n)
b = rng.uniform(-1, 1, n)
want = a.copy()
assert oracle.reduce_local(b.copy(), want, n, m.MPI_DOUBLE, m.MPI_SUM) == 0
before = tasks()
for _ in range(3):
    got = a.copy()
    assert lib.MPI_Reduce_local(b.ctypes.data, got.ctypes.data, n, m.MPI_DOUBLE, m.MPI_SUM) == 0
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))
print(before, tasks())
"""


def _run(cpus):
    if not shutil.which("taskset"):
        pytest.skip("taskset not available")
    avail = sorted(os.sched_getaffinity(0))
    if len(avail) < len(cpus):
        pytest.skip(f"needs {len(cpus)} CPUs")
    mask = ",".join(str(avail[c]) for c in cpus)
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1")
    env.pop("MPIR_CVAR_REDUCE_LOCAL_STAGE_THREADS", None)
    p = subprocess.run(["taskset", "-c", mask, sys.executable, "-c", CHILD.format(root=ROOT)],
                       capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    before, after = map(int, p.stdout.split()[-2:])
    return before, after


def test_one_cpu_starts_no_thread():
    before, after = _run([0])
    assert after == before, f"{after - before} thread(s) started on a one-CPU rank"


def test_two_cpus_one_worker_at_most():
    before, after = _run([0, 1])
    assert after - before <= 1, f"{after - before} threads started for two usable CPUs"

"""The host combine shares the node's CPUs with the other ranks on it
(reference: one single-threaded loop per rank, opsum.c:21-76,
and Hydra's MPI_LOCALNRANKS, pmip_cb.c:658-662).

8 processes under one shared affinity mask, each told MPI_LOCALNRANKS=8, do a
64 MiB fp32 SUM MPI_Reduce_local on host buffers at the same moment (a barrier
on a pipe, tests/_local_ranks.py): together they run no more threads than the
CPUs the job may use, and every result is bit-exact against the oracle.  The
sizing rule itself (hip_reduce.hip share_threads) is checked through single
processes under chosen masks and rank counts.
"""
import os
import shutil
import subprocess
import sys

import pytest

import _local_ranks

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_eight_ranks_share_the_node():
    res = _local_ranks.run(8, mib=64, reps=2, localnranks=8)
    assert res["exact"], res
    assert res["threads"] <= res["usable_cpus"], res
    # every rank sized its pool to its share, and started no more than that
    share = max(1, min(16, res["usable_cpus"] // 8))
    for r in res["ranks"]:
        assert r["pool"] == share, r
        assert r["workers"] <= share - 1, r


POOL = r"""
import sys
sys.path[:0] = [{root!r}, {pkg!r}]
import mpich_pip_amd as m
print(m.load().MPIR_Hip_host_threads())
"""


def _pool(cpus, env_extra):
    if not shutil.which("taskset"):
        pytest.skip("taskset not available")
    avail = sorted(os.sched_getaffinity(0))
    if len(avail) < len(cpus):
        pytest.skip(f"needs {len(cpus)} CPUs")
    env = dict(os.environ)
    for k in ("MPIR_CVAR_REDUCE_LOCAL_STAGE_THREADS", "MPI_LOCALNRANKS", "MPIR_PIP_SIZE", "LOCAL_WORLD_SIZE",
              "OMPI_COMM_WORLD_LOCAL_SIZE"):
        env.pop(k, None)
    env.update(env_extra)
    mask = ",".join(str(avail[c]) for c in cpus)
    code = POOL.format(root=ROOT, pkg=os.path.join(ROOT, "mpich-pip_amd"))
    p = subprocess.run(["taskset", "-c", mask, sys.executable, "-c", code], capture_output=True, text=True,
                       timeout=120, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    return int(p.stdout.split()[-1])


def _quota():
    q = _local_ranks.usable_cpus()
    return q if q < len(os.sched_getaffinity(0)) else None


@pytest.mark.skipif(len(os.sched_getaffinity(0)) < 8 or len(os.sched_getaffinity(0)) != _local_ranks.job_cpus(),
                    reason="needs an unbound process on a node of >= 8 CPUs")
def test_sizing_rule():
    c = _local_ranks.job_cpus()
    q = _quota()
    full = list(range(c))

    def want(mask, L):
        sharers = max(1, min(L, -(-(L * mask) // c)))
        n = mask // sharers
        if q:
            n = min(n, q // L)
        return max(1, min(16, n))

    # unbound ranks: the node's CPUs split L ways (each launcher's variable)
    for var in ("MPI_LOCALNRANKS", "MPIR_PIP_SIZE", "LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE"):
        assert _pool(full, {var: "4"}) == want(c, 4), var
    assert _pool(full, {}) == want(c, 1)
    assert _pool(full, {"MPI_LOCALNRANKS": str(4 * c)}) == 1          # fewer CPUs than ranks: the caller alone
    # ranks bound to disjoint halves: each owns its half
    half = list(range(c // 2))
    assert _pool(half, {"MPI_LOCALNRANKS": "2"}) == want(c // 2, 2)
    # the first variable found wins (Hydra's over torchrun's)
    assert _pool(full, {"MPI_LOCALNRANKS": "2", "LOCAL_WORLD_SIZE": "8"}) == want(c, 2)
    # the explicit cvar overrides the share
    assert _pool(full, {"MPI_LOCALNRANKS": "8", "MPIR_CVAR_REDUCE_LOCAL_STAGE_THREADS": "3"}) == 3

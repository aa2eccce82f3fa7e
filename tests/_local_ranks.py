"""N ranks of one node reaching a host-buffer combine at the same moment
(VERDICT r4 #1): the harness behind tests/test_local_ranks_cpu.py and
tools/local_ranks_ab.py.

Every rank of a host-buffer MPI_Allreduce reaches its combine together (the
reference's combine is a single-threaded loop per rank, opsum.c:21-76).  Each
of `nranks` child processes, started under the parent's affinity mask with
the launcher's environment (MPI_LOCALNRANKS, as Hydra sets it,
pmip_cb.c:658-662), allocates its operands, then blocks on a shared pipe;
the parent releases all of them at once, and each times `reps` 64 MiB fp32
MPI_SUM MPI_Reduce_local calls on host buffers (accumulating into one inoutbuf).  A child reports the
threads the library started (/proc/self/task before / after), its pool size
(MPIR_Hip_host_threads), its wall time and whether every result was bit-exact
against the oracle (the checker runs after the timed region).
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys, time
sys.path[:0] = [{root!r}, os.path.join({root!r}, "mpich-pip_amd")]
import numpy as np
import mpich_pip_amd as m
import oracle
lib = m.load()
oracle.load()
rank, reps, n = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
go = int(sys.argv[4])
tasks = lambda: len(os.listdir("/proc/self/task"))
rng = np.random.default_rng(100 + rank)
a = rng.uniform(-1, 1, n).astype(np.float32)
b = rng.uniform(-1, 1, n).astype(np.float32)
out = a.copy()
before = tasks()
print("ready", flush=True)
os.read(go, 1)                                  # the barrier: one byte per rank
t0 = time.perf_counter()
for k in range(reps):                           # out = ((a + b) + b) + ...
    rc = lib.MPI_Reduce_local(b.ctypes.data, out.ctypes.data, n, m.MPI_FLOAT, m.MPI_SUM)
    assert rc == 0, rc
t1 = time.perf_counter()
after = tasks()
want = a.copy()
for k in range(reps):
    assert oracle.reduce_local(b.copy(), want, n, m.MPI_FLOAT, m.MPI_SUM) == 0
exact = bool(np.array_equal(out.view(np.uint32), want.view(np.uint32)))
print(json.dumps({{"rank": rank, "workers": after - before, "pool": lib.MPIR_Hip_host_threads(),
                   "t0": t0, "t1": t1, "exact": exact}}), flush=True)
"""


def _cpulist(path: str) -> int:
    try:
        txt = open(path).read().strip()
    except OSError:
        return 0
    n = 0
    for part in txt.split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        n += int(b or a) - int(a) + 1
    return n


def job_cpus() -> int:
    """The CPUs the job's ranks share, as the library counts them
    (hip_reduce.hip online_cpus): the cgroup's cpuset, else the online CPUs."""
    for path in ("/sys/fs/cgroup/cpuset.cpus.effective", "/sys/fs/cgroup/cpuset/cpuset.effective_cpus"):
        n = _cpulist(path)
        if n:
            return n
    return os.cpu_count()


def usable_cpus() -> int:
    """This process's affinity mask, capped by a cgroup CPU quota (v2 or v1)."""
    n = len(os.sched_getaffinity(0))
    quota = period = 0
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            quota, period = int(q), int(p)
    except (OSError, ValueError):
        try:
            quota = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            period = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        except (OSError, ValueError):
            pass
    if quota > 0 and period > 0:
        n = min(n, -(-quota // period))
    return n


def run(nranks: int, mib: int = 64, reps: int = 3, localnranks: int | None = None,
        stage_threads: int | None = None, timeout: float = 300) -> dict:
    """Runs the children; returns per-rank records and the aggregate rate
    (3 x operand bytes per call -- two reads, one write -- over the span from
    the first start to the last end, in GiB/s)."""
    n = (mib << 20) // 4
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", HIP_VISIBLE_DEVICES="-1")
    for k in ("MPIR_CVAR_REDUCE_LOCAL_STAGE_THREADS", "MPI_LOCALNRANKS", "MPIR_PIP_SIZE", "LOCAL_WORLD_SIZE",
              "OMPI_COMM_WORLD_LOCAL_SIZE"):
        env.pop(k, None)
    if localnranks is not None:
        env["MPI_LOCALNRANKS"] = str(localnranks)
    if stage_threads is not None:
        env["MPIR_CVAR_REDUCE_LOCAL_STAGE_THREADS"] = str(stage_threads)
    rfd, wfd = os.pipe()
    procs = []
    try:
        for r in range(nranks):
            procs.append(subprocess.Popen(
                [sys.executable, "-c", CHILD.format(root=ROOT), str(r), str(reps), str(n), str(rfd)],
                stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env, pass_fds=(rfd,)))
        deadline = time.time() + timeout
        for p in procs:
            line = p.stdout.readline()
            if line.strip() != "ready":
                raise RuntimeError(f"child not ready: {line!r} {p.stderr.read()[-2000:]}")
            if time.time() > deadline:
                raise TimeoutError("children did not get ready")
        os.write(wfd, b"x" * nranks)            # release every rank at once
        recs = []
        for p in procs:
            out, err = p.communicate(timeout=max(1.0, deadline - time.time()))
            if p.returncode != 0:
                raise RuntimeError(f"child failed ({p.returncode}): {err[-2000:]}")
            recs.append(json.loads(out.strip().splitlines()[-1]))
    finally:
        os.close(rfd)
        os.close(wfd)
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    span = max(r["t1"] for r in recs) - min(r["t0"] for r in recs)
    total = 3.0 * (mib << 20) * reps * nranks
    return {"ranks": recs, "span_s": span, "gib_s": total / span / 2**30,
            "threads": sum(r["workers"] + 1 for r in recs), "usable_cpus": usable_cpus(),
            "exact": all(r["exact"] for r in recs)}

"""Config-1 plumbing without a GPU: bin/mpiexec, the
shared-memory world, MPI_Init/Comm_size/rank/Bcast/Barrier/Finalize, and
MPI_Reduce's binomial schedule driven with a user-defined (host) op whose
result fingerprints the exact combine order (reduce_intra_binomial.c:100-160).
Builtin-op reductions on host buffers run the library's host combine (the
kernels' functors compiled for the host -- product code, not the oracle), which
needs no device, as the reference's loop (opsum.c:21) runs anywhere: cpi's
golden line and MPI_Reduce's schedules are checked here on a CPU-only rank
(HIP_VISIBLE_DEVICES=-1) against the oracle, and again with a GPU visible in
test_pip_runtime_gpu.py.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPIEXEC = os.path.join(ROOT, "mpich-pip_amd", "bin", "mpiexec")
LIBDIR = os.path.join(ROOT, "mpich-pip_amd", "lib")
M32 = 0xFFFFFFFF


def build_prog(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("progs") / "pip_plumbing")
    subprocess.run(["gcc", "-O2", "-std=gnu99", "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "progs", "pip_plumbing.c"), "-o", out,
                    "-L" + LIBDIR, "-lmpich_reduce_local", "-Wl,-rpath," + LIBDIR], check=True)
    return out


@pytest.fixture(scope="module")
def prog(tmp_path_factory, mpi):
    assert os.path.exists(MPIEXEC), "run `make -C mpich-pip_amd` first"
    return build_prog(tmp_path_factory)


def run(n, *cmd, timeout=120, env=None):
    return subprocess.run([MPIEXEC, "-n", str(n), "--timeout", str(timeout - 10), *cmd],
                          capture_output=True, text=True, timeout=timeout, env=env)


NO_GPU = dict(os.environ, HIP_VISIBLE_DEVICES="-1")


def val(rank, i):
    return (rank * 1000003 + i * 7919 + 17) & M32


def fp(inv, inout):
    return (31 * inv + inout) & M32


def binomial(xs, root, commute):
    """reduce_intra_binomial.c:100-160 on scalars: returns the root's value."""
    p = len(xs)
    lroot = root if commute else 0
    acc = list(xs)
    mask = 1
    while mask < p:
        for rel in range(0, p, 2 * mask):
            src = rel | mask
            if src < p:
                a, b = (rel + lroot) % p, (src + lroot) % p
                # commutative: MPIR_Reduce_local(tmp=recv, recvbuf); else (recvbuf, tmp) + copy
                acc[a] = fp(acc[b], acc[a]) if commute else fp(acc[a], acc[b])
        mask <<= 1
    return acc[lroot]


def parse(stdout):
    rows = {}
    for ln in stdout.splitlines():
        k, *v = ln.split()
        rows.setdefault(k, []).append(v)
    return rows


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 8])
def test_plumbing_user_op(prog, n):
    r = run(n, prog, "cpu")
    assert r.returncode == 0, r.stderr
    rows = parse(r.stdout)
    assert sorted(int(v[0]) for v in rows["hello"]) == list(range(n))
    assert all(int(v[1]) == n and v[2] == "1" for v in rows["hello"])
    assert len(rows["bcast"]) == n * n
    for rank, root, x, bad in rows["bcast"]:
        assert int(x) == 4242 + int(root) and int(bad) == 0
    got = {(int(c), int(root)): v for c, root, *v in rows["ureduce"]}
    assert len(got) == 2 * n
    for (c, root), (rc, *vals) in got.items():
        assert int(rc) == 0
        for i in range(3):
            assert int(vals[i]) == binomial([val(q, i) for q in range(n)], root, bool(c)), (c, root, i)
    # MPI_ERR_ROOT, MPI_ERR_COMM, MPI_ERR_COUNT, MPI_ERR_OP (BYTE + SUM)
    assert rows["errs"][0] == ["7", "5", "2", "9"]


@pytest.mark.parametrize("n", [2, 4])
def test_mismatched_counts_error_not_hang(prog, n):
    """A collective whose counts differ across ranks returns an error on the
    receiving ranks instead of hanging (MPICH: MPIC_Recv MPI_ERR_TRUNCATE for a
    longer message, "**collective_size_mismatch" MPI_ERR_OTHER for a shorter
    one, bcast_intra_binomial.c:116-124), and the world stays usable."""
    r = run(n, prog, "mismatch", timeout=60)
    assert r.returncode == 0, r.stderr
    rows = {int(v[0]): [int(x) for x in v[1:]] for v in parse(r.stdout)["mismatch"]}
    assert sorted(rows) == list(range(n))
    children = {m for m in (1, 2, 4) if m < n}          # root 0's binomial children
    for rank, (long_, short, red, dropped, x) in rows.items():
        assert long_ == (14 if rank in children else 0), rank      # MPI_ERR_TRUNCATE
        assert short == (15 if rank in children else 0), rank      # MPI_ERR_OTHER
        assert dropped == 1 and x == 77
        # rank 1 sends 5 elements to rank 0 (its binomial parent), which expects 3
        assert red == (14 if rank == 0 else 0), rank


def test_cpi_np2_golden_cpu_only_rank():
    """cpi on ranks that see no GPU: every MPI_Reduce combine step is a host
    combine; the reference's golden line."""
    r = run(2, os.path.join(ROOT, "examples", "cpi"), env=NO_GPU)
    assert r.returncode == 0, r.stderr
    assert "pi is approximately 3.1415926544231318, Error is 0.0000000008333387" in r.stdout


@pytest.mark.parametrize("p", [2, 3, 5, 8])
def test_builtin_reduce_schedules_cpu_only_rank(prog, orc, mpi, p):
    """Builtin MPI_SUM MPI_Reduce of 1 and 4099 doubles on every root with no
    device visible: bit-identical to the oracle's step-by-step schedules."""
    from test_pip_runtime_gpu import check_builtin_reduce_rows
    r = run(p, prog, "gpu", timeout=300, env=NO_GPU)
    assert r.returncode == 0, r.stderr
    check_builtin_reduce_rows(parse(r.stdout), p, mpi)


def test_cpi_singleton_needs_no_reduction():
    # np = 1: MPI_Reduce over one rank is a local copy (golden: SURVEY.md §3.4)
    r = subprocess.run([os.path.join(ROOT, "examples", "cpi")], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "pi is approximately 3.1415926544231341," in r.stdout


def test_launcher_propagates_failure_and_timeout(tmp_path):
    r = run(3, "sh", "-c", 'if [ "$MPIR_PIP_RANK" = 1 ]; then exit 7; fi; exec sleep 30', timeout=60)
    assert r.returncode == 7
    r = subprocess.run([MPIEXEC, "-n", "2", "--timeout", "1", "sleep", "30"], capture_output=True, text=True,
                       timeout=30)
    assert r.returncode == 124 and "timeout" in r.stderr
    r = subprocess.run([MPIEXEC, "-n", "1", os.path.join(str(tmp_path), "missing")], capture_output=True,
                       text=True, timeout=30)
    assert r.returncode == 127

"""INTEGRATION.md Option 1, rehearsed without MPICH: the library's host sources
(mpich-pip_amd/Makefile DROPIN_SRC) compiled INTO a "libmpi" together with
unchanged-style schedule code (tests/progs/mock_libmpi.c), with
-fvisibility=hidden as MPICH's configure.ac:1443 builds libmpi, linked
against lib/libmpir_hip.so.  Checks that only the public API is exported,
that the schedules bind internally to MPIR_Reduce_local / MPIR_Op_table and
find user ops through the MPIR_Op object store, and that libmpi's strong
MPIR_Err_* routines replace the library's weak ones.  No GPU needed (host
buffers, user op)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mpich-pip_amd", "lib")


def _make_var(name):
    mk = open(os.path.join(ROOT, "mpich-pip_amd", "Makefile")).read()
    m = re.search(r"^%s\s*:=\s*(.+)$" % name, mk, re.M)
    return [os.path.join(ROOT, "mpich-pip_amd", s) for s in m.group(1).split()]


def dropin_sources():
    return _make_var("DROPIN_SRC")


@pytest.mark.parametrize("granularity", [1, 2, 3], ids=["GLOBAL", "POBJ", "VCI"])
def test_dropin_into_hidden_visibility_libmpi(tmp_path, granularity):
    """Option 1 at each of MPICH's thread granularities: DROPIN_SRC + DROPIN_GLUE
    built with -DMPIR_DROPIN_IN_LIBMPI against (a stand-in of) MPICH's mpiimpl.h.
    mock_app.c checks op_errno through an unchanged schedule and 8 threads of
    MPI_Op_create / MPI_Op_free racing a progress engine's inline releases."""
    so = str(tmp_path / "libmockmpi.so")
    inc = ["-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "mpich-pip_amd", "csrc", "host"),
           "-I" + os.path.join(ROOT, "tests", "progs", "mock_mpich"),
           "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__"]
    subprocess.run(["gcc", "-shared", "-fPIC", "-O2", "-std=gnu99", "-fvisibility=hidden", "-Wall",
                    "-DMPIR_DROPIN_IN_LIBMPI", "-DMOCK_GRANULARITY=%d" % granularity, *inc,
                    os.path.join(ROOT, "tests", "progs", "mock_libmpi.c"), *dropin_sources(),
                    *_make_var("DROPIN_GLUE"),
                    "-L" + LIB, "-lmpir_hip", "-Wl,-rpath," + LIB, "-lpthread", "-o", so], check=True)
    dyn = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in dyn.splitlines() if ln.strip()}
    for public in ("MPI_Reduce_local", "PMPI_Reduce_local", "MPI_Op_create", "MPI_Op_free", "MPI_Op_commutative",
                   "MPIX_Reduce_local_stream", "mock_sched_reduce"):
        assert public in exported, public
    for internal in ("MPIR_Reduce_local", "MPIR_Op_table", "MPIR_Op_direct", "MPIR_Op_mem", "MPIR_SUM",
                     "MPIR_Err_create_code", "MPIR_Err_return_comm", "MPIR_Op_errno_ptr", "MPIR_Dropin_cs_enter"):
        assert internal not in exported, internal
    app = str(tmp_path / "mock_app")
    subprocess.run(["gcc", "-std=gnu99", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "progs", "mock_app.c"), so, "-Wl,-rpath," + str(tmp_path),
                    "-ldl", "-lpthread", "-o", app], check=True)
    # no device visible: the host combine runs without one (CPU-only rank)
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1")
    r = subprocess.run([app], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mock libmpi ok" in r.stdout


def test_op_store_as_mpich_sees_it(tmp_path):
    """tests/progs/op_store.c: MPIR_Getb_ptr / add-ref / MPIR_Handle_obj_free
    restated as libmpi inlines them, against MPI_Op_create / MPI_Op_free."""
    exe = str(tmp_path / "op_store")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-pedantic",
                    "-I" + os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "progs", "op_store.c"),
                    "-o", exe, "-L" + LIB, "-lmpich_reduce_local", "-Wl,-rpath," + LIB], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "op_store ok" in r.stdout


def test_error_stack(mpi):
    """MPI_Reduce_local failures carry an MPICH-style error stack
    (reduce_local.c:208-217): the class via MPI_Error_class, the call and the
    cause via MPI_Error_string."""
    import numpy as np
    a = np.zeros(4, np.float32)
    b = np.zeros(4, np.float32)
    rc = mpi.reduce_local(a.ctypes.data, b.ctypes.data, 4, mpi.MPI_FLOAT, mpi.MPI_OP_NULL)
    assert rc != mpi.MPI_ERR_OP and mpi.error_class(rc) == mpi.MPI_ERR_OP
    s = mpi.error_string(rc)
    assert s.startswith("Invalid MPI_Op, error stack:"), s
    assert "MPI_Reduce_local(inbuf=0x" in s and "count=4, datatype=MPI_FLOAT, op=MPI_OP_NULL) failed" in s, s
    assert "Null MPI_Op" in s, s
    rc = mpi.reduce_local(a.ctypes.data, b.ctypes.data, 4, mpi.MPI_FLOAT, mpi.MPI_BAND)
    assert mpi.error_class(rc) == mpi.MPI_ERR_OP
    assert "MPI_Op MPI_BAND operation not defined for this datatype" in mpi.error_string(rc)


def test_preload_shim_replaces_only_the_public_entry(tmp_path):
    """INTEGRATION.md Option 2: LD_PRELOAD=lib/libmpich_reduce_local_preload.so
    in front of an installed, hidden-visibility libmpi
    (tests/progs/mock_installed_mpi.c).  The shim exports only
    MPI_Reduce_local / PMPI_Reduce_local; builtin ops take the drop-in path,
    user ops (libmpi's objects) go on to libmpi's PMPI_Reduce_local, and
    libmpi's internal schedules are not affected."""
    pre = os.path.join(LIB, "libmpich_reduce_local_preload.so")
    dyn = subprocess.run(["nm", "-D", "--defined-only", pre], capture_output=True, text=True, check=True).stdout
    assert {ln.split()[-1] for ln in dyn.splitlines() if ln.strip() and not ln.split()[-1].startswith("_")} == \
        {"MPI_Reduce_local", "PMPI_Reduce_local"}
    so = str(tmp_path / "libmpi.so")
    subprocess.run(["gcc", "-shared", "-fPIC", "-O2", "-fvisibility=hidden", "-Wall",
                    os.path.join(ROOT, "tests", "progs", "mock_installed_mpi.c"), "-o", so], check=True)
    app = str(tmp_path / "app")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", os.path.join(ROOT, "tests", "progs", "mock_preload_app.c"),
                    so, "-Wl,-rpath," + str(tmp_path), "-o", app], check=True)
    # prepend: whatever the environment already preloads stays preloaded
    env = dict(os.environ, LD_PRELOAD=" ".join(x for x in (pre, os.environ.get("LD_PRELOAD", "")) if x),
               MPIR_CVAR_REDUCE_LOCAL_ERRHANDLER="return")
    r = subprocess.run([app], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr
    assert "preload ok" in r.stdout

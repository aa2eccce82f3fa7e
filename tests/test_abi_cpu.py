"""C-ABI boundary checks that need no GPU (CPU only).

* the library loads and exports every function / table include/*.h declares;
* the check_dtype table agrees with the oracle for every (op, datatype);
* MPI_Reduce_local's validation block returns the reference's error classes
  (all of these return before any device work);
* user-defined ops (MPI_Op_create / free / commutative) on host buffers,
  including the reference's reduce_local.c non-commutative op test;
* the default MPI_ERRORS_ARE_FATAL handler aborts like the reference.
"""
import ctypes
import os
import re
import subprocess
import sys

import numpy as np
import pytest

import _types as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    names = set()
    for h in ("mpi_reduce_local.h", "mpir_hip_reduce.h", "mpix_hip_coll.h", "mpi_pip.h", "mpir_op_objects.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*(?:extern\s+)?[A-Za-z_][\w\s\*]*?\b((?:P?MPI[RX]?|MPI)_\w+)\s*(\(|\[)", src, re.M):
            if not src[m.start():m.end()].lstrip().startswith("#"):
                names.add(m.group(1))
    return sorted(n for n in names if not n.startswith("MPIR_OP_HDL"))


def test_library_exports_every_header_symbol(mpi):
    lib = mpi.load()
    declared = header_symbols()
    assert len(declared) >= 50
    missing = [n for n in declared if not hasattr(lib, n)]
    assert not missing, missing
    assert set(declared) <= set(mpi.EXPORTED_SYMBOLS) | set(declared)
    for n in mpi.EXPORTED_SYMBOLS:
        assert hasattr(lib, n), n


def test_op_table_layout(mpi):
    lib = mpi.load()
    table = (ctypes.c_void_p * 15).in_dll(lib, "MPIR_Op_table")
    chk = (ctypes.c_void_p * 15).in_dll(lib, "MPIR_Op_check_dtype_table")
    order = ["MPIR_MAXF", "MPIR_MINF", "MPIR_SUM", "MPIR_PROD", "MPIR_LAND", "MPIR_BAND", "MPIR_LOR",
             "MPIR_BOR", "MPIR_LXOR", "MPIR_BXOR", "MPIR_MINLOC", "MPIR_MAXLOC", "MPIR_REPLACE", "MPIR_NO_OP"]
    assert table[0] is None and chk[0] is None
    for i, name in enumerate(order, start=1):
        assert table[i] == ctypes.cast(getattr(lib, name), ctypes.c_void_p).value, name
        assert chk[i] == ctypes.cast(getattr(lib, name + "_check_dtype"), ctypes.c_void_p).value, name
    # op handle low nibble indexes the table (mpir_op.h:188)
    assert mpi.MPI_MAXLOC & 0xF == 12 and mpi.MPI_MINLOC & 0xF == 11


def test_check_dtype_matches_oracle(mpi, orc):
    lib = mpi.load()
    fns = {mpi.MPI_MAX: "MPIR_MAXF", mpi.MPI_MIN: "MPIR_MINF", mpi.MPI_SUM: "MPIR_SUM", mpi.MPI_PROD: "MPIR_PROD",
           mpi.MPI_LAND: "MPIR_LAND", mpi.MPI_BAND: "MPIR_BAND", mpi.MPI_LOR: "MPIR_LOR", mpi.MPI_BOR: "MPIR_BOR",
           mpi.MPI_LXOR: "MPIR_LXOR", mpi.MPI_BXOR: "MPIR_BXOR", mpi.MPI_MINLOC: "MPIR_MINLOC",
           mpi.MPI_MAXLOC: "MPIR_MAXLOC"}
    types = list(mpi.DATATYPES.values()) + [mpi.MPI_DATATYPE_NULL, 0x4C00100C, 0x12345678]
    for op, fname in fns.items():
        f = getattr(lib, fname + "_check_dtype")
        for dt in types:
            assert f(dt) == orc.check_dtype(op, dt), (fname, hex(dt))
    assert lib.MPIR_REPLACE_check_dtype(0x12345678) == 0
    assert lib.MPIR_NO_OP_check_dtype(mpi.MPI_FLOAT) == 0


def test_has_kernel_for_every_compute_pair(mpi):
    """Every (op, type) the reference computes has a gfx950 kernel."""
    lib = mpi.load()
    nelems = next(e for e in range(1, 256) if lib.MPIR_Hip_elem_size(e) == 0)
    elem_of = {}
    for t in T.ALL_TYPES:
        for op in T.OPS:
            if T.compute_ok(op, t):
                opidx = mpi.OPS[op] & 0xF
                # resolve through the same path the op kernels use: a kernel must exist
                found = any(lib.MPIR_Hip_has_kernel(opidx, e) and lib.MPIR_Hip_elem_size(e) == T.elem_size(t)
                            for e in range(1, nelems))
                assert found, (op, t)
        elem_of[t] = T.elem_size(t)
    assert nelems == 22
    for e in range(1, nelems):
        assert lib.MPIR_Hip_elem_size(e) in (1, 2, 4, 8, 16, 32)


@pytest.mark.parametrize("op,dt,count,same,expect", [
    ("MPI_OP_NULL", "MPI_FLOAT", 4, False, 9),
    ("MPI_NO_OP", "MPI_FLOAT", 4, False, 9),
    ("MPI_REPLACE", "MPI_FLOAT", 4, False, 9),
    ("BAD_HANDLE", "MPI_FLOAT", 4, False, 9),
    ("BUILTIN_IDX0", "MPI_FLOAT", 4, False, 9),
    ("MPI_BAND", "MPI_FLOAT", 4, False, 9),
    ("MPI_SUM", "MPI_BYTE", 4, False, 9),
    ("MPI_MAXLOC", "MPI_INT", 4, False, 9),
    ("MPI_MAX", "MPI_C_FLOAT_COMPLEX", 4, False, 9),
    ("MPI_SUM", "MPI_DATATYPE_NULL", 4, False, 9),
    ("MPI_SUM", "MPI_FLOAT", 4, True, 1),          # aliased buffers
    ("MPI_SUM", "MPI_FLOAT", 0, True, 0),          # count 0: no alias check, no work
    ("MPI_SUM", "MPI_FLOAT", 0, False, 0),
    ("MPI_SUM", "MPI_FLOAT", -5, False, 0),        # count < 0 is not validated; loop runs 0 times
])
def test_reduce_local_validation(mpi, op, dt, count, same, expect):
    handles = dict(mpi.OPS, MPI_OP_NULL=mpi.MPI_OP_NULL, MPI_NO_OP=mpi.MPI_NO_OP, MPI_REPLACE=mpi.MPI_REPLACE,
                   BAD_HANDLE=0x44000003, BUILTIN_IDX0=0x58000000)
    d = mpi.MPI_DATATYPE_NULL if dt == "MPI_DATATYPE_NULL" else mpi.DATATYPES[dt]
    a = np.zeros(8, dtype=np.float64)
    b = a if same else np.zeros(8, dtype=np.float64)
    rc = mpi.reduce_local(a.ctypes.data, b.ctypes.data, count, d, handles[op])
    assert mpi.error_class(rc) == expect
    if rc:
        assert "Invalid" in mpi.error_string(rc) or "buffer" in mpi.error_string(rc).lower()


def test_in_place_rejected(mpi):
    a = np.zeros(4, dtype=np.float32)
    IN_PLACE = ctypes.c_void_p(-1 & 0xFFFFFFFFFFFFFFFF).value
    assert mpi.error_class(mpi.reduce_local(IN_PLACE, a.ctypes.data, 4, mpi.MPI_FLOAT, mpi.MPI_SUM)) == mpi.MPI_ERR_BUFFER
    assert mpi.error_class(mpi.reduce_local(a.ctypes.data, IN_PLACE, 4, mpi.MPI_FLOAT, mpi.MPI_SUM)) == mpi.MPI_ERR_BUFFER
    assert mpi.reduce_local(IN_PLACE, a.ctypes.data, 0, mpi.MPI_FLOAT, mpi.MPI_SUM) == 0


def test_multi_overlap_refused_before_any_device_work(mpi):
    """MPIX_Reduce_local_multi refuses an outbuf overlapping any operand but
    inbufs[0]-exactly, before it looks at residency (no GPU needed)."""
    a = np.zeros(64, dtype=np.float32)
    b = np.zeros(64, dtype=np.float32)
    p = [a.ctypes.data, b.ctypes.data]
    for out in (b.ctypes.data, b.ctypes.data + 8, a.ctypes.data + 4, b.ctypes.data - 4):
        rc = mpi.reduce_local_multi(p, out, 64, mpi.MPI_FLOAT, mpi.MPI_SUM, mpi.MPIX_ORDER_CHAIN)
        msg = mpi.error_string(rc)
        assert mpi.error_class(rc) == mpi.MPI_ERR_BUFFER and ("overlaps outbuf" in msg or "aliased" in msg)
    # exactly operand 0 passes the check (then host operands are refused as non-device)
    rc = mpi.reduce_local_multi(p, a.ctypes.data, 64, mpi.MPI_FLOAT, mpi.MPI_SUM, mpi.MPIX_ORDER_CHAIN)
    assert mpi.error_class(rc) == mpi.MPI_ERR_BUFFER and "overlaps" not in mpi.error_string(rc)


def test_user_op_noncommutative_host(mpi):
    """test/mpi/coll/reduce_local.c: a non-commutative user op via MPI_Reduce_local
    (with the inout check the reference test forgot to reach)."""
    lib = mpi.load()
    calls = []

    @mpi.MPI_User_function
    def user_op(invec, inoutvec, lenp, dtp):
        n = lenp[0]
        a = np.ctypeslib.as_array(ctypes.cast(invec, ctypes.POINTER(ctypes.c_int)), (n,))
        b = np.ctypeslib.as_array(ctypes.cast(inoutvec, ctypes.POINTER(ctypes.c_int)), (n,))
        calls.append((n, dtp[0]))
        b[:] = 2 * b + a     # non-commutative: inout = 2*inout + in

    op = ctypes.c_int(0)
    assert lib.MPI_Op_create(user_op, 0, ctypes.byref(op)) == 0
    assert op.value & 0xFC000000 == 0x98000000          # DIRECT kind, MPI kind OP
    flag = ctypes.c_int(-1)
    assert lib.MPI_Op_commutative(op.value, ctypes.byref(flag)) == 0 and flag.value == 0
    assert lib.MPIR_Op_is_commutative(op.value) == 0
    for count in [0, 1, 2, 4, 8, 32768]:
        inb = np.arange(count, dtype=np.int32)
        io = 3 * np.arange(count, dtype=np.int32)
        rc = mpi.reduce_local(inb.ctypes.data, io.ctypes.data, count, mpi.MPI_INT, op.value)
        assert rc == 0
        assert np.array_equal(io, 7 * np.arange(count, dtype=np.int32))
    assert calls and all(c[1] == mpi.MPI_INT for c in calls) and (0, mpi.MPI_INT) not in calls
    assert lib.MPI_Op_free(ctypes.byref(op)) == 0 and op.value == mpi.MPI_OP_NULL
    # freeing a builtin op is an error (op_free.c "**permop")
    b = ctypes.c_int(mpi.MPI_SUM)
    assert mpi.error_class(lib.MPI_Op_free(ctypes.byref(b))) == mpi.MPI_ERR_OP
    # a freed user op is an invalid handle
    assert mpi.error_class(mpi.reduce_local(inb.ctypes.data, io.ctypes.data, 2, mpi.MPI_INT, 0x98000000)) == mpi.MPI_ERR_OP


def test_user_op_commutative_flag(mpi):
    lib = mpi.load()

    @mpi.MPI_User_function
    def noop(a, b, n, d):
        pass

    ops = []
    for i in range(20):            # past the 16 direct handles -> indirect handles
        o = ctypes.c_int(0)
        assert lib.MPI_Op_create(noop, 1, ctypes.byref(o)) == 0
        ops.append(o)
    kinds = {(o.value & 0xFFFFFFFF) >> 30 for o in ops}
    assert kinds <= {2, 3}
    for o in ops:
        f = ctypes.c_int(-1)
        assert lib.MPI_Op_commutative(o.value, ctypes.byref(f)) == 0 and f.value == 1
    for o in ops:
        assert lib.MPI_Op_free(ctypes.byref(o)) == 0
    f = ctypes.c_int(0)
    assert lib.MPI_Op_commutative(mpi.MPI_SUM, ctypes.byref(f)) == 0 and f.value == 1


def test_errors_are_fatal_by_default():
    code = (
        "import sys; sys.path.insert(0, %r); import mpich_pip_amd as m, numpy as np; "
        "a = np.zeros(4, np.float32); m.reduce_local(a.ctypes.data, a.ctypes.data, 4, m.MPI_FLOAT, m.MPI_SUM); "
        "print('NOT REACHED')" % os.path.join(ROOT, "mpich-pip_amd"))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == 1
    assert "Fatal error in PMPI_Reduce_local" in p.stderr
    assert "NOT REACHED" not in p.stdout


def test_error_class_and_string(mpi):
    lib = mpi.load()
    c = ctypes.c_int(-1)
    assert lib.MPI_Error_class(mpi.MPI_ERR_OP, ctypes.byref(c)) == 0 and c.value == mpi.MPI_ERR_OP
    assert mpi.error_string(0) == "No MPI error"


@pytest.mark.parametrize("compiler", [["gcc", "-std=c99", "-pedantic"], ["g++", "-std=c++17", "-x", "c++"]],
                         ids=["c99", "c++17"])
def test_public_headers_compile_and_link(mpi, tmp_path, compiler):
    """include/*.h are self-contained C99 and C++; the entry points have the
    reference prototypes; a program using them links against the library."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "mpich-pip_amd", "lib")
    exe = str(tmp_path / "abi_link")
    subprocess.run([*compiler, "-Wall", "-Wextra", "-Werror", "-I" + os.path.join(root, "include"),
                    os.path.join(root, "tests", "progs", "abi_link.c"), "-o", exe, "-L" + lib,
                    "-lmpich_reduce_local", "-Wl,-rpath," + lib], check=True)
    assert subprocess.run([exe]).returncode == 0


def test_fastcall_binding_same_library_and_errors(mpi):
    """The compiled CPython binding bench.py times MPI_Reduce_local through
    (csrc/py/fastcall.c) calls the same library instance as ctypes: the
    validation classes match call for call (no device work on these paths)."""
    f = mpi.fast_reduce_local()
    a = np.zeros(4, np.float32)
    b = np.zeros(4, np.float32)
    cases = [
        (b.ctypes.data, a.ctypes.data, 4, mpi.MPI_FLOAT, mpi.MPI_BAND),      # op/type mismatch
        (a.ctypes.data, a.ctypes.data, 4, mpi.MPI_FLOAT, mpi.MPI_SUM),       # alias
        (b.ctypes.data, a.ctypes.data, 0, mpi.MPI_FLOAT, mpi.MPI_SUM),       # count 0
        (b.ctypes.data, a.ctypes.data, 4, mpi.MPI_FLOAT, mpi.MPI_OP_NULL),   # null op
    ]
    for c in cases:
        assert mpi.error_class(f(*c)) == mpi.error_class(mpi.reduce_local(*c)), c
    with pytest.raises(OverflowError):
        f(0, 0, 1 << 40, mpi.MPI_FLOAT, mpi.MPI_SUM)
    with pytest.raises(TypeError):
        f(0, 0, 1)

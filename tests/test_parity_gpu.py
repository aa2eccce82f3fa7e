"""GPU parity: the gfx950 MPI_Reduce_local against the CPU oracle (MI355X).

Every call goes through the C ABI (MPI_Reduce_local / MPIX_Reduce_local_stream
in libmpich_reduce_local.so) with device buffers allocated by torch (plumbing
only).  The bar is bit-exact for every op and type -- each element is one
IEEE round-to-nearest-even operation on both sides (SURVEY.md §8c
'Tolerance') -- so outputs are compared as bytes.
"""
import ctypes
import json
import os
import time

import numpy as np
import pytest

import _types as T

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


class host_max:
    """Set MPIR_Hip_set_host_max_bytes for a block (0 = both-host calls take the
    GPU staging pipeline instead of the host combine), restoring it after."""

    def __init__(self, mpi, nbytes):
        self.lib, self.nbytes = mpi.load(), nbytes

    def __enter__(self):
        self.lib.MPIR_Hip_set_host_max_bytes.restype = ctypes.c_uint64
        self.lib.MPIR_Hip_set_host_max_bytes.argtypes = [ctypes.c_uint64]
        self.prev = self.lib.MPIR_Hip_set_host_max_bytes(self.nbytes)
        return self

    def __exit__(self, *exc):
        self.lib.MPIR_Hip_set_host_max_bytes(self.prev)
        return False


def dev(torch, host_bytes: np.ndarray, offset: int = 0):
    """Copy bytes to a fresh device allocation at `offset`; returns (tensor, address)."""
    n = host_bytes.size
    t = torch.zeros(n + offset + 256, dtype=torch.uint8, device="cuda")
    if n:
        t[offset:offset + n].copy_(torch.from_numpy(np.ascontiguousarray(host_bytes)))
    torch.cuda.synchronize()
    return t, t.data_ptr() + offset


def back(t, offset, n):
    import torch
    torch.cuda.synchronize()
    return t[offset:offset + n].cpu().numpy()


def explain(got, want, a, b, esz, limit=6):
    g = got.reshape(-1, esz)
    w = want.reshape(-1, esz)
    bad = np.nonzero((g != w).any(axis=1))[0]
    lines = [f"{bad.size} of {g.shape[0]} elements differ"]
    for i in bad[:limit]:
        lines.append(f"  [{i}] inout={a.reshape(-1, esz)[i].tobytes()[::-1].hex()} in={b.reshape(-1, esz)[i].tobytes()[::-1].hex()}"
                     f" gpu={g[i].tobytes()[::-1].hex()} oracle={w[i].tobytes()[::-1].hex()}")
    return "\n".join(lines)


def same(got: np.ndarray, want: np.ndarray, t: str) -> bool:
    """Bit-exact, except the NaN payload/sign of C _Complex results: C leaves the
    payload of a NaN result to codegen, and gcc -O2 orders the complex
    component operations differently depending on the surrounding switch
    (probed: standalone `a[i] + b[i]` puts a.im first, the same loop inside the
    op switch puts b.im first), so it is not a property of the reference.
    Non-NaN complex components (infinities of the Annex G recovery included)
    stay bit-exact; real types are bit-exact including NaN payloads."""
    if np.array_equal(got, want):
        return True
    if t not in T.CPLX:
        return False
    if t == "MPI_C_LONG_DOUBLE_COMPLEX":
        g, w = got.view(T.CX80), want.view(T.CX80)
        ok = True
        for part in ("re", "im"):
            gp, wp = g[part], w[part]
            value_eq = (gp["m"] == wp["m"]) & (gp["se"] == wp["se"])
            ok &= bool(((value_eq | (T.x80_nanish(gp) & T.x80_nanish(wp))) & (gp["pad"] == wp["pad"])).all())
        return ok
    ft = np.float32 if t == "MPI_C_FLOAT_COMPLEX" else np.float64
    ut = np.uint32 if ft == np.float32 else np.uint64
    g = got.view(ft)
    w = want.view(ft)
    ok = (got.view(ut) == want.view(ut)) | (np.isnan(g) & np.isnan(w))
    return bool(ok.all())


def run_pair(mpi, orc, torch, op, t, n, seed, off_in=0, off_io=0):
    rng = np.random.default_rng(seed)
    a = T.to_bytes(T.gen(t, n, rng, op))          # inout
    b = T.to_bytes(T.gen(t, n, rng, op))          # in
    want = a.copy()
    rc_o = orc.reduce_local(b.copy(), want, n, mpi.DATATYPES[t], mpi.OPS[op])
    tio, pio = dev(torch, a, off_io)
    tin, pin = dev(torch, b, off_in)
    rc = mpi.reduce_local(pin, pio, n, mpi.DATATYPES[t], mpi.OPS[op])
    got = back(tio, off_io, a.size)
    assert mpi.error_class(rc) == rc_o, (op, t, rc, rc_o)
    assert np.array_equal(back(tin, off_in, b.size), b), "inbuf modified"
    if not same(got, want, t):
        pytest.fail(f"{op} {t} n={n} off=({off_in},{off_io}):\n" + explain(got, want, a, b, T.elem_size(t)))


MATRIX = [(op, t) for op in T.OPS for t in T.ALL_TYPES if T.check_ok(op, t)]


@pytest.mark.parametrize("op,t", MATRIX, ids=[f"{o}-{t}" for o, t in MATRIX])
def test_matrix_vs_oracle(mpi, orc, cuda, op, t):
    """Every (op, type) the reference accepts, edge values included, ragged counts."""
    for n, seed in ((1, 1), (7, 2), (1000, 3), (65536 + 13, 4)):
        run_pair(mpi, orc, cuda, op, t, n, seed)


@pytest.mark.parametrize("t", ["MPI_FLOAT", "MPI_UNSIGNED_CHAR", "MPIX_C_FLOAT16", "MPI_DOUBLE",
                               "MPI_C_DOUBLE_COMPLEX", "MPI_SHORT_INT", "MPI_LONG_INT"])
def test_alignment_offsets(mpi, orc, cuda, t):
    """Sub-range displacements: equal and unequal misalignment of in / inout mod 16."""
    op = "MPI_MAXLOC" if t in T.PAIRS else "MPI_SUM"
    esz = T.elem_size(t)
    for off_in, off_io in ((0, 0), (esz, esz), (esz, 0), (0, 3 * esz), (8, 8), (4, 12), (1, 1), (3, 5)):
        for n in (1, 5, 33, 4099):
            run_pair(mpi, orc, cuda, op, t, n, 100 + n + off_in, off_in, off_io)


SHIFT_CASES = [("MPI_SUM", "MPI_FLOAT"), ("MPI_MAX", "MPI_DOUBLE"), ("MPI_SUM", "MPIX_C_FLOAT16"),
               ("MPI_BXOR", "MPI_UNSIGNED_CHAR"), ("MPI_PROD", "MPI_INT64_T"), ("MPI_SUM", "MPI_C_FLOAT_COMPLEX"),
               ("MPI_MINLOC", "MPI_DOUBLE_INT"), ("MPI_SUM", "MPI_LONG_DOUBLE"), ("MPI_LXOR", "MPI_SHORT")]


@pytest.mark.parametrize("op,t", SHIFT_CASES, ids=[f"{o}-{t}" for o, t in SHIFT_CASES])
def test_relative_misalignment_tile_path(mpi, orc, cuda, op, t):
    """Counts of several tiles with inbuf at every offset mod 16 relative to
    inoutbuf: the aligned-load + wavefront-shuffle + funnel kernel
    (k_reduce_shift), its head / tail elements and ragged last tile."""
    esz = T.elem_size(t)
    n = (3 * 16384 + 37 * 16) // esz + 3
    for off_io in (0, esz, 16 - esz if esz < 16 else 0):
        for off_in in range(0, 16):
            if (off_in - off_io) % 16 == 0:
                continue
            run_pair(mpi, orc, cuda, op, t, n, 7 * off_in + off_io, off_in, off_io)


def test_golden_kat_fold_on_gpu(mpi, cuda):
    """The reference's own known-answer tests, folded on the GPU, bit for bit."""
    torch = cuda
    man = json.load(open(os.path.join(GOLD, "kat_reference.json")))["cases"]
    data = np.load(os.path.join(GOLD, "kat_reference.npz"))
    bad = []
    for c in man:
        ranks = data[c["key"] + "_ranks"]
        sol = data[c["key"] + "_sol"]
        dr = torch.from_numpy(ranks.copy()).cuda()
        acc = dr[0].clone()
        for r in range(1, c["p"]):
            rc = mpi.reduce_local(dr[r].data_ptr(), acc.data_ptr(), c["count"], c["handle"], c["op_handle"])
            assert rc == 0, c["id"]
        if not np.array_equal(acc.cpu().numpy(), sol):
            bad.append(c["id"])
    assert not bad, f"{len(bad)} of {len(man)} KAT cases differ, e.g. {bad[:6]}"


def test_survey_probes_on_gpu(mpi, cuda):
    torch = cuda
    for c in json.load(open(os.path.join(GOLD, "probe_survey.json")))["cases"]:
        w = c["width"]
        dt = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[w]
        io = np.array(c["inout"], dtype=dt)
        src = np.array(c["in"], dtype=dt)
        tio, pio = dev(torch, io.view(np.uint8))
        tin, pin = dev(torch, src.view(np.uint8))
        rc = mpi.reduce_local(pin, pio, len(io), mpi.DATATYPES[c["datatype"]], mpi.OPS[c["op"]])
        got = back(tio, 0, io.nbytes).view(dt)
        assert mpi.error_class(rc) == c.get("expect_rc", 0), c["id"]
        assert [int(x) for x in got] == c["expect"], c["id"]


@pytest.mark.parametrize("staged", [False, True], ids=["dispatch", "staged"])
@pytest.mark.parametrize("where", ["host-host", "host-dev", "dev-host", "pinned-pinned", "pinned-dev",
                                   "host-pinned", "pinned-host", "hostoff-hostoff"])
def test_host_and_mixed_pointers(mpi, orc, cuda, where, staged):
    """Rank buffers that arrive in host memory (PiP shm): with the default
    dispatch, both-host calls run the host combine and mixed ones the pinned
    slot (<= 1 MiB) or the staging pipeline; `staged` forces every both-host
    call through the GPU staging pipeline too (MPIR_Hip_set_host_max_bytes(0)):
    pageable operands through the pinned bounce slots (several chunks per call at
    the 192 MiB size, so slots are reused), pinned ones DMA'd directly.
    `hostoff` is a pageable buffer 4 bytes past 64 B alignment."""
    with host_max(mpi, 0 if staged else (1 << 64) - 1):
        _host_and_mixed_pointers(mpi, orc, cuda, where)


def _host_and_mixed_pointers(mpi, orc, cuda, where):
    torch = cuda
    for n, t, op in ((1000, "MPI_FLOAT", "MPI_SUM"), (3 * (16 << 20) + 5, "MPI_INT", "MPI_MAX"),
                     (777, "MPI_DOUBLE_INT", "MPI_MINLOC"), ((9 << 20) + 3, "MPI_DOUBLE", "MPI_SUM")):
        rng = np.random.default_rng(n)
        a = T.to_bytes(T.gen(t, n, rng, op))
        b = T.to_bytes(T.gen(t, n, rng, op))
        want = a.copy()
        assert orc.reduce_local(b.copy(), want, n, mpi.DATATYPES[t], mpi.OPS[op]) == 0
        src_kind, dst_kind = where.split("-")

        def make(x, kind):
            if kind == "dev":
                tt, p = dev(torch, x)
                return tt, p
            if kind == "pinned":
                tt = torch.from_numpy(x.copy()).pin_memory()
                return tt, tt.data_ptr()
            if kind == "hostoff":
                raw = np.zeros(x.size + 64 + 4, np.uint8)
                o = (-raw.ctypes.data) % 64 + 4
                h = raw[o:o + x.size]
                h[:] = x
                return h, h.ctypes.data
            h = x.copy()
            return h, h.ctypes.data

        tin, pin = make(b, src_kind)
        tio, pio = make(a, dst_kind)
        assert mpi.reduce_local(pin, pio, n, mpi.DATATYPES[t], mpi.OPS[op]) == 0
        torch.cuda.synchronize()
        got = tio.cpu().numpy()[:a.size] if hasattr(tio, "cpu") else tio
        assert np.array_equal(got, want), (where, t, op)


def test_stream_variant(mpi, orc, cuda):
    torch = cuda
    n = (1 << 20) + 3
    rng = np.random.default_rng(11)
    a = T.to_bytes(T.gen("MPI_FLOAT", n, rng))
    b = T.to_bytes(T.gen("MPI_FLOAT", n, rng))
    want = a.copy()
    orc.reduce_local(b.copy(), want, n, mpi.MPI_FLOAT, mpi.MPI_SUM)
    tio, pio = dev(torch, a)
    tin, pin = dev(torch, b)
    s = torch.cuda.Stream()
    assert mpi.reduce_local_stream(pin, pio, n, mpi.MPI_FLOAT, mpi.MPI_SUM, s.cuda_stream) == 0
    s.synchronize()
    assert np.array_equal(back(tio, 0, a.size), want)
    # host pointers are refused by the stream variant
    h = np.zeros(16, np.float32)
    assert mpi.error_class(mpi.reduce_local_stream(h.ctypes.data, pio, 4, mpi.MPI_FLOAT, mpi.MPI_SUM, 0)) == \
        mpi.MPI_ERR_BUFFER
    # float LAND passes check_dtype then fails in the compute switch (op_errno)
    assert mpi.error_class(mpi.reduce_local_stream(pin, pio, 4, mpi.MPI_FLOAT, mpi.MPI_LAND, 0)) == mpi.MPI_ERR_OP


def test_stream_variant_in_hip_graph(mpi, orc, cuda):
    """MPIX_Reduce_local_stream is capturable: a schedule's combine steps can be
    recorded once into a HIP graph and replayed.  Three steps (aligned, relatively
    misaligned, int MAX) captured, the graph replayed twice; the result is six
    reductions, checked against the oracle applying the same six."""
    torch = cuda
    n = 70001
    rng = np.random.default_rng(5)
    a = T.to_bytes(T.gen("MPI_FLOAT", n, rng, specials=False))
    b = T.to_bytes(T.gen("MPI_FLOAT", n, rng, specials=False))
    ia = T.to_bytes(T.gen("MPI_INT", n, rng))
    ib = T.to_bytes(T.gen("MPI_INT", n, rng))
    tio, pio = dev(torch, a)
    tin, pin = dev(torch, b)
    tmis, pmis = dev(torch, b, 4)          # inbuf 4 bytes off inoutbuf mod 16
    tia, pia = dev(torch, ia)
    tib, pib = dev(torch, ib)
    want, iwant = a.copy(), ia.copy()
    for _ in range(2):
        orc.reduce_local(b.copy(), want, n, mpi.MPI_FLOAT, mpi.MPI_SUM)
        orc.reduce_local(b.copy(), want, n, mpi.MPI_FLOAT, mpi.MPI_SUM)
        orc.reduce_local(ib.copy(), iwant, n, mpi.MPI_INT, mpi.MPI_MAX)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            cs = torch.cuda.current_stream().cuda_stream
            assert mpi.reduce_local_stream(pin, pio, n, mpi.MPI_FLOAT, mpi.MPI_SUM, cs) == 0
            assert mpi.reduce_local_stream(pmis, pio, n, mpi.MPI_FLOAT, mpi.MPI_SUM, cs) == 0
            assert mpi.reduce_local_stream(pib, pia, n, mpi.MPI_INT, mpi.MPI_MAX, cs) == 0
    torch.cuda.synchronize()
    # capture records, it does not run: the operands are still the inputs
    assert np.array_equal(back(tio, 0, a.size), a)
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(back(tio, 0, a.size), want)
    assert np.array_equal(back(tia, 0, ia.size), iwant)


def test_user_op_on_device_buffers(mpi, cuda):
    torch = cuda
    lib = mpi.load()

    @mpi.MPI_User_function
    def user_op(invec, inoutvec, lenp, dtp):
        n = lenp[0]
        a = np.ctypeslib.as_array(ctypes.cast(invec, ctypes.POINTER(ctypes.c_int)), (n,))
        b = np.ctypeslib.as_array(ctypes.cast(inoutvec, ctypes.POINTER(ctypes.c_int)), (n,))
        b[:] = 2 * b + a

    op = ctypes.c_int(0)
    assert lib.MPI_Op_create(user_op, 0, ctypes.byref(op)) == 0
    n = 4096
    inb = torch.arange(n, dtype=torch.int32, device="cuda")
    io = 3 * torch.arange(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    assert mpi.reduce_local(inb.data_ptr(), io.data_ptr(), n, mpi.MPI_INT, op.value) == 0
    assert torch.equal(io.cpu(), 7 * torch.arange(n, dtype=torch.int32))
    assert lib.MPI_Op_free(ctypes.byref(op)) == 0


def test_reference_reduce_local_program(mpi, cuda):
    """The reference's own MPI_Reduce_local test (test/mpi/coll/reduce_local.c:
    MPI_INT with MPI_SUM, then a non-commutative user op, counts 0, 1, 2, 4, ...,
    32768, inbuf[i] = inoutbuf[i] = i) on device buffers.  Its result check is
    nested inside the inbuf check (reduce_local.c:63-65, 80-82), so
    here both buffers are checked: inbuf unchanged, inoutbuf = 2i for SUM and
    the user op's value for every element."""
    torch = cuda
    lib = mpi.load()

    @mpi.MPI_User_function
    def user_op(invec, inoutvec, lenp, dtp):
        n = lenp[0]
        a = np.ctypeslib.as_array(ctypes.cast(invec, ctypes.POINTER(ctypes.c_int)), (n,))
        b = np.ctypeslib.as_array(ctypes.cast(inoutvec, ctypes.POINTER(ctypes.c_int)), (n,))
        b[:] = a - 3 * b          # non-commutative: f(a, b) != f(b, a)

    uop = ctypes.c_int(0)
    assert lib.MPI_Op_create(user_op, 0, ctypes.byref(uop)) == 0
    counts = [0] + [1 << k for k in range(16)]
    for count in counts:
        ref = torch.arange(count, dtype=torch.int32, device="cuda")
        for op, want in ((mpi.MPI_SUM, 2 * ref), (uop.value, ref - 3 * ref)):
            inb = ref.clone()
            io = ref.clone()
            torch.cuda.synchronize()
            assert mpi.reduce_local(inb.data_ptr(), io.data_ptr(), count, mpi.MPI_INT, op) == 0, count
            assert torch.equal(inb, ref), ("inbuf modified", count)
            assert torch.equal(io, want), ("inoutbuf", count, op)
    assert lib.MPI_Op_free(ctypes.byref(uop)) == 0


@pytest.mark.parametrize("op", ["MPI_SUM", "MPI_MAX", "MPI_MIN", "MPI_PROD"])
@pytest.mark.parametrize("t", ["MPI_INT", "MPI_INT64_T", "MPI_FLOAT", "MPI_DOUBLE"])
def test_config3_sweep_256mib(mpi, orc, cuda, op, t):
    """BASELINE config 3: {SUM,MAX,MIN,PROD} x {int32,int64,fp32,fp64} at 256 MiB per operand,
    compared with the oracle over the full buffer."""
    torch = cuda
    esz = T.elem_size(t)
    n = (256 << 20) // esz
    rng = np.random.default_rng(2024)
    a = T.to_bytes(T.gen(t, n, rng, op))
    b = T.to_bytes(T.gen(t, n, rng, op))
    tio, pio = dev(torch, a)
    tin, pin = dev(torch, b)
    assert mpi.reduce_local(pin, pio, n, mpi.DATATYPES[t], mpi.OPS[op]) == 0
    got = back(tio, 0, a.size)
    del tio, tin
    assert orc.reduce_local(b, a, n, mpi.DATATYPES[t], mpi.OPS[op]) == 0
    if not np.array_equal(got, a):
        pytest.fail(explain(got, a, a, b, esz))


def test_config2_64mib_repeat_idempotence(mpi, cuda):
    """BASELINE config 2 (fp32 SUM, 64 MiB): size-independent properties --
    x + 0 == x bitwise, and 2 accumulations of b equal oracle-free torch adds."""
    torch = cuda
    n = (64 << 20) // 4
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.rand(n, device="cuda", generator=g) * 2 - 1
    z = torch.zeros(n, device="cuda")
    x0 = x.clone()
    torch.cuda.synchronize()
    assert mpi.reduce_local(z.data_ptr(), x.data_ptr(), n, mpi.MPI_FLOAT, mpi.MPI_SUM) == 0
    assert torch.equal(x.view(torch.int32), x0.view(torch.int32))
    y = torch.rand(n, device="cuda", generator=g)
    ref = x0 + y + y          # IEEE fp32 adds in the same order
    torch.cuda.synchronize()
    for _ in range(2):
        assert mpi.reduce_local(y.data_ptr(), x.data_ptr(), n, mpi.MPI_FLOAT, mpi.MPI_SUM) == 0
    assert torch.equal(x.view(torch.int32), ref.view(torch.int32))


def _pairs(specials, ut):
    v = np.array(specials, dtype=ut)
    return np.repeat(v, len(v)), np.tile(v, len(v))


@pytest.mark.parametrize("op", ["MPI_SUM", "MPI_PROD", "MPI_MAX", "MPI_MIN", "MPI_LXOR"])
@pytest.mark.parametrize("t", ["MPI_FLOAT", "MPI_DOUBLE", "MPIX_C_FLOAT16"])
def test_nan_inf_zero_pairs(mpi, orc, cuda, op, t):
    """Every pairing of NaN (quiet/signalling, both signs, payloads), +-inf, +-0,
    denormals and extremes: NaN payload propagation and the default NaN of
    invalid operations (inf - inf, 0 * inf) must match the reference bit for bit."""
    ut, sp = {"MPI_FLOAT": (np.uint32, T.F32_SPECIALS), "MPI_DOUBLE": (np.uint64, T.F64_SPECIALS),
              "MPIX_C_FLOAT16": (np.uint16, T.F16_SPECIALS)}[t]
    a, b = _pairs(sp, ut)
    want = a.copy()
    assert orc.reduce_local(b.copy(), want, len(a), mpi.DATATYPES[t], mpi.OPS[op]) == 0
    tio, pio = dev(cuda, a.view(np.uint8))
    tin, pin = dev(cuda, b.view(np.uint8))
    assert mpi.reduce_local(pin, pio, len(a), mpi.DATATYPES[t], mpi.OPS[op]) == 0
    got = back(tio, 0, a.nbytes)
    if not np.array_equal(got, want.view(np.uint8)):
        pytest.fail(f"{op} {t}:\n" + explain(got, want.view(np.uint8), a.view(np.uint8), b.view(np.uint8),
                                             np.dtype(ut).itemsize, limit=40))


@pytest.mark.parametrize("op", ["MPI_SUM", "MPI_PROD"])
@pytest.mark.parametrize("t", ["MPI_C_FLOAT_COMPLEX", "MPI_C_DOUBLE_COMPLEX"])
def test_complex_special_pairs(mpi, orc, cuda, op, t):
    """C99 Annex G complex multiply (NaN recovery branch) and component sums over
    special real/imaginary parts."""
    ft = np.float32 if t == "MPI_C_FLOAT_COMPLEX" else np.float64
    vals = np.array([np.nan, np.nan, np.nan, np.inf, -np.inf, 0.0, -0.0, 1.5, -2.0,
                     3e38 if ft == np.float32 else 1e308], dtype=ft)
    ut = np.uint32 if ft == np.float32 else np.uint64
    bits = vals.view(ut)          # NaNs with distinct payloads / sign
    bits[1] = 0xFFC00000 if ft == np.float32 else 0xFFF8000000000000
    bits[2] = 0x7FC00123 if ft == np.float32 else 0x7FF8000000000123
    z = (vals[:, None] + 0j * vals[None, :]).astype(np.complex64 if ft == np.float32 else np.complex128)
    z.real = np.repeat(vals, len(vals)).reshape(len(vals), len(vals))
    z.imag = np.tile(vals, len(vals)).reshape(len(vals), len(vals))
    z = z.reshape(-1)
    a = np.repeat(z, len(z))
    b = np.tile(z, len(z))
    want = a.copy()
    assert orc.reduce_local(b.copy(), want, len(a), mpi.DATATYPES[t], mpi.OPS[op]) == 0
    tio, pio = dev(cuda, a.view(np.uint8))
    tin, pin = dev(cuda, b.view(np.uint8))
    assert mpi.reduce_local(pin, pio, len(a), mpi.DATATYPES[t], mpi.OPS[op]) == 0
    got = back(tio, 0, a.nbytes)
    if not same(got, want.view(np.uint8), t):
        pytest.fail(f"{op} {t}:\n" + explain(got, want.view(np.uint8), a.view(np.uint8), b.view(np.uint8),
                                             a.itemsize, limit=30))
    # the non-NaN part really is exercised: infinities from the Annex G recovery
    if op == "MPI_PROD":
        assert np.isinf(got.view(ft)).sum() > 100


def test_maximum_count_int_max(mpi, cuda):
    """count = INT_MAX (the reference's `int count` limit): 2 GiB of MPI_BYTE
    BXOR and 8 GiB fp32 SUM per operand; checked on the device with torch
    (XOR / IEEE add are exact elementwise, so torch's result is the oracle's)."""
    torch = cuda
    n = 2 ** 31 - 1
    a = torch.randint(0, 256, (n + 1,), dtype=torch.uint8, device="cuda")[:n]
    b = torch.randint(0, 256, (n + 1,), dtype=torch.uint8, device="cuda")[:n]
    want = torch.bitwise_xor(a, b)
    torch.cuda.synchronize()
    assert mpi.reduce_local(b.data_ptr(), a.data_ptr(), n, mpi.MPI_BYTE, mpi.MPI_BXOR) == 0
    assert torch.equal(a, want)
    del a, b, want
    torch.cuda.empty_cache()
    x = torch.rand(n, device="cuda")
    y = torch.rand(n, device="cuda")
    want = x + y
    torch.cuda.synchronize()
    assert mpi.reduce_local(y.data_ptr(), x.data_ptr(), n, mpi.MPI_FLOAT, mpi.MPI_SUM) == 0
    assert torch.equal(x.view(torch.int32), want.view(torch.int32))
    # the last elements (tail of the final tile) really were combined
    assert torch.equal(x[-5:].view(torch.int32), want[-5:].view(torch.int32))


def test_concurrent_host_threads(mpi, orc, cuda):
    """MPIR_Reduce_local is reentrant (per-thread op_errno, stream, wait flag):
    8 host threads reduce their own buffers at once."""
    import threading
    torch = cuda
    n = (1 << 20) + 11
    rng = np.random.default_rng(3)
    data = []
    for i in range(8):
        a = T.to_bytes(T.gen("MPI_DOUBLE", n, rng))
        b = T.to_bytes(T.gen("MPI_DOUBLE", n, rng))
        w = a.copy()
        orc.reduce_local(b.copy(), w, n, mpi.MPI_DOUBLE, mpi.MPI_SUM)
        data.append((torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda(), w))
    torch.cuda.synchronize()
    errs = []

    def work(i):
        da, db, _ = data[i]
        rc = mpi.reduce_local(db.data_ptr(), da.data_ptr(), n, mpi.MPI_DOUBLE, mpi.MPI_SUM)
        if rc:
            errs.append(rc)
        # an invalid call on the same thread must not disturb the others
        if mpi.error_class(mpi.reduce_local(db.data_ptr(), da.data_ptr(), n, mpi.MPI_DOUBLE, mpi.MPI_BAND)) != \
                mpi.MPI_ERR_OP:
            errs.append("band")

    ths = [threading.Thread(target=work, args=(i,)) for i in range(8)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(120)
    assert not errs
    for da, db, w in data:
        assert np.array_equal(da.cpu().numpy(), w)


def test_thread_contexts_reused(mpi, cuda):
    """Per-thread HIP contexts return to a pool at thread exit: 64 short-lived
    threads, 4 alive at a time, create at most the peak concurrency's worth of
    new contexts (streams, completion words), and every call stays exact."""
    import threading
    torch = cuda
    n = 4099
    x = torch.arange(n, dtype=torch.int64, device="cuda")
    ones = torch.ones(n, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    assert mpi.reduce_local(ones.data_ptr(), x.data_ptr(), n, mpi.MPI_INT64_T, mpi.MPI_SUM) == 0
    before = mpi.load().MPIR_Hip_thread_contexts()
    lock = threading.Lock()
    errs = []

    def work():
        with lock:
            if mpi.reduce_local(ones.data_ptr(), x.data_ptr(), n, mpi.MPI_INT64_T, mpi.MPI_SUM):
                errs.append(mpi.load().MPIR_Hip_error_string())

    for _ in range(16):
        ths = [threading.Thread(target=work) for _ in range(4)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(60)
    assert not errs
    assert mpi.load().MPIR_Hip_thread_contexts() - before <= 4
    assert torch.equal(x, torch.arange(n, dtype=torch.int64, device="cuda") + 65)


@pytest.mark.parametrize("staged", [False, True], ids=["dispatch", "staged"])
def test_concurrent_pageable_threads(mpi, orc, cuda, staged):
    """Four host threads reduce pageable host buffers at once (the binding
    releases the GIL around the call).  Staged (MPIR_Hip_set_host_max_bytes(0)):
    each thread has its own staging streams and bounce slots and they share the
    copy pool (one split copy at a time); default dispatch: the host combine,
    split over the same pool.  Every result bit-exact."""
    with host_max(mpi, 0 if staged else (1 << 64) - 1):
        _concurrent_pageable_threads(mpi)


def _concurrent_pageable_threads(mpi):
    import threading
    n = (10 << 20) + 17                      # 40 MiB of fp32: several 16 MiB chunks per call
    rng = np.random.default_rng(9)
    data = []
    for i in range(4):
        a = rng.uniform(-1, 1, n).astype(np.float32)
        b = rng.uniform(-1, 1, n).astype(np.float32)
        data.append((a, b, a + b, a.copy()))  # one IEEE add per element, as the reference
    errs = []

    fast = mpi.fast_reduce_local()

    def work(i):
        # all four through the compiled binding, which releases the GIL for the
        # call, so the four really overlap
        a, b, _, a0 = data[i]
        for rep in range(2):
            rc = fast(b.ctypes.data, a.ctypes.data, n, mpi.MPI_FLOAT, mpi.MPI_SUM)
            if rc:
                errs.append((i, rc))
            if rep == 0:
                np.copyto(a, a0)                # restore: the second call recomputes the same sum

    ths = [threading.Thread(target=work, args=(i,)) for i in range(4)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(120)
    assert not errs
    for a, b, want, _ in data:
        assert np.array_equal(a, want)


def test_long_double_complex_prod_fast_path_edges(mpi, orc, cuda):
    """long double _Complex PROD takes a class-check-free path when all four parts
    are normal with biased exponents in [8200, 24560] (x87.hpp x80_cmul); parts
    at and just outside those bounds, and products that reach the overflow /
    underflow edges from inside and outside the range, against the host x87."""
    rng = np.random.default_rng(0xCB0)
    n = 4099
    edges = np.array([8199, 8200, 8201, 16383, 24559, 24560, 24561, 1, 32766, 0], dtype=np.uint16)

    def parts():
        v = np.zeros(n, dtype=T.X80)
        e = edges[rng.integers(0, edges.size, n)]
        m = rng.integers(0, 2 ** 63, n, dtype=np.uint64) | np.uint64(1 << 63)
        m[e == 0] >>= np.uint64(rng.integers(1, 63))            # denormals
        v["m"] = m
        v["se"] = e | (rng.integers(0, 2, n, dtype=np.uint16) << np.uint16(15))
        v["pad"] = np.frombuffer(rng.bytes(6 * n), dtype="V6")
        return v

    for _ in range(3):
        a = np.zeros(n, dtype=T.CX80)
        b = np.zeros(n, dtype=T.CX80)
        a["re"], a["im"], b["re"], b["im"] = parts(), parts(), parts(), parts()
        ab, bb = T.to_bytes(a), T.to_bytes(b)
        want = ab.copy()
        t = "MPI_C_LONG_DOUBLE_COMPLEX"
        assert orc.reduce_local(bb.copy(), want, n, mpi.DATATYPES[t], mpi.OPS["MPI_PROD"]) == 0
        tio, pio = dev(cuda, ab)
        tin, pin = dev(cuda, bb)
        assert mpi.reduce_local(pin, pio, n, mpi.DATATYPES[t], mpi.OPS["MPI_PROD"]) == 0
        got = back(tio, 0, ab.size)
        if not same(got, want, t):
            pytest.fail(explain(got, want, ab, bb, T.elem_size(t)))


@pytest.mark.parametrize("dtname,handle,size", [("MPI_WCHAR", 0x4c00040e, 4), ("MPI_PACKED", 0x4c00010f, 1),
                                                ("MPI_INTEGER(Fortran)", 0x4c00041b, 4), ("MPI_LB", 0x4c000010, 0),
                                                ("MPI_FLOAT", 0x4c00040a, 4), ("MPI_DOUBLE_INT", 0x8c000001, 16)])
def test_replace_every_predefined_type(mpi, cuda, dtname, handle, size):
    """MPIR_REPLACE through the op table (RMA accumulate's route, mpidrma.h:902) is
    MPIR_Localcopy (opreplace.c:18) for every predefined datatype, including the
    ones outside the reduction type table (size from the handle, bits 8-15);
    a derived-type handle gives MPI_ERR_TYPE through op_errno."""
    torch = cuda
    lib = mpi.load()
    n = 1001
    nbytes = n * (size if handle != 0x8c000001 else 16)
    rng = np.random.default_rng(5)
    src = rng.integers(0, 256, max(nbytes, 1), dtype=np.uint8)
    dst = rng.integers(0, 256, max(nbytes, 1), dtype=np.uint8)
    tin, pin = dev(torch, src)
    tio, pio = dev(torch, dst)
    ln = ctypes.c_int(n)
    ty = ctypes.c_int(handle)
    tbl = (ctypes.c_void_p * 15).in_dll(lib, "MPIR_Op_table")
    assert tbl[13] == ctypes.cast(lib.MPIR_REPLACE, ctypes.c_void_p).value
    errno_slot = lib.MPIR_Op_errno_ptr
    errno_slot.restype = ctypes.POINTER(ctypes.c_int)
    errno_slot()[0] = 0
    lib.MPIR_REPLACE(ctypes.c_void_p(pin), ctypes.c_void_p(pio), ctypes.byref(ln), ctypes.byref(ty))
    assert errno_slot()[0] == 0
    got = back(tio, 0, max(nbytes, 1))
    want = src[:nbytes] if nbytes else dst[:1]
    assert np.array_equal(got[:max(nbytes, 1)], want if nbytes else dst[:1]), dtname
    # a derived datatype (direct handle of kind DATATYPE) is refused
    ty2 = ctypes.c_int(0x8c000100)
    lib.MPIR_REPLACE(ctypes.c_void_p(pin), ctypes.c_void_p(pio), ctypes.byref(ln), ctypes.byref(ty2))
    assert errno_slot()[0] == mpi.MPI_ERR_TYPE


def run_pair_host(mpi, orc, op, t, n, seed, off=0):
    """Both operands in pageable host memory (byte offset `off`): at most
    MPIR_Hip_host_max_bytes() per operand the combine runs on the calling
    thread through the same functors as the kernels (hip_reduce.hip)."""
    rng = np.random.default_rng(seed)
    a = T.to_bytes(T.gen(t, n, rng, op))
    b = T.to_bytes(T.gen(t, n, rng, op))
    want = a.copy()
    rc_o = orc.reduce_local(b.copy(), want, n, mpi.DATATYPES[t], mpi.OPS[op])
    ha = np.zeros(a.size + off, np.uint8)
    hb = np.zeros(b.size + off, np.uint8)
    ha[off:] = a
    hb[off:] = b
    rc = mpi.reduce_local(hb.ctypes.data + off, ha.ctypes.data + off, n, mpi.DATATYPES[t], mpi.OPS[op])
    got = ha[off:]
    assert mpi.error_class(rc) == rc_o, (op, t, rc, rc_o)
    assert np.array_equal(hb[off:], b), "inbuf modified"
    if not same(got, want, t):
        pytest.fail(f"host {op} {t} n={n} off={off}:\n" + explain(got, want, a, b, T.elem_size(t)))


@pytest.mark.parametrize("op,t", MATRIX, ids=[f"{o}-{t}" for o, t in MATRIX])
def test_host_path_matrix_vs_oracle(mpi, orc, cuda, op, t):
    """Small host-resident operands (the host combine), every (op, type) pair,
    edge values included, aligned and misaligned."""
    for n, seed, off in ((1, 11, 0), (7, 12, 3), (1000, 13, 0), (4099, 14, 1)):
        run_pair_host(mpi, orc, op, t, n, seed, off)


def _node_cpus():
    nodes, k = [], 0
    full = os.sched_getaffinity(0)
    while os.path.exists(f"/sys/devices/system/node/node{k}/cpulist"):
        cpus = set()
        for part in open(f"/sys/devices/system/node/node{k}/cpulist").read().strip().split(","):
            lo, _, hi = part.partition("-")
            cpus.update(range(int(lo), int(hi or lo) + 1))
        nodes.append(cpus & full)
        k += 1
    return nodes


@pytest.mark.parametrize("op,t", [("MPI_SUM", "MPI_FLOAT"), ("MPI_MAX", "MPI_DOUBLE"), ("MPI_BXOR", "MPI_INT"),
                                  ("MPI_MINLOC", "MPI_FLOAT_INT")])
def test_host_combine_numa_pools_vs_oracle(mpi, orc, cuda, op, t):
    """Split host combines (>= 512 KiB per operand) on operands first-touched on
    each NUMA node of the host (the node pools), on operands straddling two
    nodes (the floating pool) and with odd part boundaries: bit-exact against
    the oracle.  On a one-node host every case takes the floating pool."""
    nodes = [c for c in _node_cpus() if c]
    full = os.sched_getaffinity(0)
    rng = np.random.default_rng(2024)
    n = (3 << 20) // 8 + 5                       # ~3 MiB of 8-byte elements, ragged
    cases = [(k, None) for k in range(len(nodes))] + ([(0, 1)] if len(nodes) > 1 else [])
    for first, second in cases:
        a = T.to_bytes(T.gen(t, n, rng, op))
        b = T.to_bytes(T.gen(t, n, rng, op))
        want = a.copy()
        assert orc.reduce_local(b.copy(), want, n, mpi.DATATYPES[t], mpi.OPS[op]) == 0
        try:
            os.sched_setaffinity(0, nodes[first])
            ha = np.empty_like(a)
            hb = np.empty_like(b)
            half = a.size // 2
            ha[:half] = a[:half]
            hb[:half] = b[:half]
            if second is not None:               # the other half on the other node
                os.sched_setaffinity(0, nodes[second])
            ha[half:] = a[half:]
            hb[half:] = b[half:]
        finally:
            os.sched_setaffinity(0, full)
        rc = mpi.reduce_local(hb.ctypes.data, ha.ctypes.data, n, mpi.DATATYPES[t], mpi.OPS[op])
        assert rc == 0, mpi.error_string(rc)
        assert same(ha, want, t), explain(ha, want, a, b, ha.size // n)


@pytest.mark.parametrize("path", ["host_combine", "mixed_slot"])
def test_pinned_host_operand_ordered_after_null_stream(mpi, orc, cuda, path):
    """A pinned host operand filled by an async D2H copy on the legacy null
    stream, queued behind slow device work, is read only after that copy lands:
    the host combine (both operands host) and the mixed path's slot copy (host
    inbuf, device inoutbuf) first synchronise with the null stream, as the
    device path does (hip_reduce.hip order_after_null_stream)."""
    import torch
    n = (256 << 10) if path == "mixed_slot" else (8 << 20)          # mixed: <= 1 MiB per operand
    rng = np.random.default_rng(77)
    a = rng.uniform(-1, 1, n).astype(np.float32)                   # inout
    b = rng.uniform(-1, 1, n).astype(np.float32)                   # in (arrives by D2H)
    want = a.copy()
    assert orc.reduce_local(b.copy(), want, n, mpi.MPI_FLOAT, mpi.MPI_SUM) == 0
    for rep in range(3):
        db = torch.from_numpy(b).cuda()
        big = torch.ones(64 << 20, device="cuda")
        torch.cuda.synchronize()
        hb = torch.full((n,), float("nan"), dtype=torch.float32).pin_memory()
        if path == "host_combine":
            ha = torch.from_numpy(a.copy()).pin_memory()
            io = ha.data_ptr()
        else:
            da = torch.from_numpy(a.copy()).cuda()
            io = da.data_ptr()
        torch.cuda.synchronize()
        for _ in range(20):                  # ~ms of work on the null stream ahead of the copy
            big.mul_(1.0000001)
        hb.copy_(db, non_blocking=True)      # D2H into pinned memory, null stream, returns at once
        rc = mpi.reduce_local(hb.data_ptr(), io, n, mpi.MPI_FLOAT, mpi.MPI_SUM)
        assert rc == 0, mpi.error_string(rc)
        got = ha.numpy() if path == "host_combine" else da.cpu().numpy()
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), (path, rep)


def test_host_path_crossover(mpi, orc, cuda):
    """Either side of a host limit set with MPIR_Hip_set_host_max_bytes (host
    combine below, GPU staging above; the default is no limit), and the host
    combine split over the copy pool's threads from 512 KiB (ragged and
    misaligned): all bit-exact."""
    lib = mpi.load()
    lib.MPIR_Hip_host_max_bytes.restype = ctypes.c_uint64
    assert lib.MPIR_Hip_host_max_bytes() == (1 << 64) - 1      # default: no limit
    lim = 1 << 20
    with host_max(mpi, lim):
        for op, t in (("MPI_SUM", "MPI_FLOAT"), ("MPI_PROD", "MPI_C_DOUBLE_COMPLEX"),
                      ("MPI_MAXLOC", "MPI_DOUBLE_INT"), ("MPI_BXOR", "MPI_UNSIGNED_CHAR"),
                      ("MPI_SUM", "MPI_LONG_DOUBLE")):
            esz = T.elem_size(t)
            # the host combine split over threads (>= 512 KiB), ragged, then either side of the limit
            for n, off in (((600 << 10) // esz + 3, 0), ((600 << 10) // esz + 1, 3), (lim // esz, 0),
                           (lim // esz + 1, 0)):
                run_pair_host(mpi, orc, op, t, n, 21 + n, off)


def run_pair_mixed(mpi, orc, torch, op, t, n, seed, host_side, pinned=False, off_host=0, off_dev=0):
    """One operand in host memory (`host_side` "in" or "inout"; pageable numpy or
    pinned torch memory, at byte offset `off_host`), the other on the device."""
    rng = np.random.default_rng(seed)
    a = T.to_bytes(T.gen(t, n, rng, op))          # inout
    b = T.to_bytes(T.gen(t, n, rng, op))          # in
    want = a.copy()
    rc_o = orc.reduce_local(b.copy(), want, n, mpi.DATATYPES[t], mpi.OPS[op])

    def host(x):
        if pinned:
            h = torch.zeros(x.size + off_host, dtype=torch.uint8).pin_memory()
            h[off_host:] = torch.from_numpy(x)
            return h, h.data_ptr() + off_host
        h = np.zeros(x.size + off_host, np.uint8)
        h[off_host:] = x
        return h, h.ctypes.data + off_host

    def host_back(h, size):
        return (h.numpy() if pinned else h)[off_host:off_host + size].copy()
    if host_side == "in":
        hin, pin = host(b)
        tio, pio = dev(torch, a, off_dev)
        rc = mpi.reduce_local(pin, pio, n, mpi.DATATYPES[t], mpi.OPS[op])
        got = back(tio, off_dev, a.size)
        assert np.array_equal(host_back(hin, b.size), b), "inbuf modified"
    else:
        tin, pin = dev(torch, b, off_dev)
        hio, pio = host(a)
        rc = mpi.reduce_local(pin, pio, n, mpi.DATATYPES[t], mpi.OPS[op])
        got = host_back(hio, a.size)
        assert np.array_equal(back(tin, off_dev, b.size), b), "inbuf modified"
    assert mpi.error_class(rc) == rc_o, (op, t, rc, rc_o)
    if not same(got, want, t):
        pytest.fail(f"mixed ({host_side} on host, pinned={pinned}) {op} {t} n={n} off=({off_host},{off_dev}):\n"
                    + explain(got, want, a, b, T.elem_size(t)))


MIXED = [("MPI_SUM", "MPI_FLOAT"), ("MPI_MAX", "MPI_DOUBLE"), ("MPI_PROD", "MPI_INT"), ("MPI_SUM", "MPIX_C_FLOAT16"),
         ("MPI_BXOR", "MPI_UNSIGNED_CHAR"), ("MPI_MINLOC", "MPI_DOUBLE_INT"), ("MPI_PROD", "MPI_C_DOUBLE_COMPLEX"),
         ("MPI_LAND", "MPI_SHORT"), ("MPI_SUM", "MPI_LONG_DOUBLE"), ("MPI_MAXLOC", "MPI_LONG_DOUBLE_INT")]


@pytest.mark.parametrize("op,t", MIXED, ids=[f"{o}-{t}" for o, t in MIXED])
def test_mixed_small_path_vs_oracle(mpi, orc, cuda, op, t):
    """One operand host memory, the other device memory, below
    MPIR_Hip_mixed_max_bytes: the host operand goes through the thread's pinned
    slot that the kernel reads / writes directly.  Both directions, pageable and
    pinned host memory, aligned and misaligned, ragged counts; bit-exact."""
    for side in ("in", "inout"):
        for pinned in (False, True):
            for n, seed, oh, od in ((1, 41, 0, 0), (7, 42, 3, 0), (1000, 43, 0, 16), (4099, 44, 5, 8),
                                    (65536 + 3, 45, 0, 0)):
                run_pair_mixed(mpi, orc, cuda, op, t, n, seed, side, pinned, oh, od)


@pytest.mark.parametrize("op,t", MATRIX, ids=[f"{o}-{t}" for o, t in MATRIX])
def test_mixed_path_matrix_vs_oracle(mpi, orc, cuda, op, t):
    """Every (op, type) the reference accepts through the mixed-residency path,
    both directions, a ragged count aligned and a short one misaligned."""
    for side in ("in", "inout"):
        run_pair_mixed(mpi, orc, cuda, op, t, 4099, 71, side)
        run_pair_mixed(mpi, orc, cuda, op, t, 33, 72, side, off_host=5, off_dev=3)


def test_mixed_path_crossover(mpi, orc, cuda):
    """Either side of MPIR_Hip_mixed_max_bytes (pinned slot below, staging
    pipeline above), both directions: bit-exact; below it the direct dispatch
    runs (aligned fp32 SUM)."""
    lib = mpi.load()
    lib.MPIR_Hip_mixed_max_bytes.restype = ctypes.c_uint64
    lim = lib.MPIR_Hip_mixed_max_bytes()
    assert lim == 1 << 20
    for op, t in (("MPI_SUM", "MPI_FLOAT"), ("MPI_MAXLOC", "MPI_DOUBLE_INT")):
        esz = T.elem_size(t)
        for side in ("in", "inout"):
            for n in (lim // esz, lim // esz + 1):
                run_pair_mixed(mpi, orc, cuda, op, t, n, 51 + n, side)
    d0 = _direct_count(mpi)
    run_pair_mixed(mpi, orc, cuda, "MPI_SUM", "MPI_FLOAT", 4096, 60, "in")
    run_pair_mixed(mpi, orc, cuda, "MPI_SUM", "MPI_FLOAT", 4096, 61, "inout")
    assert _direct_count(mpi) == d0 + 2


def _direct_count(mpi):
    lib = mpi.load()
    lib.MPIR_Hip_direct_dispatches.restype = ctypes.c_uint64
    return lib.MPIR_Hip_direct_dispatches()


def test_direct_dispatch_path(mpi, orc, cuda):
    """Synchronous device-resident calls go through the direct AQL dispatch
    (direct_dispatch.hip) with the kernel of plan_reduce's launch plan: the
    lean tile kernel (16 B-aligned 16 B multiples), the full one (head / tail
    elements), the shift kernel (unequal alignment mod 16) and the element
    kernels (small unequal or unnatural alignment), for every op but REPLACE;
    the 32-byte classes take the HIP launch.  Every result bit-exact."""
    torch = cuda
    before = _direct_count(mpi)
    for op, t in (("MPI_SUM", "MPI_FLOAT"), ("MPI_MAX", "MPI_DOUBLE"), ("MPI_PROD", "MPI_INT"),
                  ("MPI_MIN", "MPIX_C_FLOAT16"), ("MPI_SUM", "MPI_C_DOUBLE_COMPLEX")):
        run_pair(mpi, orc, torch, op, t, (1 << 18) + (16 // T.elem_size(t)) * 5, 31)
    mid = _direct_count(mpi)
    assert mid - before == 5, (before, mid)
    cases = [("MPI_SUM", "MPI_FLOAT", (1 << 18) + 1, 0, 0), ("MPI_SUM", "MPI_FLOAT", 3, 0, 0),     # full
             ("MPI_BXOR", "MPI_INT", 1 << 18, 0, 0), ("MPI_LAND", "MPI_UNSIGNED_CHAR", 4099, 5, 5),
             ("MPI_MAXLOC", "MPI_2INT", 1001, 8, 8), ("MPI_MINLOC", "MPI_DOUBLE_INT", 33, 0, 0),
             ("MPI_SUM", "MPI_LONG_DOUBLE", 257, 0, 0), ("MPI_LXOR", "MPI_DOUBLE", 77, 8, 8),
             ("MPI_PROD", "MPI_C_FLOAT_COMPLEX", 65537, 8, 8), ("MPI_BOR", "MPI_SHORT", 1, 2, 2),
             ("MPI_SUM", "MPI_FLOAT", 65539, 4, 0), ("MPI_MAX", "MPI_DOUBLE", 40000, 8, 0),            # shift
             ("MPI_SUM", "MPI_FLOAT", 4099, 4, 0), ("MPI_MINLOC", "MPI_SHORT_INT", 99, 4, 0),          # elements
             ("MPI_SUM", "MPI_DOUBLE", 1000, 3, 5)]                                                    # unnatural
    for k, (op, t, n, oi, oo) in enumerate(cases):
        run_pair(mpi, orc, torch, op, t, n, 40 + k, oi, oo)
    after = _direct_count(mpi)
    assert after - mid == len(cases), (mid, after)
    # the 32-byte classes: the HIP launch
    run_pair(mpi, orc, torch, "MPI_SUM", "MPI_C_LONG_DOUBLE_COMPLEX", 513, 61)
    run_pair(mpi, orc, torch, "MPI_MAXLOC", "MPI_LONG_DOUBLE_INT", 99, 62)
    assert _direct_count(mpi) == after


@pytest.mark.parametrize("op,t", MATRIX, ids=[f"{o}-{t}" for o, t in MATRIX])
def test_direct_dispatch_matrix(mpi, orc, cuda, op, t):
    """Every (op, type) the reference accepts, at ragged counts, equal and
    unequal misalignment: the classes of 16 bytes or less take the direct
    dispatch (counted), the 32-byte ones the HIP launch; all bit-exact."""
    esz = T.elem_size(t)
    eq = esz if 16 % esz == 0 and esz < 16 else 0
    shapes = [(1, 0, 0), (5, eq, eq), (4099, 0, 0), ((1 << 16) + 3, 0, 0),
              ((1 << 16) + 3, 4 if esz % 4 == 0 else 1, 0), (77, 0, 2 if esz % 2 == 0 else 1)]
    d0 = _direct_count(mpi)
    for n, oi, oo in shapes:
        run_pair(mpi, orc, cuda, op, t, n, 7 + n + oi, oi, oo)
    got = _direct_count(mpi) - d0
    # LAND / LOR on the reals pass check_dtype and then fail in the kernel's
    # type switch (the reference's quirk): no kernel runs
    quirk = op in ("MPI_LAND", "MPI_LOR") and t in T.REAL
    assert got == (len(shapes) if esz <= 16 and not quirk else 0), (op, t, got)


def test_direct_dispatch_many_threads_distinct_windows(mpi, cuda):
    """8 host threads, each rotating over its own 6 windows: the direct
    dispatch's kernarg cache entries collide across threads and spill to ring
    slots, which must never be rewritten while a dispatch that reads them is in
    flight.  Every window's in-place fp32 sums are bit-exact against numpy's
    float32 sequence of the same additions."""
    import threading
    torch = cuda
    nthreads, nwin, n, iters = 8, 6, (1 << 18) + 16, 30
    rng = np.random.default_rng(77)
    a0 = [[rng.uniform(-1, 1, n).astype(np.float32) for _ in range(nwin)] for _ in range(nthreads)]
    b0 = [[rng.uniform(-1, 1, n).astype(np.float32) for _ in range(nwin)] for _ in range(nthreads)]
    da = [[torch.from_numpy(x.copy()).cuda() for x in row] for row in a0]
    db = [[torch.from_numpy(x.copy()).cuda() for x in row] for row in b0]
    torch.cuda.synchronize()
    f = mpi.fast_reduce_local()
    d0 = _direct_count(mpi)
    errors = []

    def run(k):
        for i in range(iters):
            w = (i * 5 + k) % nwin
            rc = f(db[k][w].data_ptr(), da[k][w].data_ptr(), n, mpi.MPI_FLOAT, mpi.MPI_SUM)
            if rc:
                errors.append(rc)
    th = [threading.Thread(target=run, args=(k,)) for k in range(nthreads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    assert _direct_count(mpi) - d0 >= nthreads * iters // 2      # most calls went direct
    for k in range(nthreads):
        want = [x.copy() for x in a0[k]]
        for i in range(iters):
            w = (i * 5 + k) % nwin
            want[w] = want[w] + b0[k][w]
        for w in range(nwin):
            assert np.array_equal(da[k][w].cpu().numpy(), want[w]), (k, w)


def test_direct_dispatch_fresh_args_every_call(mpi, cuda):
    """Every call with new kernel arguments (a window shifted by 256 B each
    time, 1500 calls over 1024 distinct argument sets): each misses the kernarg
    cache, so its arguments are written into a VRAM slot that earlier
    dispatches read (128 cache slots, each rewritten ~10 times), written before
    the doorbell and checked by the kernel's nonce.  A stale read would combine
    the wrong window: each element's final value counts exactly the calls whose
    window covered it, checked against numpy's replay of the same sequence."""
    torch = cuda
    n, nbuf, noff, calls = 4096, 4, 256, 1500
    span = n + noff * 64
    da = [torch.zeros(span, dtype=torch.float32, device="cuda") for _ in range(nbuf)]
    db = [torch.ones(span, dtype=torch.float32, device="cuda") for _ in range(nbuf)]
    torch.cuda.synchronize()
    f = mpi.fast_reduce_local()
    lib = mpi.load()
    w0, d0 = lib.MPIR_Hip_direct_kernarg_writes(), _direct_count(mpi)
    want = [np.zeros(span, np.float32) for _ in range(nbuf)]
    for i in range(calls):
        j, o = i % nbuf, ((i // nbuf) * 37) % noff * 64          # element offsets, 256 B steps
        assert f(db[j].data_ptr() + 4 * o, da[j].data_ptr() + 4 * o, n, mpi.MPI_FLOAT, mpi.MPI_SUM) == 0
        want[j][o:o + n] += 1
    assert _direct_count(mpi) - d0 == calls
    assert lib.MPIR_Hip_direct_kernarg_writes() - w0 >= calls - 2 * nbuf
    for j in range(nbuf):
        assert np.array_equal(da[j].cpu().numpy(), want[j]), j


def test_direct_dispatch_verified_hits_small_grids(mpi, cuda):
    """A kernarg-cache hit whose slot a checked dispatch has verified runs the
    UNchecked kernel on the slot as it stands.  With grids of 1-7 workgroups a
    checked dispatch touches only some XCDs, so an XCD it did not reach could
    still hold the slot's previous occupant in its L2.  600 operand pairs of
    1-7 tiles share the 128 cache slots (every slot rewritten many times); each
    pair is called twice in a row (miss -> checked, then verified hit ->
    unchecked) and again later.  A stale read would add into the previous
    occupant's buffers: every buffer must count exactly its own calls."""
    torch = cuda
    f = mpi.fast_reduce_local()
    npairs, rounds = 600, 5
    sizes = [4096 * (1 + k % 7) for k in range(npairs)]         # 16 KiB tiles: 1-7 workgroups
    da = [torch.zeros(n, dtype=torch.float32, device="cuda") for n in sizes]
    db = [torch.ones(n, dtype=torch.float32, device="cuda") for n in sizes]
    torch.cuda.synchronize()
    d0 = _direct_count(mpi)
    rng = np.random.default_rng(7)
    calls = np.zeros(npairs, np.int64)
    for _ in range(rounds):
        for k in rng.permutation(npairs):
            for _rep in range(2):
                assert f(db[k].data_ptr(), da[k].data_ptr(), sizes[k], mpi.MPI_FLOAT, mpi.MPI_SUM) == 0
            calls[k] += 2
    assert _direct_count(mpi) - d0 == int(calls.sum())
    for k in range(npairs):
        got = da[k].cpu().numpy()
        assert np.all(got == calls[k]), (k, sizes[k], np.unique(got))


def test_direct_dispatch_preempted_writer(mpi, cuda):
    """A kernarg-cache miss writes its slot before ringing the doorbell; should
    the write ever lose the race to the CP (the test hook moves it behind the
    doorbell and holds it back 20 ms, as a host thread preempted at that point
    would), the dispatched workgroups wait for the nonce instead of combining
    stale arguments.  For every launch plan the checked kernels serve (lean
    tile, tile with head / tail, shift, elements): every call completes
    through the direct path, bit-exact, and the path stays open afterwards."""
    torch = cuda
    lib = mpi.load()
    lib.MPIR_Hip_direct_test_write_delay_us.restype = ctypes.c_uint32
    lib.MPIR_Hip_direct_test_write_delay_us.argtypes = [ctypes.c_uint32]
    f = mpi.fast_reduce_local()
    x = torch.zeros(2, device="cuda")
    torch.cuda.synchronize()
    assert f(x.data_ptr(), x.data_ptr() + 4, 1, mpi.MPI_FLOAT, mpi.MPI_SUM) == 0
    if lib.MPIR_Hip_direct_state(torch.cuda.current_device()) != 1:
        pytest.skip("direct dispatch not in nonce mode (unavailable or under a queue-intercepting tool)")
    rng = np.random.default_rng(7)
    # (count, inbuf byte offset, inoutbuf byte offset): lean tile, head/tail tile, shift, elements
    shapes = [(1 << 20, 0, 0), ((1 << 20) + 5, 4, 4), ((1 << 20) + 3, 4, 0), (1000, 4, 8)]
    keep = []                                   # distinct addresses: every call misses the cache
    prev = lib.MPIR_Hip_direct_test_write_delay_us(20000)
    try:
        for rep in range(2):
            for n, oi, oo in shapes:
                a = rng.uniform(-1, 1, n).astype(np.float32)
                b = rng.uniform(-1, 1, n).astype(np.float32)
                din = torch.zeros(n + 16, dtype=torch.float32, device="cuda")
                dio = torch.zeros(n + 16, dtype=torch.float32, device="cuda")
                din[oi // 4: oi // 4 + n] = torch.from_numpy(b).cuda()
                dio[oo // 4: oo // 4 + n] = torch.from_numpy(a).cuda()
                keep += [din, dio]
                torch.cuda.synchronize()
                d0, w0 = _direct_count(mpi), lib.MPIR_Hip_direct_kernarg_writes()
                t0 = time.perf_counter()
                rc = f(din.data_ptr() + oi, dio.data_ptr() + oo, n, mpi.MPI_FLOAT, mpi.MPI_SUM)
                dt = time.perf_counter() - t0
                assert rc == 0, mpi.error_string(rc)
                assert _direct_count(mpi) - d0 == 1 and lib.MPIR_Hip_direct_kernarg_writes() - w0 == 1
                assert dt >= 0.019, dt            # the call really waited for the held-back write
                got = dio[oo // 4: oo // 4 + n].cpu().numpy()
                assert np.array_equal(got.view(np.uint32), (a + b).view(np.uint32)), (n, oi, oo)
    finally:
        lib.MPIR_Hip_direct_test_write_delay_us(prev)
    assert lib.MPIR_Hip_direct_state(torch.cuda.current_device()) == 1
    d0 = _direct_count(mpi)
    assert f(din.data_ptr() + oi, dio.data_ptr() + oo, n, mpi.MPI_FLOAT, mpi.MPI_SUM) == 0
    assert _direct_count(mpi) - d0 == 1


def test_direct_dispatch_orders_after_null_stream(mpi, cuda):
    """Work the caller left running on the legacy null stream for the operands
    is finished before the reduction reads them: the direct path first
    synchronises with a null stream that reports pending work, then dispatches
    (hipStreamQuery(nullptr) alone keeps reporting finished work as pending
    until the host synchronises, tools/archive/direct_probe.py)."""
    torch = cuda
    if torch.cuda.current_stream().cuda_stream != 0:
        pytest.skip("torch's current stream is not the legacy null stream")
    n = 1 << 24
    src = torch.rand(n, device="cuda")
    b = torch.rand(n, device="cuda")
    a = torch.zeros(n, device="cuda")
    big = torch.rand(4096, 4096, device="cuda")
    torch.cuda.synchronize()
    for _ in range(3):
        big = big @ big / 4096.0          # keep the null stream busy for a while ...
    a.copy_(src)                           # ... then produce the inout operand on it
    lib = mpi.load()
    d0, s0 = _direct_count(mpi), lib.MPIR_Hip_direct_busy_skips()
    rc = mpi.reduce_local(b.data_ptr(), a.data_ptr(), n, mpi.MPI_FLOAT, mpi.MPI_SUM)   # no sync before
    assert rc == 0
    assert _direct_count(mpi) == d0 + 1 and lib.MPIR_Hip_direct_busy_skips() == s0 + 1
    want = (src + b).cpu().numpy()
    assert np.array_equal(a.cpu().numpy(), want)


def test_direct_dispatch_timestamps(mpi, cuda):
    """MPIR_Hip_direct_profile: the first call after switching it on already
    reports its kernel's CP start / end interval (the queue records timestamps
    from its creation), and it lies within the call's own wall time."""
    import time
    torch = cuda
    n = 1 << 24
    a = torch.rand(n, device="cuda")
    b = torch.rand(n, device="cuda")
    torch.cuda.synchronize()
    lib = mpi.load()
    assert lib.MPIR_Hip_direct_state(torch.cuda.current_device()) in (0, 1)
    assert mpi.reduce_local(b.data_ptr(), a.data_ptr(), n, mpi.MPI_FLOAT, mpi.MPI_SUM) == 0
    # 1: the queue's dispatch ids are its packet indices (no intercepting tool),
    # so the nonce protocol is on
    assert lib.MPIR_Hip_direct_state(torch.cuda.current_device()) == 1
    lib.MPIR_Hip_direct_profile(1)
    try:
        for _ in range(3):
            t0 = time.perf_counter()
            assert mpi.reduce_local(b.data_ptr(), a.data_ptr(), n, mpi.MPI_FLOAT, mpi.MPI_SUM) == 0
            wall_ns = (time.perf_counter() - t0) * 1e9
            ns = lib.MPIR_Hip_direct_last_kernel_ns()
            assert 0 < ns < wall_ns, (ns, wall_ns)
    finally:
        lib.MPIR_Hip_direct_profile(0)


def test_stream_variant_then_sync_call_ordered(mpi, cuda):
    """MPIX_Reduce_local_stream on the library stream (hip_stream NULL, no wait)
    then MPI_Reduce_local on the same buffers: the second call sees the first's
    result ((a + b) + b, fp32 rounded twice)."""
    torch = cuda
    n = (1 << 22)
    a0 = torch.rand(n, device="cuda")
    b = torch.rand(n, device="cuda")
    a = a0.clone()
    torch.cuda.synchronize()
    assert mpi.reduce_local_stream(b.data_ptr(), a.data_ptr(), n, mpi.MPI_FLOAT, mpi.MPI_SUM, 0) == 0
    assert mpi.reduce_local(b.data_ptr(), a.data_ptr(), n, mpi.MPI_FLOAT, mpi.MPI_SUM) == 0
    want = ((a0 + b) + b).cpu().numpy()
    assert np.array_equal(a.cpu().numpy(), want)

"""Datatype table and seeded input generators shared by the parity tests.

Every MPI basic type of the build (x86-64, no Fortran / C++; long double is
the x87 80-bit format in a 16-byte slot),
its numpy element representation, and the ops whose compute switch handles
it (src/mpi/coll/op/op*.c).  Inputs are seeded uniform values with fixed
positions overwritten by edge values (NaN, +-0, +-inf, denormals, INT_MIN /
INT_MAX, equal MAXLOC values) -- SURVEY.md §8c fixture plan.
"""
from __future__ import annotations

import numpy as np

OPS = ["MPI_MAX", "MPI_MIN", "MPI_SUM", "MPI_PROD", "MPI_LAND", "MPI_BAND", "MPI_LOR", "MPI_BOR",
       "MPI_LXOR", "MPI_BXOR", "MPI_MINLOC", "MPI_MAXLOC"]

INT = {"MPI_INT": "i4", "MPI_LONG": "i8", "MPI_SHORT": "i2", "MPI_UNSIGNED_SHORT": "u2", "MPI_UNSIGNED": "u4",
       "MPI_UNSIGNED_LONG": "u8", "MPI_LONG_LONG": "i8", "MPI_UNSIGNED_LONG_LONG": "u8",
       "MPI_SIGNED_CHAR": "i1", "MPI_UNSIGNED_CHAR": "u1", "MPI_INT8_T": "i1", "MPI_INT16_T": "i2",
       "MPI_INT32_T": "i4", "MPI_INT64_T": "i8", "MPI_UINT8_T": "u1", "MPI_UINT16_T": "u2",
       "MPI_UINT32_T": "u4", "MPI_UINT64_T": "u8", "MPI_CHAR": "i1", "MPI_AINT": "i8", "MPI_OFFSET": "i8",
       "MPI_COUNT": "i8"}
REAL = {"MPI_FLOAT": "f4", "MPI_DOUBLE": "f8", "MPIX_C_FLOAT16": "f2", "MPI_LONG_DOUBLE": "x80"}
CPLX = {"MPI_C_FLOAT_COMPLEX": "c8", "MPI_C_DOUBLE_COMPLEX": "c16", "MPI_C_LONG_DOUBLE_COMPLEX": "cx80"}
# x87 extended: 8-byte significand (explicit integer bit), 2-byte sign/exponent,
# 6 padding bytes that a long double store never writes
X80 = np.dtype([("m", "<u8"), ("se", "<u2"), ("pad", "V6")])
CX80 = np.dtype([("re", X80), ("im", X80)])
OTHER = {"MPI_C_BOOL": "b1", "MPI_BYTE": "u1"}
PAIRS = {
    "MPI_2INT": np.dtype([("value", "<i4"), ("loc", "<i4")]),
    "MPI_FLOAT_INT": np.dtype([("value", "<f4"), ("loc", "<i4")]),
    "MPI_LONG_INT": np.dtype([("value", "<i8"), ("loc", "<i4"), ("pad", "<i4")]),
    "MPI_SHORT_INT": np.dtype([("value", "<i2"), ("pad", "<i2"), ("loc", "<i4")]),
    "MPI_DOUBLE_INT": np.dtype([("value", "<f8"), ("loc", "<i4"), ("pad", "<i4")]),
    "MPI_LONG_DOUBLE_INT": np.dtype([("value", X80), ("loc", "<i4"), ("pad", "V12")]),
}
ALL_TYPES = list(INT) + list(REAL) + list(CPLX) + list(OTHER) + list(PAIRS)


def compute_ok(op: str, t: str) -> bool:
    """Does the reference's compute switch for `op` handle `t` (op*.c)?"""
    integers = t in INT
    real = t in REAL
    if op in ("MPI_MAX", "MPI_MIN"):
        return integers or real
    if op in ("MPI_SUM", "MPI_PROD"):
        return integers or real or t in CPLX
    if op in ("MPI_LAND", "MPI_LOR"):
        return integers or t == "MPI_C_BOOL"
    if op == "MPI_LXOR":
        return integers or real or t == "MPI_C_BOOL"
    if op in ("MPI_BAND", "MPI_BOR", "MPI_BXOR"):
        return integers or t == "MPI_BYTE"
    if op in ("MPI_MAXLOC", "MPI_MINLOC"):
        return t in PAIRS
    return False


def check_ok(op: str, t: str) -> bool:
    """Does the reference's check_dtype for `op` accept `t`?  (LAND/LOR also floats)"""
    if op in ("MPI_LAND", "MPI_LOR") and t in REAL:
        return True
    return compute_ok(op, t)


def np_dtype(t: str) -> np.dtype:
    if t in PAIRS:
        return PAIRS[t]
    if t == "MPI_LONG_DOUBLE":
        return X80
    if t == "MPI_C_LONG_DOUBLE_COMPLEX":
        return CX80
    code = {**INT, **REAL, **CPLX, **OTHER}[t]
    return np.dtype({"f2": "<u2", "b1": "u1"}.get(code, "<" + code if code[0] != "b" else code))


def elem_size(t: str) -> int:
    return np_dtype(t).itemsize


F32_SPECIALS = [0x7FC00000, 0xFFC00000, 0x7F800000, 0xFF800000, 0x00000000, 0x80000000, 0x00000001,
                0x807FFFFF, 0x7F7FFFFF, 0x3F800000, 0x7FA00001]
F64_SPECIALS = [0x7FF8000000000000, 0xFFF8000000000000, 0x7FF0000000000000, 0xFFF0000000000000, 0,
                0x8000000000000000, 1, 0x800FFFFFFFFFFFFF, 0x7FEFFFFFFFFFFFFF, 0x3FF0000000000000,
                0x7FF4000000000001]
F16_SPECIALS = [0x7E00, 0xFE00, 0x7C00, 0xFC00, 0x0000, 0x8000, 0x0001, 0x83FF, 0x7BFF, 0x3C00, 0x7D01]


def gen_x80(n: int, rng: np.random.Generator, specials: bool = True, pool: int = 0) -> np.ndarray:
    """n x87 extended values as raw encodings: mostly normals (exponents near
    1.0, some short significands for exact / tie cases, some across the range),
    plus -- with specials -- denormals, pseudo-denormals, zeros, infinities,
    quiet and signalling NaNs, unnormals and pseudo-NaN / pseudo-infinities.
    Padding bytes are random (they must come through untouched).
    pool > 0: draw from `pool` distinct values (many equal pairs, for MAXLOC)."""
    x = np.zeros(n, dtype=X80)
    m = rng.integers(0, 2 ** 63, n, dtype=np.uint64) | np.uint64(1 << 63)
    short = rng.random(n) < 0.3
    m[short] &= np.uint64(0xFFFFFF0000000000)
    e = (0x3FFF - 20 + rng.integers(0, 40, n)).astype(np.uint16)
    wide = rng.random(n) < 0.1
    e[wide] = rng.integers(1, 0x7FFF, int(wide.sum())).astype(np.uint16)
    sign = (rng.integers(0, 2, n) << 15).astype(np.uint16)
    if specials:
        k = rng.integers(0, 100, n)
        cls = [(k < 3, 0, None), ((k >= 3) & (k < 5), 0, "pseudo"), ((k >= 5) & (k < 7), 0, "zero"),
               ((k >= 7) & (k < 9), 0x7FFF, "inf"), ((k >= 9) & (k < 11), 0x7FFF, "qnan"),
               ((k >= 11) & (k < 13), 0x7FFF, "snan"), ((k >= 13) & (k < 14), None, "unnormal"),
               ((k >= 14) & (k < 15), 0x7FFF, "pseudonan")]
        for mask, ev, kind in cls:
            c = int(mask.sum())
            if not c:
                continue
            r = rng.integers(0, 2 ** 62, c, dtype=np.uint64)
            if kind is None:                     # denormal
                mm = r >> rng.integers(0, 62, c).astype(np.uint64)
            elif kind == "pseudo":
                mm = r | np.uint64(1 << 63)
            elif kind == "zero":
                mm = np.zeros(c, np.uint64)
            elif kind == "inf":
                mm = np.full(c, 1 << 63, np.uint64)
            elif kind == "qnan":
                mm = r | np.uint64(3 << 62)
            elif kind == "snan":
                mm = (r >> np.uint64(1)) | np.uint64(1 << 63) | np.uint64(1)
            elif kind == "unnormal":
                mm = r
            else:
                mm = r
            m[mask] = mm
            if ev is None:
                e[mask] = rng.integers(1, 0x7FFF, c).astype(np.uint16)
            else:
                e[mask] = ev
    x["m"] = m
    x["se"] = sign | e
    x["pad"] = rng.integers(0, 256, (n, 6), dtype=np.uint8).view("V6").reshape(n)
    if pool:
        pick = rng.integers(0, min(pool, n), n)
        x["m"], x["se"] = x["m"][pick], x["se"][pick]
    return x


def x80_nanish(v: np.ndarray) -> np.ndarray:
    """x87 operands a compare finds unordered: NaNs and invalid encodings."""
    e = v["se"] & 0x7FFF
    j = (v["m"] >> np.uint64(63)) == 1
    nan = (e == 0x7FFF) & j & ((v["m"] << np.uint64(1)) != 0)
    invalid = ((e == 0x7FFF) & ~j) | ((e > 0) & (e < 0x7FFF) & ~j)
    return nan | invalid


def gen(t: str, n: int, rng: np.random.Generator, op: str = "MPI_SUM", specials: bool = True) -> np.ndarray:
    """n elements of type t; raw bit patterns for floats so NaN payloads survive."""
    dt = np_dtype(t)
    if t == "MPI_LONG_DOUBLE":
        return gen_x80(n, rng, specials)
    if t == "MPI_C_LONG_DOUBLE_COMPLEX":
        x = np.zeros(n, dtype=CX80)
        x["re"], x["im"] = gen_x80(n, rng, specials), gen_x80(n, rng, specials)
        return x
    if t == "MPI_LONG_DOUBLE_INT":
        x = np.zeros(n, dtype=dt)
        x["value"] = gen_x80(n, rng, specials, pool=7)
        x["loc"] = rng.integers(-1000, 1000, n)
        x["pad"] = rng.integers(0, 256, (n, 12), dtype=np.uint8).view("V12").reshape(n)
        return x
    if t in PAIRS:
        x = np.zeros(n, dtype=dt)
        vdt = dt["value"]
        if vdt.kind == "f":
            x["value"] = rng.integers(-8, 8, n).astype(vdt)   # small range -> many ties
        else:
            info = np.iinfo(vdt)
            x["value"] = rng.integers(-4, 4, n).astype(vdt) if rng.random() < 0.5 else \
                rng.integers(info.min, info.max, n, dtype=vdt, endpoint=True)
        x["loc"] = rng.integers(-1000, 1000, n)
        if "pad" in dt.names:
            x["pad"] = rng.integers(-2 ** 15, 2 ** 15, n)
        if specials and n > 4 and vdt.kind == "f":
            x["value"][1] = np.nan
            x["value"][3] = np.nan
        return x
    if t in CPLX:
        w = 4 if t == "MPI_C_FLOAT_COMPLEX" else 8
        ft = np.float32 if w == 4 else np.float64
        re = rng.uniform(-2, 2, n).astype(ft)
        im = rng.uniform(-2, 2, n).astype(ft)
        out = np.empty(n, dtype=np.complex64 if w == 4 else np.complex128)
        out.real, out.imag = re, im
        if specials and n > 8:
            out.real[1], out.imag[1] = np.inf, np.nan
            out.real[2], out.imag[2] = np.nan, np.nan
            out.real[3], out.imag[3] = np.inf, 0.0
            out.real[5], out.imag[5] = 1e38 if w == 4 else 1e308, 1e38 if w == 4 else 1e308
        return out
    if t == "MPI_C_BOOL":
        return rng.integers(0, 2, n).astype(np.uint8)
    if t == "MPIX_C_FLOAT16":
        if op == "MPI_PROD":
            v = rng.uniform(-2, 2, n).astype(np.float16).view(np.uint16)
        else:
            v = rng.uniform(-100, 100, n).astype(np.float16).view(np.uint16)
        if specials:
            k = min(n, len(F16_SPECIALS))
            pos = rng.choice(n, size=k, replace=False) if n > k else np.arange(k)
            v[pos] = np.array(F16_SPECIALS[:k], dtype=np.uint16)
        return v
    if t == "MPI_FLOAT":
        v = rng.uniform(-1, 1, n).astype(np.float32)
        if op == "MPI_PROD":
            v = rng.uniform(-2, 2, n).astype(np.float32)
        v = v.view(np.uint32)
        if specials:
            k = min(n, len(F32_SPECIALS))
            pos = rng.choice(n, size=k, replace=False) if n > k else np.arange(k)
            v[pos] = np.array(F32_SPECIALS[:k], dtype=np.uint32)
        return v.view(np.float32)
    if t == "MPI_DOUBLE":
        v = rng.uniform(-1, 1, n).view(np.uint64)
        if specials:
            k = min(n, len(F64_SPECIALS))
            pos = rng.choice(n, size=k, replace=False) if n > k else np.arange(k)
            v[pos] = np.array(F64_SPECIALS[:k], dtype=np.uint64)
        return v.view(np.float64)
    # integers (incl. MPI_BYTE): full range -> wraparound exercised; logical ops get many zeros
    info = np.iinfo(dt)
    if op in ("MPI_LAND", "MPI_LOR", "MPI_LXOR"):
        v = rng.integers(-1, 2, n).astype(np.int64)
        v = np.where(v < 0, info.max, v).astype(dt)
        return v
    v = rng.integers(info.min, info.max, n, dtype=dt, endpoint=True)
    if specials and n >= 4:
        v[0], v[1] = info.min, info.max
    return v


def to_bytes(a: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(a).view(np.uint8).reshape(-1)

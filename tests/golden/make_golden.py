#!/usr/bin/env python3
"""Generate the golden fixtures for MPI_Reduce_local parity.

Two fixture families, both DATA (inputs + expected outputs), no reference
source:

1. kat_reference.npz / kat_reference.json -- the reference's own
   known-answer tests, evaluated for rank counts p in {2, 3, 8}:
     * test/mpi/coll/allred.c:160-300 closed forms (sum_test1 `sol = i*size`,
       prod_test1 `sol = i^size`, max_test1 `i+size-1`, min_test1 `i`,
       lor/lxor/land/bor/band/bxor const tests, maxloc/minloc struct tests)
       over the type sets of allred.c:302-397 (set1 integers, set2 + float
       and double, set3 MPI_BYTE, set4 C complex, set5 _Bool) at the
       reference default count 10 (allred.c:390) and a ragged count 257;
     * the 3-element tests of test/mpi/coll/opsum.c:50-120,240-262,
       opmax.c:40-170, opmin.c:40-170, opprod.c:50-120 (char, signed char,
       unsigned char, long long) and their long double blocks
       (opsum.c:203-232, opmax.c:113-144, opmin.c:113-144, opprod.c:257-287,
       oplxor.c:196-232, opmaxloc.c:265-310, opminloc.c:222-262), plus
       allred.c's long double _Complex set4 member (:333-345).
     Long double values are x87 80-bit encodings in a 16-byte slot, padding 0.
   An Allreduce over p ranks equals the fold acc = in_0;
   acc = Reduce_local(in_r, acc) for r = 1..p-1 (every op here is
   commutative and the KAT values make every fold order exact), so each case
   stores the p rank buffers and the closed-form solution.

2. probe_survey.json -- reference outputs recorded in SURVEY.md §7 / §8c,
   probed from the reference's own src/mpi/coll/op/op{sum,max,min,prod,land,
   lxor}.c compiled in the survey container (bit patterns, inout = a,
   in = b).

Usage:  python tests/golden/make_golden.py   (deterministic; rewrites files)
"""
from __future__ import annotations

import json
import hashlib
import os
import struct

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

# (MPI name, handle, numpy dtype or struct spec)
SET1 = [  # allred.c:345-355 test_types_set1 (+ set_mpi_2_2_integer, set_mpi_3_0_integer)
    ("MPI_INT", 0x4C000405, "i4"), ("MPI_LONG", 0x4C000807, "i8"), ("MPI_SHORT", 0x4C000203, "i2"),
    ("MPI_UNSIGNED_SHORT", 0x4C000204, "u2"), ("MPI_UNSIGNED", 0x4C000406, "u4"),
    ("MPI_UNSIGNED_LONG", 0x4C000808, "u8"), ("MPI_UNSIGNED_CHAR", 0x4C000102, "u1"),
    ("MPI_INT8_T", 0x4C000137, "i1"), ("MPI_INT16_T", 0x4C000238, "i2"), ("MPI_INT32_T", 0x4C000439, "i4"),
    ("MPI_INT64_T", 0x4C00083A, "i8"), ("MPI_UINT8_T", 0x4C00013B, "u1"), ("MPI_UINT16_T", 0x4C00023C, "u2"),
    ("MPI_UINT32_T", 0x4C00043D, "u4"), ("MPI_UINT64_T", 0x4C00083E, "u8"), ("MPI_AINT", 0x4C000843, "i8"),
    ("MPI_OFFSET", 0x4C000844, "i8"), ("MPI_COUNT", 0x4C000845, "i8"),
]
SET2 = SET1 + [("MPI_FLOAT", 0x4C00040A, "f4"), ("MPI_DOUBLE", 0x4C00080B, "f8")]
SET3 = [("MPI_BYTE", 0x4C00010D, "u1")]
SET4 = [("MPI_C_FLOAT_COMPLEX", 0x4C000840, "c8"), ("MPI_C_DOUBLE_COMPLEX", 0x4C001041, "c16")]
SET5 = [("MPI_C_BOOL", 0x4C00013F, "b1")]
SET4_LD = [("MPI_C_LONG_DOUBLE_COMPLEX", 0x4C002042, "cx80")]

# x87 extended encodings (little-endian significand with explicit integer bit,
# sign + 15-bit exponent, 6 padding bytes)
X80 = np.dtype([("m", "<u8"), ("se", "<u2"), ("pad", "V6")])
CX80 = np.dtype([("re", X80), ("im", X80)])
LDINT = np.dtype([("a", X80), ("b", "<i4"), ("pad", "V12")])


def x80_of_int(v):
    """(significand, sign/exponent) of an integer exactly representable in 64 bits of significand."""
    v = int(v)
    sgn = 0x8000 if v < 0 else 0
    n = abs(v)
    if n == 0:
        return 0, sgn
    k = n.bit_length() - 1
    m = n << (63 - k) if k <= 63 else n >> (k - 63)
    assert (m << max(0, k - 63)) == n or k <= 63, v
    return m, sgn | (16383 + k)


def x80_arr(vals):
    out = np.zeros(len(vals), dtype=X80)
    for i, v in enumerate(vals):
        out["m"][i], out["se"][i] = x80_of_int(v)
    return out


def cx80_arr(vals):
    out = np.zeros(len(vals), dtype=CX80)
    out["re"] = x80_arr(vals)
    out["im"] = x80_arr([0] * len(vals))
    return out

OPS = {"MPI_MAX": 0x58000001, "MPI_MIN": 0x58000002, "MPI_SUM": 0x58000003, "MPI_PROD": 0x58000004,
       "MPI_LAND": 0x58000005, "MPI_BAND": 0x58000006, "MPI_LOR": 0x58000007, "MPI_BOR": 0x58000008,
       "MPI_LXOR": 0x58000009, "MPI_BXOR": 0x5800000A, "MPI_MINLOC": 0x5800000B, "MPI_MAXLOC": 0x5800000C}

# MAXLOC/MINLOC struct layouts on x86-64 (allred.c:19-38)
PAIRS = [
    ("MPI_2INT", 0x4C000816, np.dtype([("a", "<i4"), ("b", "<i4")])),
    ("MPI_LONG_INT", 0x8C000002, np.dtype({"names": ["a", "b"], "formats": ["<i8", "<i4"], "offsets": [0, 8], "itemsize": 16})),
    ("MPI_SHORT_INT", 0x8C000003, np.dtype({"names": ["a", "b"], "formats": ["<i2", "<i4"], "offsets": [0, 4], "itemsize": 8})),
    ("MPI_FLOAT_INT", 0x8C000000, np.dtype({"names": ["a", "b"], "formats": ["<f4", "<i4"], "offsets": [0, 4], "itemsize": 8})),
    ("MPI_DOUBLE_INT", 0x8C000001, np.dtype({"names": ["a", "b"], "formats": ["<f8", "<i4"], "offsets": [0, 8], "itemsize": 16})),
]

NP = {"i1": np.int8, "u1": np.uint8, "i2": np.int16, "u2": np.uint16, "i4": np.int32, "u4": np.uint32,
      "i8": np.int64, "u8": np.uint64, "f4": np.float32, "f8": np.float64, "c8": np.complex64,
      "c16": np.complex128, "b1": np.bool_}


def cast(vals, code):
    """Python ints/floats -> array of the C type with C conversion semantics (integer wrap)."""
    t = NP[code]
    if code in ("f4", "f8", "c8", "c16"):
        return np.array(vals, dtype=t)
    if code == "b1":
        return np.array([bool(v) for v in vals], dtype=np.bool_)
    bits = np.dtype(t).itemsize * 8
    u = np.array([int(v) % (1 << bits) for v in vals], dtype=np.dtype(t).str.replace("i", "u"))
    return u.view(t)


def power_seq(i, n, code):
    """SET_INDEX_POWER (allred.c:85-93): arr = 1; n times arr *= i, in type arithmetic."""
    t = NP[code]
    if code in ("f4", "f8", "c8", "c16"):
        acc = t(1)
        for _ in range(n):
            acc = t(acc * t(i))
        return acc
    bits = np.dtype(t).itemsize * 8
    acc = 1
    for _ in range(n):
        acc = (acc * i) % (1 << bits)
    return acc


cases = []   # (id, op, type name, handle, p, count, rank buffers (p, bytes), solution bytes)


def add(cid, op, tname, handle, ranks, sol):
    ranks = [np.ascontiguousarray(r) for r in ranks]
    cases.append({"id": cid, "op": op, "datatype": tname, "handle": handle, "p": len(ranks),
                  "count": int(ranks[0].shape[0]), "ranks": np.stack([r.view(np.uint8) for r in ranks]),
                  "sol": np.ascontiguousarray(sol).view(np.uint8)})


def allred_cases(p, count):
    idx = list(range(count))
    for tname, h, code in SET2 + SET4:
        # sum_test1 (allred.c:160-167): in = i, sol = i*size
        add(f"allred_sum1_{tname}_p{p}_n{count}", "MPI_SUM", tname, h,
            [cast(idx, code) for _ in range(p)], cast([i * p for i in idx], code) if code[0] not in "fc"
            else np.array([NP[code](i * p) for i in idx], dtype=NP[code]))
        # prod_test1 (allred.c:169-176): sol = i^size
        add(f"allred_prod1_{tname}_p{p}_n{count}", "MPI_PROD", tname, h,
            [cast(idx, code) for _ in range(p)],
            cast([power_seq(i, p, code) for i in idx], code) if code[0] not in "fc"
            else np.array([power_seq(i, p, code) for i in idx], dtype=NP[code]))
    for tname, h, code in SET4_LD:
        # allred.c set4 long double _Complex (:333-345): sum_test1 / prod_test1
        add(f"allred_sum1_{tname}_p{p}_n{count}", "MPI_SUM", tname, h,
            [cx80_arr(idx) for _ in range(p)], cx80_arr([i * p for i in idx]))
        add(f"allred_prod1_{tname}_p{p}_n{count}", "MPI_PROD", tname, h,
            [cx80_arr(idx) for _ in range(p)], cx80_arr([i ** p for i in idx]))
    for tname, h, code in SET2:
        # max_test1 / min_test1 (allred.c:178-194): in = i + rank.  The closed
        # form assumes no wrap (true at the reference's count 10); skip 1-byte
        # types at the ragged count, where i + rank wraps.
        if code[1:] == "1" and count + p - 1 > 127:
            continue
        ranks = [cast([i + r for i in idx], code) for r in range(p)]
        add(f"allred_max1_{tname}_p{p}_n{count}", "MPI_MAX", tname, h, ranks, cast([i + p - 1 for i in idx], code))
        add(f"allred_min1_{tname}_p{p}_n{count}", "MPI_MIN", tname, h, ranks, cast(idx, code))

    def const(name, op, types, val_of_rank, sol):
        for tname, h, code in types:
            add(f"allred_{name}_{tname}_p{p}_n{count}", op, tname, h,
                [cast([val_of_rank(r, code)] * count, code) for r in range(p)], cast([sol(code)] * count, code))

    def ones(code):  # ~0 in the type
        return -1 if code[0] == "i" else (1 << (np.dtype(NP[code]).itemsize * 8)) - 1

    logical = SET1 + SET5
    const("lor1", "MPI_LOR", logical, lambda r, c: r & 1, lambda c: int(p > 1))          # allred.c:205-206
    const("lor2", "MPI_LOR", logical, lambda r, c: 0, lambda c: 0)                       # :207-208
    const("lxor1", "MPI_LXOR", logical, lambda r, c: int(r == 1), lambda c: int(p > 1))  # :209-210
    const("lxor2", "MPI_LXOR", logical, lambda r, c: 0, lambda c: 0)                     # :211-212
    const("lxor3", "MPI_LXOR", logical, lambda r, c: 1, lambda c: p & 1)                 # :213-214
    const("land1", "MPI_LAND", logical, lambda r, c: r & 1, lambda c: 0)                 # :215-216
    const("land2", "MPI_LAND", logical, lambda r, c: 1, lambda c: 1)                     # :217-218
    bitwise = SET1 + SET3
    const("bor1", "MPI_BOR", bitwise, lambda r, c: r & 3, lambda c: (p - 1) if p < 3 else 3)  # :219-220
    const("bxor1", "MPI_BXOR", bitwise, lambda r, c: int(r == 1) * 0xF0, lambda c: int(p > 1) * 0xF0)  # :221-222
    const("bxor2", "MPI_BXOR", bitwise, lambda r, c: 0, lambda c: 0)                     # :223-224
    const("bxor3", "MPI_BXOR", bitwise, lambda r, c: ones(c), lambda c: ones(c) if p & 1 else 0)  # :225-226
    for tname, h, code in bitwise:
        # band_test1 / band_test2 (allred.c:228-256)
        r1 = [cast(idx, code) if r == p - 1 else cast([ones(code)] * count, code) for r in range(p)]
        add(f"allred_band1_{tname}_p{p}_n{count}", "MPI_BAND", tname, h, r1, cast(idx, code))
        r2 = [cast(idx, code) if r == p - 1 else cast([0] * count, code) for r in range(p)]
        add(f"allred_band2_{tname}_p{p}_n{count}", "MPI_BAND", tname, h, r2, cast([0] * count, code))
    for tname, h, dt in PAIRS:
        # maxloc_test / minloc_test (allred.c:258-282): a = i + rank, b = rank
        ranks = []
        for r in range(p):
            x = np.zeros(count, dtype=dt)
            x["a"] = np.array([i + r for i in idx])
            x["b"] = r
            ranks.append(x)
        smax = np.zeros(count, dtype=dt)
        smax["a"] = np.array([i + p - 1 for i in idx])
        smax["b"] = p - 1
        smin = np.zeros(count, dtype=dt)
        smin["a"] = np.array(idx)
        smin["b"] = 0
        add(f"allred_maxloc_{tname}_p{p}_n{count}", "MPI_MAXLOC", tname, h, ranks, smax)
        add(f"allred_minloc_{tname}_p{p}_n{count}", "MPI_MINLOC", tname, h, ranks, smin)


def opfile_cases(p):
    chars = [("MPI_CHAR", 0x4C000101, "i1"), ("MPI_SIGNED_CHAR", 0x4C000118, "i1"),
             ("MPI_UNSIGNED_CHAR", 0x4C000102, "u1"), ("MPI_LONG_LONG", 0x4C000809, "i8")]
    maxsize = min(p, 5)
    fact = [1, 1, 2, 6, 24, 120]
    for tname, h, code in chars:
        # opsum.c:50-70: in = {1, 0, rank > 0}; sol = {size, 0, size - 1}
        add(f"opsum_{tname}_p{p}", "MPI_SUM", tname, h, [cast([1, 0, int(r > 0)], code) for r in range(p)],
            cast([p, 0, p - 1], code))
        # opmax.c:40-60: in = {1, 0, rank}; sol = {1, 0, size - 1}
        add(f"opmax_{tname}_p{p}", "MPI_MAX", tname, h, [cast([1, 0, r], code) for r in range(p)],
            cast([1, 0, p - 1], code))
        # opmin.c:40-60: in = {1, 0, rank & 0x7f}; sol = {1, 0, 0}
        add(f"opmin_{tname}_p{p}", "MPI_MIN", tname, h, [cast([1, 0, r & 0x7F], code) for r in range(p)],
            cast([1, 0, 0], code))
        # opprod.c:50-70: in = {(rank<maxsize && rank>0) ? rank : 1, 0, rank > 1}; sol = {result[maxsize-1], 0, 0}
        add(f"opprod_{tname}_p{p}", "MPI_PROD", tname, h,
            [cast([r if 0 < r < maxsize else 1, 0, int(r > 1)], code) for r in range(p)],
            cast([fact[maxsize - 1], 0, 0], code))


def opfile_long_double_cases(p):
    """The HAVE_LONG_DOUBLE blocks of the op*.c tests (3 elements)."""
    h, hi = 0x4C00100C, 0x8C000004
    maxsize = min(p, 5)
    fact = [1, 1, 2, 6, 24, 120]
    add(f"opsum_MPI_LONG_DOUBLE_p{p}", "MPI_SUM", "MPI_LONG_DOUBLE", h,       # opsum.c:203-232
        [x80_arr([1, 0, int(r > 0)]) for r in range(p)], x80_arr([p, 0, p - 1]))
    add(f"opmax_MPI_LONG_DOUBLE_p{p}", "MPI_MAX", "MPI_LONG_DOUBLE", h,       # opmax.c:113-144
        [x80_arr([1, 0, r]) for r in range(p)], x80_arr([1, 0, p - 1]))
    add(f"opmin_MPI_LONG_DOUBLE_p{p}", "MPI_MIN", "MPI_LONG_DOUBLE", h,       # opmin.c:113-144
        [x80_arr([1, 0, r]) for r in range(p)], x80_arr([1, 0, 0]))
    add(f"opprod_MPI_LONG_DOUBLE_p{p}", "MPI_PROD", "MPI_LONG_DOUBLE", h,     # opprod.c:257-287
        [x80_arr([r if 0 < r < maxsize else 1, 0, int(r > 0)]) for r in range(p)],
        x80_arr([fact[maxsize - 1], 0, 0]))
    add(f"oplxor_MPI_LONG_DOUBLE_p{p}", "MPI_LXOR", "MPI_LONG_DOUBLE", h,     # oplxor.c:196-232
        [x80_arr([1, 0, int(r > 0)]) for r in range(p)], x80_arr([p % 2, 0, (p - 1) % 2]))
    for op, sol in (("MPI_MAXLOC", [(1, 0), (0, 0), (p - 1, p - 1)]),        # opmaxloc.c:265-310
                    ("MPI_MINLOC", [(1, 0), (0, 0), (0, 0)])):                 # opminloc.c:222-262
        ranks = []
        for r in range(p):
            x = np.zeros(3, dtype=LDINT)
            x["a"] = x80_arr([1, 0, r])
            x["b"] = r
            ranks.append(x)
        want = np.zeros(3, dtype=LDINT)
        want["a"] = x80_arr([v for v, _ in sol])
        want["b"] = [l for _, l in sol]
        add(f"{op[4:].lower()}_MPI_LONG_DOUBLE_INT_p{p}", op, "MPI_LONG_DOUBLE_INT", hi, ranks, want)


def f32(x):
    return struct.unpack("<I", struct.pack("<f", x))[0]


def probes():
    """SURVEY.md §7 'Hard parts' and §8c 'Oracle' probe outputs, as bit patterns."""
    nan = 0x7FC00000
    out = []
    a = [f32(1.5), 0x80000000, nan, f32(3.0)]
    b = [f32(2.25), 0x00000000, f32(1.0), nan]
    out.append({"id": "survey_sum_f32", "op": "MPI_SUM", "datatype": "MPI_FLOAT", "width": 4,
                "inout": a, "in": b, "expect": [f32(3.75), 0x00000000, nan, nan], "source": "SURVEY.md §8c row 1"})
    out.append({"id": "survey_max_f32", "op": "MPI_MAX", "datatype": "MPI_FLOAT", "width": 4,
                "inout": a, "in": b, "expect": [f32(2.25), 0x00000000, f32(1.0), nan], "source": "SURVEY.md §8c row 1"})
    # MAX/MIN NaN and signed-zero semantics (SURVEY.md §7 hard parts)
    x = f32(2.0)
    out.append({"id": "survey_max_nan_zero_f32", "op": "MPI_MAX", "datatype": "MPI_FLOAT", "width": 4,
                "inout": [nan, x, 0x00000000, 0x80000000], "in": [x, nan, 0x80000000, 0x00000000],
                "expect": [x, nan, 0x80000000, 0x00000000], "source": "SURVEY.md §7"})
    out.append({"id": "survey_min_nan_zero_f32", "op": "MPI_MIN", "datatype": "MPI_FLOAT", "width": 4,
                "inout": [nan, x, 0x00000000, 0x80000000], "in": [x, nan, 0x80000000, 0x00000000],
                "expect": [x, nan, 0x80000000, 0x00000000], "source": "SURVEY.md §7 (MIN symmetric)"})
    # fp16: 1 + 2^-10 = 1.00098 (0x3c01), 65504 + 32 = inf (0x7c00), MAX(3, -2) = 3, PROD(0.1, 0.3) = 0x27ae
    out.append({"id": "survey_sum_f16", "op": "MPI_SUM", "datatype": "MPIX_C_FLOAT16", "width": 2,
                "inout": [0x3C00, 0x7BFF], "in": [0x1400, 0x5000], "expect": [0x3C01, 0x7C00], "source": "SURVEY.md §8c"})
    out.append({"id": "survey_max_f16", "op": "MPI_MAX", "datatype": "MPIX_C_FLOAT16", "width": 2,
                "inout": [0x4200], "in": [0xC000], "expect": [0x4200], "source": "SURVEY.md §8c"})
    out.append({"id": "survey_prod_f16", "op": "MPI_PROD", "datatype": "MPIX_C_FLOAT16", "width": 2,
                "inout": [0x2E66], "in": [0x34CD], "expect": [0x27AE], "source": "SURVEY.md §8c"})
    # integer wraparound: INT_MAX + 1 -> INT_MIN; int8 127 + 1 -> -128; int64 LLONG_MAX * 2 -> -2
    out.append({"id": "survey_sum_int_wrap", "op": "MPI_SUM", "datatype": "MPI_INT", "width": 4,
                "inout": [0x7FFFFFFF], "in": [1], "expect": [0x80000000], "source": "SURVEY.md §8c"})
    out.append({"id": "survey_sum_int8_wrap", "op": "MPI_SUM", "datatype": "MPI_INT8_T", "width": 1,
                "inout": [0x7F], "in": [1], "expect": [0x80], "source": "SURVEY.md §8c"})
    out.append({"id": "survey_prod_int64_wrap", "op": "MPI_PROD", "datatype": "MPI_INT64_T", "width": 8,
                "inout": [0x7FFFFFFFFFFFFFFF], "in": [2], "expect": [0xFFFFFFFFFFFFFFFE], "source": "SURVEY.md §8c"})
    # LXOR on float: 0 xor 2.5 -> 1.0
    out.append({"id": "survey_lxor_f32", "op": "MPI_LXOR", "datatype": "MPI_FLOAT", "width": 4,
                "inout": [0x00000000], "in": [f32(2.5)], "expect": [f32(1.0)], "source": "SURVEY.md §8c"})
    # LAND on MPI_FLOAT: check_dtype passes, kernel sets op_errno (MPI_ERR_OP), inout untouched
    out.append({"id": "survey_land_f32_errno", "op": "MPI_LAND", "datatype": "MPI_FLOAT", "width": 4,
                "inout": [f32(1.0)], "in": [f32(1.0)], "expect": [f32(1.0)], "expect_rc": 9,
                "source": "SURVEY.md §8a a8 / §8c"})
    # MPI_BYTE with SUM sets op_errno / fails check_dtype
    out.append({"id": "survey_sum_byte_err", "op": "MPI_SUM", "datatype": "MPI_BYTE", "width": 1,
                "inout": [1], "in": [2], "expect": [1], "expect_rc": 9, "source": "SURVEY.md §8c"})
    return out


def main():
    for p in (2, 3, 8):
        for count in (10, 257):
            allred_cases(p, count)
        opfile_cases(p)
        opfile_long_double_cases(p)
    arrays, manifest = {}, []
    for k, c in enumerate(cases):
        arrays[f"c{k}_ranks"] = c["ranks"]
        arrays[f"c{k}_sol"] = c["sol"]
        manifest.append({"key": f"c{k}", "id": c["id"], "op": c["op"], "op_handle": OPS[c["op"]],
                         "datatype": c["datatype"], "handle": c["handle"], "p": c["p"], "count": c["count"],
                         "elem_bytes": int(c["sol"].size // c["count"])})
    npz = os.path.join(HERE, "kat_reference.npz")
    np.savez_compressed(npz, **arrays)
    digest = hashlib.sha256(open(npz, "rb").read()).hexdigest()
    with open(os.path.join(HERE, "kat_reference.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "sha256_npz": digest,
                   "source": "test/mpi/coll/allred.c, opsum.c, opmax.c, opmin.c, opprod.c, oplxor.c, opmaxloc.c, "
                             "opminloc.c closed forms",
                   "cases": manifest}, f, indent=0)
    with open(os.path.join(HERE, "probe_survey.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py",
                   "note": "bit patterns; inout = a (the reference's a[i]), in = b", "cases": probes()}, f, indent=1)
    print(f"{len(cases)} KAT cases, npz {os.path.getsize(npz)} bytes")


if __name__ == "__main__":
    main()

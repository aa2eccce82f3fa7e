/*
 * op_oracle.c -- CPU ORACLE for MPI_Reduce_local.  TEST INFRASTRUCTURE ONLY.
 *
 * This file is the parity checker for the MI355X implementation in
 * mpich-pip_amd/.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product library never links or calls it.
 *
 * It restates, in plain C compiled by gcc -O2 on x86-64 (MPICH's default
 * --enable-fast=O2, configure.ac:399-408), the reference's algorithm for the
 * hot path:
 *   - MPI_Reduce_local's validation block    reduce_local.c:166-191
 *       MPIR_ERRTEST_OP                       mpir_err.h:499-510
 *       check_dtype via MPIR_Op_check_dtype_table[op & 0xf]  reduce_local.c:180
 *       MPIR_ERRTEST_ALIAS_COLL               mpir_err.h:277-285
 *       MPIR_ERRTEST_NAMED_BUF_INPLACE        mpir_err.h:440-446
 *   - MPIR_Reduce_local                       reduce_local.c:35-122
 *       count == 0 early exit :48, op_errno reset/read :51-59,107-117
 *   - the per-(op, type) loops `a[i] = OP(a[i], b[i])`, a = inoutvec,
 *     b = invec                               mpir_op_util.h:48-55
 *       MPIR_LSUM  opsum.c:15      MPIR_LPROD opprod.c:15
 *       MPL_MAX / MPL_MIN          mpl_base.h:124-125  (opmax.c:20, opmin.c:19)
 *       MPIR_LLAND opland.c:17     MPIR_LLOR oplor.c:17   MPIR_LLXOR oplxor.c:17
 *       MPIR_LBAND opband.c:16     MPIR_LBOR opbor.c:16   MPIR_LBXOR opbxor.c:16
 *       MAXLOC / MINLOC            opmaxloc.c:48-59, opminloc.c:48-59
 *   - type groups per op                      mpir_op_util.h:263-364, op*.c
 *
 * Build configuration mirrored: x86-64, --disable-fortran, --disable-cxx,
 * with long double (MPI_LONG_DOUBLE, MPI_C_LONG_DOUBLE_COMPLEX,
 * MPI_LONG_DOUBLE_INT; configure.ac:3456-3460,3486-3491,3699-3702): those
 * loops are the reference's own shape on `long double`, so gcc compiles them
 * to x87 instructions exactly as it compiles op*.c.  MPIX_C_FLOAT16 exists only when the
 * C compiler has _Float16 (configure.ac:3703-3705); gcc 11 on x86 does not,
 * so the reference's fp16 path is the AMD clang build.  clang lowers each
 * _Float16 operation on x86-64 (no AVX512-FP16) as extend-to-float, float
 * op, truncate-to-half (compiler-rt __extendhfsf2 / __truncsfhf2); that
 * lowering is restated bit by bit in h2f()/f2h() below.  Float/double
 * arithmetic is native x86 SSE, i.e. exactly the reference's.
 *
 * Pinned against: the reference's own known-answer tests (tests/golden/,
 * closed forms from test/mpi/coll/allred.c, opprod.c, ...) and the reference
 * outputs recorded in SURVEY.md §8c (probed from the reference's op*.c).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <complex.h>

/* ---- handle values (mpi.h.in:310-325, configure.ac:3442-3705) ---------- */
#define O_MPI_OP_NULL 0x18000000
#define O_MAX 0x58000001
#define O_MIN 0x58000002
#define O_SUM 0x58000003
#define O_PROD 0x58000004
#define O_LAND 0x58000005
#define O_BAND 0x58000006
#define O_LOR 0x58000007
#define O_BOR 0x58000008
#define O_LXOR 0x58000009
#define O_BXOR 0x5800000a
#define O_MINLOC 0x5800000b
#define O_MAXLOC 0x5800000c
#define O_REPLACE 0x5800000d
#define O_NO_OP 0x5800000e

#define E_SUCCESS 0
#define E_BUFFER 1
#define E_OP 9

enum { K_NONE, K_I8, K_U8, K_I16, K_U16, K_I32, K_U32, K_I64, K_U64, K_F16, K_F32, K_F64,
       K_CF32, K_CF64, K_BOOL, K_P2INT, K_PFLOATINT, K_PLONGINT, K_PSHORTINT, K_PDOUBLEINT,
       K_F80, K_CF80, K_PLDINT };

/* groups */
#define CI 0x001   /* C_INTEGER */
#define CX 0x002   /* C_INTEGER_EXTRA */
#define FI 0x004   /* FORTRAN_INTEGER (AINT/OFFSET/COUNT) */
#define FP 0x008   /* FLOATING_POINT */
#define FX 0x010   /* FLOATING_POINT_EXTRA (_Float16) */
#define LG 0x020   /* LOGICAL (_Bool) */
#define CO 0x040   /* COMPLEX */
#define BY 0x080   /* BYTE */
#define PR 0x100   /* MAXLOC pairs */

static int type_info(int dt, int *grp)
{
    switch ((unsigned) dt) {
    case 0x4c000405: *grp = CI; return K_I32;   /* MPI_INT */
    case 0x4c000807: *grp = CI; return K_I64;   /* MPI_LONG */
    case 0x4c000203: *grp = CI; return K_I16;   /* MPI_SHORT */
    case 0x4c000204: *grp = CI; return K_U16;   /* MPI_UNSIGNED_SHORT */
    case 0x4c000406: *grp = CI; return K_U32;   /* MPI_UNSIGNED */
    case 0x4c000808: *grp = CI; return K_U64;   /* MPI_UNSIGNED_LONG */
    case 0x4c000809: *grp = CI; return K_I64;   /* MPI_LONG_LONG */
    case 0x4c000819: *grp = CI; return K_U64;   /* MPI_UNSIGNED_LONG_LONG */
    case 0x4c000118: *grp = CI; return K_I8;    /* MPI_SIGNED_CHAR */
    case 0x4c000102: *grp = CI; return K_U8;    /* MPI_UNSIGNED_CHAR */
    case 0x4c000137: *grp = CI; return K_I8;    /* MPI_INT8_T */
    case 0x4c000238: *grp = CI; return K_I16;
    case 0x4c000439: *grp = CI; return K_I32;
    case 0x4c00083a: *grp = CI; return K_I64;
    case 0x4c00013b: *grp = CI; return K_U8;    /* MPI_UINT8_T */
    case 0x4c00023c: *grp = CI; return K_U16;
    case 0x4c00043d: *grp = CI; return K_U32;
    case 0x4c00083e: *grp = CI; return K_U64;
    case 0x4c000101: *grp = CX; return K_I8;    /* MPI_CHAR (signed on x86-64) */
    case 0x4c000843: *grp = FI; return K_I64;   /* MPI_AINT */
    case 0x4c000844: *grp = FI; return K_I64;   /* MPI_OFFSET */
    case 0x4c000845: *grp = FI; return K_I64;   /* MPI_COUNT */
    case 0x4c00040a: *grp = FP; return K_F32;   /* MPI_FLOAT */
    case 0x4c00080b: *grp = FP; return K_F64;   /* MPI_DOUBLE */
    case 0x4c000246: *grp = FX; return K_F16;   /* MPIX_C_FLOAT16 */
    case 0x4c00013f: *grp = LG; return K_BOOL;  /* MPI_C_BOOL */
    case 0x4c000840: *grp = CO; return K_CF32;  /* MPI_C_FLOAT_COMPLEX */
    case 0x4c001041: *grp = CO; return K_CF64;  /* MPI_C_DOUBLE_COMPLEX */
    case 0x4c00010d: *grp = BY; return K_U8;    /* MPI_BYTE */
    case 0x4c000816: *grp = PR; return K_P2INT;
    case 0x8c000000: *grp = PR; return K_PFLOATINT;
    case 0x8c000002: *grp = PR; return K_PLONGINT;
    case 0x8c000003: *grp = PR; return K_PSHORTINT;
    case 0x8c000001: *grp = PR; return K_PDOUBLEINT;
    case 0x4c00100c: *grp = FP; return K_F80;    /* MPI_LONG_DOUBLE */
    case 0x4c002042: *grp = CO; return K_CF80;   /* MPI_C_LONG_DOUBLE_COMPLEX */
    case 0x8c000004: *grp = PR; return K_PLDINT; /* MPI_LONG_DOUBLE_INT */
    default: *grp = 0; return K_NONE;
    }
}

#define NUM (CI | CX | FI | FP | FX)
#define INTS (CI | CX | FI)
/* index = op & 0xf; compute groups per op (the switch cases in op*.c) */
static const int compute_grp[15] = { 0, NUM, NUM, NUM | CO, NUM | CO, INTS | LG, INTS | BY, INTS | LG,
    INTS | BY, INTS | LG | FP | FX, INTS | BY, PR, PR, -1, -1 };
/* check_dtype groups; LAND/LOR also accept floats (opland.c:105-106, oplor.c:105-106) */
static const int check_grp[15] = { 0, NUM, NUM, NUM | CO, NUM | CO, INTS | LG | FP | FX, INTS | BY,
    INTS | LG | FP | FX, INTS | BY, INTS | LG | FP | FX, INTS | BY, PR, PR, -1, -1 };

/* ---- _Float16 as clang lowers it on x86-64 (compiler-rt fp_extend / fp_trunc) */
static float h2f(uint16_t h)
{
    uint32_t sign = (uint32_t) (h & 0x8000) << 16, e = (h >> 10) & 0x1f, m = h & 0x3ff, r;
    float f;
    if (e == 0x1f)
        r = sign | 0x7f800000u | (m << 13);     /* inf / NaN: payload and quiet bit shifted */
    else if (e == 0) {
        if (m == 0)
            r = sign;
        else {                                  /* subnormal: normalize */
            int sh = 0;
            while (!(m & 0x400)) {
                m <<= 1;
                sh++;
            }
            m &= 0x3ff;
            r = sign | ((uint32_t) (127 - 15 + 1 - sh) << 23) | (m << 13);
        }
    } else
        r = sign | ((e - 15 + 127) << 23) | (m << 13);
    memcpy(&f, &r, 4);
    return f;
}

static uint16_t f2h(float f)    /* round to nearest even */
{
    uint32_t x, sign, ax;
    memcpy(&x, &f, 4);
    sign = (x >> 16) & 0x8000;
    ax = x & 0x7fffffffu;
    if (ax > 0x7f800000u)       /* NaN: qNaN bit set, payload truncated */
        return (uint16_t) (sign | 0x7c00 | 0x200 | ((ax >> 13) & 0x1ff));
    if (ax >= 0x477ff000u)      /* >= 65520: overflow to inf (or inf itself) */
        return (uint16_t) (sign | 0x7c00);
    if (ax >= 0x38800000u) {    /* normal half */
        uint32_t m = ax - ((127 - 15) << 23);
        uint32_t res = m >> 13, rem = m & 0x1fff;
        if (rem > 0x1000 || (rem == 0x1000 && (res & 1)))
            res++;
        return (uint16_t) (sign | res);
    }
    if (ax < 0x33000000u)       /* < 2^-25: rounds to zero */
        return (uint16_t) sign;
    {                           /* subnormal half: unit 2^-24 */
        uint32_t e = ax >> 23, m = (ax & 0x7fffff) | 0x800000;
        int sh = 126 - (int) e;         /* value / 2^-24 = m * 2^(e - 126) */
        uint32_t res = m >> sh, rem = m & ((1u << sh) - 1), half = 1u << (sh - 1);
        if (rem > half || (rem == half && (res & 1)))
            res++;
        return (uint16_t) (sign | res);
    }
}

/* ---- the loops ---------------------------------------------------------- */
#define LSUM(a, b) ((a) + (b))
#define LPROD(a, b) ((a) * (b))
#define LMAX(a, b) (((a) > (b)) ? (a) : (b))
#define LMIN(a, b) (((a) < (b)) ? (a) : (b))
#define LLAND(a, b) ((a) && (b))
#define LLOR(a, b) ((a) || (b))
#define LLXOR(a, b) (((a) && (!(b))) || ((!(a)) && (b)))
#define LBAND(a, b) ((a) & (b))
#define LBOR(a, b) ((a) | (b))
#define LBXOR(a, b) ((a) ^ (b))

#define LOOP(T, F) do { T *restrict a = (T *) io; const T *restrict b = (const T *) in; \
        for (i = 0; i < len; i++) a[i] = F(a[i], b[i]); } while (0)

/* signed overflow wraps in the reference's compiled code; compute integer
 * SUM/PROD in the unsigned type of the same width to stay defined in C */
#define ULOOP(ST, UT, F) do { ST *restrict a = (ST *) io; const ST *restrict b = (const ST *) in; \
        for (i = 0; i < len; i++) a[i] = (ST) (UT) F((UT) a[i], (UT) b[i]); } while (0)

/* x86 SSE NaN rule (Intel SDM vol. 1, 4.8.3.5, Table 4-7): with a NaN operand
 * the result is the FIRST source operand if it is a NaN, else the second,
 * quieted.  The reference's loops put a[i] (inout) first -- gcc -O2:
 * `movss a; addss b`, clang -O2: `addps b, a` (probed) -- so the result is
 * quiet(a) if a is NaN, else quiet(b).  Made explicit here so the oracle does
 * not depend on which operand order gcc picks for the helper calls below. */
static float f_quiet(float x)
{
    uint32_t u;
    memcpy(&u, &x, 4);
    u |= 0x00400000u;
    memcpy(&x, &u, 4);
    return x;
}

static double d_quiet(double x)
{
    uint64_t u;
    memcpy(&u, &x, 8);
    u |= 0x0008000000000000ull;
    memcpy(&x, &u, 8);
    return x;
}

#define NANRULE(Q, F) ((a[i] != a[i]) ? Q(a[i]) : (b[i] != b[i]) ? Q(b[i]) : F(a[i], b[i]))
#define FLOOP(T, Q, F) do { T *restrict a = (T *) io; const T *restrict b = (const T *) in; \
        for (i = 0; i < len; i++) a[i] = NANRULE(Q, F); } while (0)

static float h_arith(float x, float y, int prod)
{
    if (x != x)
        return f_quiet(x);
    if (y != y)
        return f_quiet(y);
    return prod ? x * y : x + y;
}

#define HLOOP_ARITH(PROD) do { uint16_t *a = (uint16_t *) io; const uint16_t *b = (const uint16_t *) in; \
        for (i = 0; i < len; i++) a[i] = f2h(h_arith(h2f(a[i]), h2f(b[i]), PROD)); } while (0)
/* MPL_MAX on _Float16: compare the promoted values, select the original bits */
#define HLOOP_SEL(CMP) do { uint16_t *a = (uint16_t *) io; const uint16_t *b = (const uint16_t *) in; \
        for (i = 0; i < len; i++) a[i] = (h2f(a[i]) CMP h2f(b[i])) ? a[i] : b[i]; } while (0)
#define HLOOP_LXOR() do { uint16_t *a = (uint16_t *) io; const uint16_t *b = (const uint16_t *) in; \
        for (i = 0; i < len; i++) a[i] = LLXOR(h2f(a[i]) != 0.0f, h2f(b[i]) != 0.0f) ? 0x3c00 : 0; } while (0)

#define LOC_LOOP(VT, LT, CMP, CMPE) do {                                           \
        typedef struct { VT value; LT loc; } pair_t;                                 \
        pair_t *a = (pair_t *) io; const pair_t *b = (const pair_t *) in;            \
        for (i = 0; i < len; i++) {                                                  \
            if (a[i].value CMP b[i].value) { a[i].value = b[i].value; a[i].loc = b[i].loc; } \
            else if (a[i].value CMPE b[i].value) a[i].loc = LMIN(a[i].loc, b[i].loc); \
        } } while (0)

/* returns 0, or E_OP for the compute switch's `default:` branch */
static int apply(int opidx, int kind, const void *in, void *io, int len)
{
    int i;
    switch (opidx) {
    case 3:    /* SUM */
        switch (kind) {
        case K_I8: ULOOP(int8_t, uint8_t, LSUM); return 0;
        case K_U8: LOOP(uint8_t, LSUM); return 0;
        case K_I16: ULOOP(int16_t, uint16_t, LSUM); return 0;
        case K_U16: LOOP(uint16_t, LSUM); return 0;
        case K_I32: ULOOP(int32_t, uint32_t, LSUM); return 0;
        case K_U32: LOOP(uint32_t, LSUM); return 0;
        case K_I64: ULOOP(int64_t, uint64_t, LSUM); return 0;
        case K_U64: LOOP(uint64_t, LSUM); return 0;
        case K_F16: HLOOP_ARITH(0); return 0;
        case K_F32: FLOOP(float, f_quiet, LSUM); return 0;
        case K_F64: FLOOP(double, d_quiet, LSUM); return 0;
        case K_CF32: LOOP(float _Complex, LSUM); return 0;
        case K_CF64: LOOP(double _Complex, LSUM); return 0;
        case K_F80: LOOP(long double, LSUM); return 0;
        case K_CF80: LOOP(long double _Complex, LSUM); return 0;
        }
        break;
    case 4:    /* PROD */
        switch (kind) {
        case K_I8: ULOOP(int8_t, uint8_t, LPROD); return 0;
        case K_U8: LOOP(uint8_t, LPROD); return 0;
        case K_I16: ULOOP(int16_t, uint32_t, LPROD); return 0;
        case K_U16: ULOOP(uint16_t, uint32_t, LPROD); return 0;
        case K_I32: ULOOP(int32_t, uint32_t, LPROD); return 0;
        case K_U32: LOOP(uint32_t, LPROD); return 0;
        case K_I64: ULOOP(int64_t, uint64_t, LPROD); return 0;
        case K_U64: LOOP(uint64_t, LPROD); return 0;
        case K_F16: HLOOP_ARITH(1); return 0;
        case K_F32: FLOOP(float, f_quiet, LPROD); return 0;
        case K_F64: FLOOP(double, d_quiet, LPROD); return 0;
        case K_CF32: LOOP(float _Complex, LPROD); return 0;
        case K_CF64: LOOP(double _Complex, LPROD); return 0;
        case K_F80: LOOP(long double, LPROD); return 0;
        case K_CF80: LOOP(long double _Complex, LPROD); return 0;
        }
        break;
    case 1:    /* MAX */
    case 2:    /* MIN */
#define SEL(F) switch (kind) { \
        case K_I8: LOOP(int8_t, F); return 0; case K_U8: LOOP(uint8_t, F); return 0; \
        case K_I16: LOOP(int16_t, F); return 0; case K_U16: LOOP(uint16_t, F); return 0; \
        case K_I32: LOOP(int32_t, F); return 0; case K_U32: LOOP(uint32_t, F); return 0; \
        case K_I64: LOOP(int64_t, F); return 0; case K_U64: LOOP(uint64_t, F); return 0; \
        case K_F32: LOOP(float, F); return 0; case K_F64: LOOP(double, F); return 0; \
        case K_F80: LOOP(long double, F); return 0; }
        if (opidx == 1) {
            if (kind == K_F16) { HLOOP_SEL(>); return 0; }
            SEL(LMAX)
        } else {
            if (kind == K_F16) { HLOOP_SEL(<); return 0; }
            SEL(LMIN)
        }
        break;
#undef SEL
    case 5: case 7: case 9:     /* LAND, LOR, LXOR */
#define LOG(F) switch (kind) { \
        case K_I8: LOOP(int8_t, F); return 0; case K_U8: LOOP(uint8_t, F); return 0; \
        case K_I16: LOOP(int16_t, F); return 0; case K_U16: LOOP(uint16_t, F); return 0; \
        case K_I32: LOOP(int32_t, F); return 0; case K_U32: LOOP(uint32_t, F); return 0; \
        case K_I64: LOOP(int64_t, F); return 0; case K_U64: LOOP(uint64_t, F); return 0; \
        case K_BOOL: LOOP(_Bool, F); return 0; }
        if (opidx == 5) { LOG(LLAND) }
        else if (opidx == 7) { LOG(LLOR) }
        else {
            if (kind == K_F16) { HLOOP_LXOR(); return 0; }
            if (kind == K_F32) { LOOP(float, LLXOR); return 0; }
            if (kind == K_F64) { LOOP(double, LLXOR); return 0; }
            if (kind == K_F80) { LOOP(long double, LLXOR); return 0; }
            LOG(LLXOR)
        }
        break;
#undef LOG
    case 6: case 8: case 10:    /* BAND, BOR, BXOR */
#define BIT(F) switch (kind) { \
        case K_I8: case K_U8: LOOP(uint8_t, F); return 0; \
        case K_I16: case K_U16: LOOP(uint16_t, F); return 0; \
        case K_I32: case K_U32: LOOP(uint32_t, F); return 0; \
        case K_I64: case K_U64: LOOP(uint64_t, F); return 0; }
        if (opidx == 6) { BIT(LBAND) }
        else if (opidx == 8) { BIT(LBOR) }
        else { BIT(LBXOR) }
        break;
#undef BIT
    case 12:   /* MAXLOC: opmaxloc.c:48-59 */
        switch (kind) {
        case K_P2INT: LOC_LOOP(int, int, <, <=); return 0;
        case K_PFLOATINT: LOC_LOOP(float, int, <, <=); return 0;
        case K_PLONGINT: LOC_LOOP(long, int, <, <=); return 0;
        case K_PSHORTINT: LOC_LOOP(short, int, <, <=); return 0;
        case K_PDOUBLEINT: LOC_LOOP(double, int, <, <=); return 0;
        case K_PLDINT: LOC_LOOP(long double, int, <, <=); return 0;
        }
        break;
    case 11:   /* MINLOC: opminloc.c:48-59 */
        switch (kind) {
        case K_P2INT: LOC_LOOP(int, int, >, >=); return 0;
        case K_PFLOATINT: LOC_LOOP(float, int, >, >=); return 0;
        case K_PLONGINT: LOC_LOOP(long, int, >, >=); return 0;
        case K_PSHORTINT: LOC_LOOP(short, int, >, >=); return 0;
        case K_PDOUBLEINT: LOC_LOOP(double, int, >, >=); return 0;
        case K_PLDINT: LOC_LOOP(long double, int, >, >=); return 0;
        }
        break;
    }
    return E_OP;
}

/* element size in bytes of an oracle kind */
static int kind_size(int k)
{
    static const int sz[] = { 0, 1, 1, 2, 2, 4, 4, 8, 8, 2, 4, 8, 8, 16, 1, 8, 8, 16, 8, 16, 16, 32, 32 };
    return sz[k];
}

/* ---- exported -------------------------------------------------------- */

/* check_dtype of builtin op `op` for `datatype`: 0 or E_OP */
int oracle_check_dtype(int op, int datatype)
{
    int grp, idx = op & 0xf;
    if (idx == 0 || idx > 14)
        return E_OP;
    if (check_grp[idx] == -1)
        return E_SUCCESS;       /* REPLACE / NO_OP accept anything */
    type_info(datatype, &grp);
    return (grp & check_grp[idx]) ? E_SUCCESS : E_OP;
}

/* MPIR_Reduce_local for builtin ops (no validation) */
int oracle_reduce_local_nocheck(const void *inbuf, void *inoutbuf, int count, int datatype, int op)
{
    int grp, kind, idx = op & 0xf;
    if (count == 0)
        return E_SUCCESS;
    if (idx == 14)      /* NO_OP */
        return E_SUCCESS;
    kind = type_info(datatype, &grp);
    if (idx == 13) {    /* REPLACE: MPIR_Localcopy */
        if (kind == K_NONE)
            return 3;
        if (count > 0)
            memmove(inoutbuf, inbuf, (size_t) count * kind_size(kind));
        return E_SUCCESS;
    }
    if (!(grp & compute_grp[idx]))
        return E_OP;
    if (count < 0)
        return E_SUCCESS;
    return apply(idx, kind, inbuf, inoutbuf, count);
}

/* MPI_Reduce_local with the reference's validation (builtin ops only) */
int oracle_reduce_local(const void *inbuf, void *inoutbuf, int count, int datatype, int op)
{
    int rc;
    if (op == O_MPI_OP_NULL)
        return E_OP;
    if (op == O_NO_OP || op == O_REPLACE)
        return E_OP;
    if ((((unsigned) op & 0x3c000000u) >> 26) != 0x6 || (((unsigned) op & 0xc0000000u) >> 30) != 0x1)
        return E_OP;    /* not a builtin op handle (user ops are not modelled) */
    rc = oracle_check_dtype(op, datatype);
    if (rc)
        return rc;
    if (count != 0 && inbuf == inoutbuf)
        return E_BUFFER;
    if (count > 0 && inbuf == (void *) -1)
        return E_BUFFER;
    if (count > 0 && inoutbuf == (void *) -1)
        return E_BUFFER;
    return oracle_reduce_local_nocheck(inbuf, inoutbuf, count, datatype, op);
}

/* half <-> float helpers exported for tests */
float oracle_h2f(uint16_t h) { return h2f(h); }
uint16_t oracle_f2h(float f) { return f2h(f); }

/*
 * op_kernels.c -- MPIR_MAXF ... MPIR_NO_OP and their _check_dtype companions,
 * the entries of MPIR_Op_table[] / MPIR_Op_check_dtype_table[].
 *
 * Reference: src/mpi/coll/op/op{max,min,sum,prod,land,band,lor,bor,lxor,bxor,
 * maxloc,minloc,replace,no_op}.c.  Each reference kernel is
 *     switch (*type) { <one scalar loop per accepted type>; default: op_errno = MPI_ERR_OP }
 * Each kernel here performs the same switch (as a lookup in the type matrix,
 * mpir_op_types.h) and replaces the scalar loop with one gfx950 launch through
 * the C-ABI shim (include/mpir_hip_reduce.h).  The `void (void*, void*, int*,
 * MPI_Datatype*)` signature, the op_errno protocol and the "len <= 0 does
 * nothing" behaviour are the reference's.
 */
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <pthread.h>
#include <stdint.h>

#include "mpir_op_types.h"

/* ------------------------------------------------------------ type matrix */

static const MPIR_Type_desc type_table[] = {
    /* C_INTEGER (mpir_op_util.h:263-282) */
    {MPI_INT, MPIR_HIP_I32, G_C_INTEGER, "MPI_INT"},
    {MPI_LONG, MPIR_HIP_I64, G_C_INTEGER, "MPI_LONG"},
    {MPI_SHORT, MPIR_HIP_I16, G_C_INTEGER, "MPI_SHORT"},
    {MPI_UNSIGNED_SHORT, MPIR_HIP_U16, G_C_INTEGER, "MPI_UNSIGNED_SHORT"},
    {MPI_UNSIGNED, MPIR_HIP_U32, G_C_INTEGER, "MPI_UNSIGNED"},
    {MPI_UNSIGNED_LONG, MPIR_HIP_U64, G_C_INTEGER, "MPI_UNSIGNED_LONG"},
    {MPI_LONG_LONG, MPIR_HIP_I64, G_C_INTEGER, "MPI_LONG_LONG"},
    {MPI_UNSIGNED_LONG_LONG, MPIR_HIP_U64, G_C_INTEGER, "MPI_UNSIGNED_LONG_LONG"},
    {MPI_SIGNED_CHAR, MPIR_HIP_I8, G_C_INTEGER, "MPI_SIGNED_CHAR"},
    {MPI_UNSIGNED_CHAR, MPIR_HIP_U8, G_C_INTEGER, "MPI_UNSIGNED_CHAR"},
    {MPI_INT8_T, MPIR_HIP_I8, G_C_INTEGER, "MPI_INT8_T"},
    {MPI_INT16_T, MPIR_HIP_I16, G_C_INTEGER, "MPI_INT16_T"},
    {MPI_INT32_T, MPIR_HIP_I32, G_C_INTEGER, "MPI_INT32_T"},
    {MPI_INT64_T, MPIR_HIP_I64, G_C_INTEGER, "MPI_INT64_T"},
    {MPI_UINT8_T, MPIR_HIP_U8, G_C_INTEGER, "MPI_UINT8_T"},
    {MPI_UINT16_T, MPIR_HIP_U16, G_C_INTEGER, "MPI_UINT16_T"},
    {MPI_UINT32_T, MPIR_HIP_U32, G_C_INTEGER, "MPI_UINT32_T"},
    {MPI_UINT64_T, MPIR_HIP_U64, G_C_INTEGER, "MPI_UINT64_T"},
    /* C_INTEGER_EXTRA: char is signed on x86-64 (mpir_op_util.h:285-286) */
    {MPI_CHAR, MPIR_HIP_I8, G_C_INTEGER_EXTRA, "MPI_CHAR"},
    /* FORTRAN_INTEGER without Fortran: the address/offset/count types (:289-293) */
    {MPI_AINT, MPIR_HIP_I64, G_FORTRAN_INTEGER, "MPI_AINT"},
    {MPI_OFFSET, MPIR_HIP_I64, G_FORTRAN_INTEGER, "MPI_OFFSET"},
    {MPI_COUNT, MPIR_HIP_I64, G_FORTRAN_INTEGER, "MPI_COUNT"},
    /* FLOATING_POINT (:306-311) and _EXTRA (:315-319) */
    {MPI_FLOAT, MPIR_HIP_F32, G_FLOATING_POINT, "MPI_FLOAT"},
    {MPI_DOUBLE, MPIR_HIP_F64, G_FLOATING_POINT, "MPI_DOUBLE"},
    {MPI_LONG_DOUBLE, MPIR_HIP_F80, G_FLOATING_POINT, "MPI_LONG_DOUBLE"},
    {MPIX_C_FLOAT16, MPIR_HIP_F16, G_FLOATING_EXTRA, "MPIX_C_FLOAT16"},
    /* LOGICAL (:324-327) */
    {MPI_C_BOOL, MPIR_HIP_U8, G_LOGICAL, "MPI_C_BOOL"},
    /* COMPLEX (:331-335) */
    {MPI_C_FLOAT_COMPLEX, MPIR_HIP_CF32, G_COMPLEX, "MPI_C_FLOAT_COMPLEX"},
    {MPI_C_DOUBLE_COMPLEX, MPIR_HIP_CF64, G_COMPLEX, "MPI_C_DOUBLE_COMPLEX"},
    {MPI_C_LONG_DOUBLE_COMPLEX, MPIR_HIP_CF80, G_COMPLEX, "MPI_C_LONG_DOUBLE_COMPLEX"},
    /* BYTE (:344-345) */
    {MPI_BYTE, MPIR_HIP_U8, G_BYTE, "MPI_BYTE"},
    /* MAXLOC/MINLOC pairs (opmaxloc.c:83-97) */
    {MPI_2INT, MPIR_HIP_P2INT, G_LOC_PAIR, "MPI_2INT"},
    {MPI_FLOAT_INT, MPIR_HIP_PFLOATINT, G_LOC_PAIR, "MPI_FLOAT_INT"},
    {MPI_LONG_INT, MPIR_HIP_PLONGINT, G_LOC_PAIR, "MPI_LONG_INT"},
    {MPI_SHORT_INT, MPIR_HIP_PSHORTINT, G_LOC_PAIR, "MPI_SHORT_INT"},
    {MPI_DOUBLE_INT, MPIR_HIP_PDOUBLEINT, G_LOC_PAIR, "MPI_DOUBLE_INT"},
    {MPI_LONG_DOUBLE_INT, MPIR_HIP_PLDOUBLEINT, G_LOC_PAIR, "MPI_LONG_DOUBLE_INT"},
};

/* Predefined handles are 0x4c00SSII (builtin, size SS, index II) or
 * 0x8c00000I (the pair types): one table slot per (kind, II), filled once. */
static const MPIR_Type_desc *by_index[2][256];
static pthread_once_t by_index_once = PTHREAD_ONCE_INIT;

static void by_index_init(void)
{
    for (size_t i = 0; i < sizeof(type_table) / sizeof(type_table[0]); i++) {
        const unsigned h = (unsigned) type_table[i].datatype;
        by_index[(h >> 24) == 0x8cu][h & 0xffu] = &type_table[i];
    }
}

const MPIR_Type_desc *MPIR_Type_lookup(MPI_Datatype datatype)
{
    const unsigned h = (unsigned) datatype;
    const MPIR_Type_desc *d;
    if ((h >> 24) != 0x4cu && (h >> 24) != 0x8cu)
        return NULL;
    pthread_once(&by_index_once, by_index_init);
    d = by_index[(h >> 24) == 0x8cu][h & 0xffu];
    return (d && d->datatype == datatype) ? d : NULL;
}

#define NUMERIC (G_C_INTEGER | G_C_INTEGER_EXTRA | G_FORTRAN_INTEGER | G_FLOATING_POINT | G_FLOATING_EXTRA)
#define INTEGERS (G_C_INTEGER | G_C_INTEGER_EXTRA | G_FORTRAN_INTEGER)

/* index = MPIR_Op_table slot (allreduce.c:121-129) */
static const unsigned compute_groups[MPIR_OP_N_BUILTIN] = {
    0,
    NUMERIC,                                   /* 1 MAX    opmax.c:33-39 */
    NUMERIC,                                   /* 2 MIN    opmin.c:32-38 */
    NUMERIC | G_COMPLEX,                       /* 3 SUM    opsum.c:34-57 */
    NUMERIC | G_COMPLEX,                       /* 4 PROD   opprod.c:34-64 */
    INTEGERS | G_LOGICAL,                      /* 5 LAND   opland.c:36-70 */
    INTEGERS | G_BYTE,                         /* 6 BAND   opband.c:33-40 */
    INTEGERS | G_LOGICAL,                      /* 7 LOR    oplor.c:36-70 */
    INTEGERS | G_BYTE,                         /* 8 BOR    opbor.c */
    INTEGERS | G_LOGICAL | G_FLOATING_POINT | G_FLOATING_EXTRA, /* 9 LXOR oplxor.c:36-71 */
    INTEGERS | G_BYTE,                         /* 10 BXOR  opbxor.c */
    G_LOC_PAIR,                                /* 11 MINLOC opminloc.c:82-108 */
    G_LOC_PAIR,                                /* 12 MAXLOC opmaxloc.c:83-109 */
    ~0u,                                       /* 13 REPLACE (any basic type) */
    ~0u,                                       /* 14 NO_OP */
};

static const unsigned check_groups[MPIR_OP_N_BUILTIN] = {
    0,
    NUMERIC,
    NUMERIC,
    NUMERIC | G_COMPLEX,
    NUMERIC | G_COMPLEX,
    INTEGERS | G_LOGICAL | G_FLOATING_POINT | G_FLOATING_EXTRA,     /* opland.c:95-107 */
    INTEGERS | G_BYTE,
    INTEGERS | G_LOGICAL | G_FLOATING_POINT | G_FLOATING_EXTRA,     /* oplor.c:95-107 */
    INTEGERS | G_BYTE,
    INTEGERS | G_LOGICAL | G_FLOATING_POINT | G_FLOATING_EXTRA,
    INTEGERS | G_BYTE,
    G_LOC_PAIR,
    G_LOC_PAIR,
    ~0u,
    ~0u,
};

unsigned MPIR_Op_compute_groups(int opidx)
{
    return (opidx > 0 && opidx < MPIR_OP_N_BUILTIN) ? compute_groups[opidx] : 0;
}

unsigned MPIR_Op_check_groups(int opidx)
{
    return (opidx > 0 && opidx < MPIR_OP_N_BUILTIN) ? check_groups[opidx] : 0;
}

int MPIR_Op_resolve_elem(int opidx, MPI_Datatype datatype)
{
    const MPIR_Type_desc *d = MPIR_Type_lookup(datatype);
    if (!d || !(d->groups & MPIR_Op_compute_groups(opidx)))
        return 0;
    return d->elem;
}

/* ------------------------------------------------------------ errors */

static __thread char err_detail[256];

#ifndef MPIR_DROPIN_IN_LIBMPI
/* standalone: the library's own slot (in libmpi: MPIR_Per_thread.op_errno,
 * mpich_glue.c) */
static __thread int op_errno_slot;

int *MPIR_Op_errno_ptr(void)
{
    return &op_errno_slot;
}
#endif

void MPIR_Err_set_detail(const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(err_detail, sizeof(err_detail), fmt, ap);
    va_end(ap);
}

const char *MPIR_Err_last_detail(void)
{
    return err_detail;
}

void MPIR_Op_report_hip_error(const char *opname, int hip_rc)
{
    switch (hip_rc) {
    case MPIR_HIP_ENODEV:
        MPIR_Err_set_detail("%s: no HIP device available for the reduction", opname);
        break;
    case MPIR_HIP_ENOKERNEL:
        MPIR_Err_set_detail("%s: no gfx950 kernel for this datatype", opname);
        break;
    default:
        MPIR_Err_set_detail("%s: HIP runtime error: %s", opname, MPIR_Hip_error_string());
    }
    *MPIR_Op_errno_ptr() = (hip_rc == MPIR_HIP_ENOKERNEL) ? MPI_ERR_OP : MPI_ERR_OTHER;
}

/* ------------------------------------------------------------ kernels */

#ifdef MPIR_DROPIN_IN_LIBMPI
/* In libmpi: the node's rank count from MPICH's node communicator
 * (mpich_glue.c), handed to the library once it is known, before the host
 * combine sizes its threads (standalone, the library reads the launcher's
 * environment itself). */
int MPIR_Dropin_local_ranks(void);

static inline void pass_local_ranks(void)
{
    static int passed;
    if (__atomic_load_n(&passed, __ATOMIC_RELAXED))
        return;
    int n = MPIR_Dropin_local_ranks();
    if (n > 0) {
        MPIR_Hip_set_local_ranks(n);
        __atomic_store_n(&passed, 1, __ATOMIC_RELAXED);
    }
}
#else
static inline void pass_local_ranks(void)
{
}
#endif

/* The body shared by every reference kernel: the datatype switch, then
 * either the combine (one GPU launch) or the `default:` branch that stores
 * MPI_ERR_OP ("**opundefined") in op_errno (e.g. opsum.c:59-73). */
static void op_apply(int opidx, const char *opname, void *invec, void *inoutvec, int *Len,
                     MPI_Datatype * type)
{
    int len = *Len;
    int elem = MPIR_Op_resolve_elem(opidx, *type);
    int rc;
    if (!elem) {
        MPIR_Err_set_detail("MPI_Op %s operation not defined for this datatype", opname);
        *MPIR_Op_errno_ptr() = MPI_ERR_OP;
        return;
    }
    if (len <= 0)       /* `for (i=0; i<len; i++)` runs zero times */
        return;
    pass_local_ranks();
    rc = MPIR_Hip_reduce(invec, inoutvec, (uint64_t) len, opidx, elem, NULL, 1);
    if (rc != MPIR_HIP_OK)
        MPIR_Op_report_hip_error(opname, rc);
}

static int op_check(int opidx, const char *opname, MPI_Datatype type)
{
    const MPIR_Type_desc *d = MPIR_Type_lookup(type);
    if (d && (d->groups & MPIR_Op_check_groups(opidx)))
        return MPI_SUCCESS;
    MPIR_Err_set_detail("MPI_Op %s operation not defined for this datatype", opname);
    return MPI_ERR_OP;
}

#define DEFINE_OP(FN, IDX, NAME)                                                  \
    void FN(void *invec, void *inoutvec, int *Len, MPI_Datatype * type)           \
    {                                                                             \
        op_apply(IDX, NAME, invec, inoutvec, Len, type);                          \
    }                                                                             \
    int FN##_check_dtype(MPI_Datatype type)                                       \
    {                                                                             \
        return op_check(IDX, NAME, type);                                         \
    }

DEFINE_OP(MPIR_MAXF, MPIR_HIP_OP_MAX, "MPI_MAX")
DEFINE_OP(MPIR_MINF, MPIR_HIP_OP_MIN, "MPI_MIN")
DEFINE_OP(MPIR_SUM, MPIR_HIP_OP_SUM, "MPI_SUM")
DEFINE_OP(MPIR_PROD, MPIR_HIP_OP_PROD, "MPI_PROD")
DEFINE_OP(MPIR_LAND, MPIR_HIP_OP_LAND, "MPI_LAND")
DEFINE_OP(MPIR_BAND, MPIR_HIP_OP_BAND, "MPI_BAND")
DEFINE_OP(MPIR_LOR, MPIR_HIP_OP_LOR, "MPI_LOR")
DEFINE_OP(MPIR_BOR, MPIR_HIP_OP_BOR, "MPI_BOR")
DEFINE_OP(MPIR_LXOR, MPIR_HIP_OP_LXOR, "MPI_LXOR")
DEFINE_OP(MPIR_BXOR, MPIR_HIP_OP_BXOR, "MPI_BXOR")
DEFINE_OP(MPIR_MINLOC, MPIR_HIP_OP_MINLOC, "MPI_MINLOC")
DEFINE_OP(MPIR_MAXLOC, MPIR_HIP_OP_MAXLOC, "MPI_MAXLOC")

/* MPIR_REPLACE (opreplace.c:15-18): MPIR_Localcopy(invec, len, type, inoutvec,
 * len, type), reached through the table by RMA accumulate (mpidrma.h:902).
 * Every predefined datatype is a contiguous copy of len * size bytes: the
 * basic ones of this library's type table, and any other builtin-kind handle
 * (MPI_WCHAR, MPI_PACKED, Fortran types, MPI_LB / MPI_UB of size 0) by the
 * size its handle encodes in bits 8-15 (MPIR_Datatype_get_basic_size,
 * mpir_datatype.h:172).  Derived datatypes need MPICH's datatype engine,
 * which is outside this library: MPI_ERR_TYPE. */
void MPIR_REPLACE(void *invec, void *inoutvec, int *Len, MPI_Datatype * type)
{
    const MPIR_Type_desc *d = MPIR_Type_lookup(*type);
    const unsigned h = (unsigned) *type;
    uint64_t count;
    int elem, rc;
    if (d) {
        elem = d->elem;
        count = *Len > 0 ? (uint64_t) * Len : 0;
    } else if ((h >> 30) == 1u && ((h >> 26) & 0xfu) == 0x3u) {         /* builtin-kind datatype */
        elem = MPIR_HIP_U8;
        count = *Len > 0 ? (uint64_t) * Len * ((h >> 8) & 0xffu) : 0;
    } else {
        MPIR_Err_set_detail("MPI_REPLACE: derived datatypes are not supported by this library");
        *MPIR_Op_errno_ptr() = MPI_ERR_TYPE;
        return;
    }
    if (count == 0)
        return;
    rc = MPIR_Hip_reduce(invec, inoutvec, count, MPIR_HIP_OP_REPLACE, elem, NULL, 1);
    if (rc != MPIR_HIP_OK)
        MPIR_Op_report_hip_error("MPI_REPLACE", rc);
}

int MPIR_REPLACE_check_dtype(MPI_Datatype type)
{
    (void) type;
    return MPI_SUCCESS;         /* opreplace.c:40-44 */
}

/* MPIR_NO_OP (opno_op.c:15): nothing */
void MPIR_NO_OP(void *invec, void *inoutvec, int *Len, MPI_Datatype * type)
{
    (void) invec;
    (void) inoutvec;
    (void) Len;
    (void) type;
}

int MPIR_NO_OP_check_dtype(MPI_Datatype type)
{
    (void) type;
    return MPI_SUCCESS;
}

/* ------------------------------------------------------------ tables */
/* allreduce.c:121-139: order must match the op handles' low 4 bits */
MPI_User_function *MPIR_Op_table[MPIR_OP_N_BUILTIN] = {
    NULL, MPIR_MAXF,
    MPIR_MINF, MPIR_SUM,
    MPIR_PROD, MPIR_LAND,
    MPIR_BAND, MPIR_LOR, MPIR_BOR,
    MPIR_LXOR, MPIR_BXOR,
    MPIR_MINLOC, MPIR_MAXLOC,
    MPIR_REPLACE, MPIR_NO_OP
};

MPIR_Op_check_dtype_fn *MPIR_Op_check_dtype_table[MPIR_OP_N_BUILTIN] = {
    NULL, MPIR_MAXF_check_dtype,
    MPIR_MINF_check_dtype, MPIR_SUM_check_dtype,
    MPIR_PROD_check_dtype, MPIR_LAND_check_dtype,
    MPIR_BAND_check_dtype, MPIR_LOR_check_dtype, MPIR_BOR_check_dtype,
    MPIR_LXOR_check_dtype, MPIR_BXOR_check_dtype,
    MPIR_MINLOC_check_dtype, MPIR_MAXLOC_check_dtype,
    MPIR_REPLACE_check_dtype, MPIR_NO_OP_check_dtype
};

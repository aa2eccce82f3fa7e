/*
 * mpi_reduce_local.h -- drop-in C ABI for MPICH's local reduction hot path,
 * implemented on MI355X (gfx950) HIP kernels.
 *
 * Every declaration here replaces the symbol of the same name in the
 * reference (pmodels/mpich-pip, MPICH 3.3).  Handle values, error classes and
 * calling conventions are identical to an x86-64 MPICH 3.3 build configured
 * with --disable-fortran --disable-cxx (long double included: the x87 80-bit
 * format is computed in software on the GPU), so the existing collective
 * schedules and the RMA accumulate path can call these functions unchanged.
 *
 * Reference interfaces replaced (file:line under the reference tree):
 *   MPI_Reduce_local / PMPI_Reduce_local  src/include/mpi.h.in:1359,
 *                                          src/mpi/coll/reduce_local/reduce_local.c:11-20,155-219
 *   MPIR_Reduce_local                      src/include/mpir_coll.h:1542,
 *                                          src/mpi/coll/reduce_local/reduce_local.c:35-122
 *   MPIR_Op_table / MPIR_Op_check_dtype_table
 *                                          src/mpi/coll/allreduce/allreduce.c:121-139,
 *                                          src/include/mpir_op.h:183-189
 *   MPIR_MAXF ... MPIR_NO_OP (+ _check_dtype)
 *                                          src/include/mpir_op.h:131-159, src/mpi/coll/op/op*.c
 *   MPI_Op_create / MPI_Op_free / MPI_Op_commutative
 *                                          src/mpi/coll/op/op_create.c:73-140,
 *                                          src/mpi/coll/op/op_free.c, op_commutative.c
 *   MPIR_Op_is_commutative                 src/mpi/coll/op/op_commutative.c:39
 *   MPI_Error_class / MPI_Error_string     src/mpi/errhan/error_class.c, error_string.c
 *
 * Extensions (MPIX_ prefix, not in the reference):
 *   MPIX_Reduce_local_stream  -- stream-ordered, non-synchronising variant for
 *                                device-resident buffers (what this library's
 *                                own schedules and benchmarks use).
 *   MPIX_Reduce_local_set_errhandler / _get_errhandler -- the reference routes
 *                                MPI_Reduce_local errors through
 *                                MPIR_Err_return_comm(NULL, ...) (errutil.c:238),
 *                                i.e. COMM_WORLD's handler; this library has no
 *                                communicators, so the handler is set here.
 */
#ifndef MPI_REDUCE_LOCAL_H_INCLUDED
#define MPI_REDUCE_LOCAL_H_INCLUDED

#ifdef __cplusplus
extern "C" {
#endif

/* The public API stays exported when these sources are compiled into a
 * libmpi built with -fvisibility=hidden (MPICH's configure.ac:1443 adds it;
 * mpi.h.in:13 marks the public prototypes the same way); the MPIR_ internals
 * follow the build's visibility, as MPICH's do. */
#ifndef MPICH_API_PUBLIC
#if defined(__GNUC__) || defined(__clang__)
#define MPICH_API_PUBLIC __attribute__((visibility("default")))
#else
#define MPICH_API_PUBLIC
#endif
#endif

/* ---- handle types (mpi.h.in:104,310) ---------------------------------- */
typedef int MPI_Datatype;
typedef int MPI_Op;
typedef int MPI_Errhandler;
typedef long MPI_Aint;          /* x86-64: MPI_AINT is 8 bytes */
typedef long long MPI_Offset;
typedef long long MPI_Count;

typedef void (MPI_User_function) (void *invec, void *inoutvec, int *len, MPI_Datatype * datatype);

#define MPI_IN_PLACE ((void *) -1)      /* mpi.h.in:544 */

/* ---- error classes (mpi.h.in:784-811) --------------------------------- */
#define MPI_SUCCESS          0
#define MPI_ERR_BUFFER       1
#define MPI_ERR_COUNT        2
#define MPI_ERR_TYPE         3
#define MPI_ERR_OP           9
#define MPI_ERR_ARG         12
#define MPI_ERR_UNKNOWN     13
#define MPI_ERR_OTHER       15
#define MPI_ERR_INTERN      16
#define MPI_ERR_NO_MEM      34

/* ---- error handlers (mpi.h.in: MPI_ERRORS_ARE_FATAL / MPI_ERRORS_RETURN) */
#define MPI_ERRHANDLER_NULL  ((MPI_Errhandler)0x14000000)
#define MPI_ERRORS_ARE_FATAL ((MPI_Errhandler)0x54000000)
#define MPI_ERRORS_RETURN    ((MPI_Errhandler)0x54000001)

/* ---- predefined ops (mpi.h.in:310-325): 0x58000000 | table index ------- */
#define MPI_OP_NULL ((MPI_Op)0x18000000)
#define MPI_MAX     ((MPI_Op)0x58000001)
#define MPI_MIN     ((MPI_Op)0x58000002)
#define MPI_SUM     ((MPI_Op)0x58000003)
#define MPI_PROD    ((MPI_Op)0x58000004)
#define MPI_LAND    ((MPI_Op)0x58000005)
#define MPI_BAND    ((MPI_Op)0x58000006)
#define MPI_LOR     ((MPI_Op)0x58000007)
#define MPI_BOR     ((MPI_Op)0x58000008)
#define MPI_LXOR    ((MPI_Op)0x58000009)
#define MPI_BXOR    ((MPI_Op)0x5800000a)
#define MPI_MINLOC  ((MPI_Op)0x5800000b)
#define MPI_MAXLOC  ((MPI_Op)0x5800000c)
#define MPI_REPLACE ((MPI_Op)0x5800000d)
#define MPI_NO_OP   ((MPI_Op)0x5800000e)

/* ---- predefined datatypes, x86-64 values (configure.ac:3442-3705,5077-5408)
 * bits 8-15 hold the size in bytes (mpir_datatype.h:172). */
#define MPI_DATATYPE_NULL       ((MPI_Datatype)0x0c000000)
#define MPI_CHAR                ((MPI_Datatype)0x4c000101)
#define MPI_UNSIGNED_CHAR       ((MPI_Datatype)0x4c000102)
#define MPI_SHORT               ((MPI_Datatype)0x4c000203)
#define MPI_UNSIGNED_SHORT      ((MPI_Datatype)0x4c000204)
#define MPI_INT                 ((MPI_Datatype)0x4c000405)
#define MPI_UNSIGNED            ((MPI_Datatype)0x4c000406)
#define MPI_LONG                ((MPI_Datatype)0x4c000807)
#define MPI_UNSIGNED_LONG       ((MPI_Datatype)0x4c000808)
#define MPI_LONG_LONG_INT       ((MPI_Datatype)0x4c000809)
#define MPI_LONG_LONG           MPI_LONG_LONG_INT
#define MPI_FLOAT               ((MPI_Datatype)0x4c00040a)
#define MPI_DOUBLE              ((MPI_Datatype)0x4c00080b)
#define MPI_LONG_DOUBLE         ((MPI_Datatype)0x4c00100c)   /* x87 80-bit in a 16-byte slot */
#define MPI_BYTE                ((MPI_Datatype)0x4c00010d)
#define MPI_WCHAR               ((MPI_Datatype)0x4c00040e)
#define MPI_PACKED              ((MPI_Datatype)0x4c00010f)
#define MPI_LB                  ((MPI_Datatype)0x4c000010)
#define MPI_UB                  ((MPI_Datatype)0x4c000011)
#define MPI_2INT                ((MPI_Datatype)0x4c000816)
#define MPI_SIGNED_CHAR         ((MPI_Datatype)0x4c000118)
#define MPI_UNSIGNED_LONG_LONG  ((MPI_Datatype)0x4c000819)
#define MPI_FLOAT_INT           ((MPI_Datatype)0x8c000000)
#define MPI_DOUBLE_INT          ((MPI_Datatype)0x8c000001)
#define MPI_LONG_INT            ((MPI_Datatype)0x8c000002)
#define MPI_SHORT_INT           ((MPI_Datatype)0x8c000003)
#define MPI_LONG_DOUBLE_INT     ((MPI_Datatype)0x8c000004)   /* {long double; int}, 32 B */
#define MPI_INT8_T              ((MPI_Datatype)0x4c000137)
#define MPI_INT16_T             ((MPI_Datatype)0x4c000238)
#define MPI_INT32_T             ((MPI_Datatype)0x4c000439)
#define MPI_INT64_T             ((MPI_Datatype)0x4c00083a)
#define MPI_UINT8_T             ((MPI_Datatype)0x4c00013b)
#define MPI_UINT16_T            ((MPI_Datatype)0x4c00023c)
#define MPI_UINT32_T            ((MPI_Datatype)0x4c00043d)
#define MPI_UINT64_T            ((MPI_Datatype)0x4c00083e)
#define MPI_C_BOOL              ((MPI_Datatype)0x4c00013f)
#define MPI_C_FLOAT_COMPLEX     ((MPI_Datatype)0x4c000840)
#define MPI_C_COMPLEX           MPI_C_FLOAT_COMPLEX
#define MPI_C_DOUBLE_COMPLEX    ((MPI_Datatype)0x4c001041)
#define MPI_C_LONG_DOUBLE_COMPLEX ((MPI_Datatype)0x4c002042) /* long double _Complex, 32 B */
#define MPIX_C_FLOAT16          ((MPI_Datatype)0x4c000246)
#define MPI_AINT                ((MPI_Datatype)0x4c000843)
#define MPI_OFFSET              ((MPI_Datatype)0x4c000844)
#define MPI_COUNT               ((MPI_Datatype)0x4c000845)

/* ---- the hot path ------------------------------------------------------ */

/* MPI_Reduce_local (reduce_local.c:155): inoutbuf[i] = op(inbuf[i], inoutbuf[i]),
 * i in [0,count).  Buffers may be HIP device memory, pinned host memory or
 * pageable host memory, in any combination; the combine always runs on the
 * GPU.  Synchronous: the result is complete in inoutbuf on return. */
MPICH_API_PUBLIC int MPI_Reduce_local(const void *inbuf, void *inoutbuf, int count, MPI_Datatype datatype, MPI_Op op);
MPICH_API_PUBLIC int PMPI_Reduce_local(const void *inbuf, void *inoutbuf, int count, MPI_Datatype datatype, MPI_Op op);

/* MPIR_Reduce_local (reduce_local.c:35): no argument validation; builtin ops
 * dispatch through MPIR_Op_table[op & 0xf], user ops through their function. */
int MPIR_Reduce_local(const void *inbuf, void *inoutbuf, int count, MPI_Datatype datatype, MPI_Op op);

/* ---- op kernels and tables (mpir_op.h:131-189, allreduce.c:121-139) --- */
void MPIR_MAXF(void *invec, void *inoutvec, int *len, MPI_Datatype * type);
void MPIR_MINF(void *invec, void *inoutvec, int *len, MPI_Datatype * type);
void MPIR_SUM(void *invec, void *inoutvec, int *len, MPI_Datatype * type);
void MPIR_PROD(void *invec, void *inoutvec, int *len, MPI_Datatype * type);
void MPIR_LAND(void *invec, void *inoutvec, int *len, MPI_Datatype * type);
void MPIR_BAND(void *invec, void *inoutvec, int *len, MPI_Datatype * type);
void MPIR_LOR(void *invec, void *inoutvec, int *len, MPI_Datatype * type);
void MPIR_BOR(void *invec, void *inoutvec, int *len, MPI_Datatype * type);
void MPIR_LXOR(void *invec, void *inoutvec, int *len, MPI_Datatype * type);
void MPIR_BXOR(void *invec, void *inoutvec, int *len, MPI_Datatype * type);
void MPIR_MAXLOC(void *invec, void *inoutvec, int *len, MPI_Datatype * type);
void MPIR_MINLOC(void *invec, void *inoutvec, int *len, MPI_Datatype * type);
void MPIR_REPLACE(void *invec, void *inoutvec, int *len, MPI_Datatype * type);
void MPIR_NO_OP(void *invec, void *inoutvec, int *len, MPI_Datatype * type);

int MPIR_MAXF_check_dtype(MPI_Datatype type);
int MPIR_MINF_check_dtype(MPI_Datatype type);
int MPIR_SUM_check_dtype(MPI_Datatype type);
int MPIR_PROD_check_dtype(MPI_Datatype type);
int MPIR_LAND_check_dtype(MPI_Datatype type);
int MPIR_BAND_check_dtype(MPI_Datatype type);
int MPIR_LOR_check_dtype(MPI_Datatype type);
int MPIR_BOR_check_dtype(MPI_Datatype type);
int MPIR_LXOR_check_dtype(MPI_Datatype type);
int MPIR_BXOR_check_dtype(MPI_Datatype type);
int MPIR_MAXLOC_check_dtype(MPI_Datatype type);
int MPIR_MINLOC_check_dtype(MPI_Datatype type);
int MPIR_REPLACE_check_dtype(MPI_Datatype type);
int MPIR_NO_OP_check_dtype(MPI_Datatype type);

#define MPIR_OP_N_BUILTIN 15
typedef int (MPIR_Op_check_dtype_fn) (MPI_Datatype);
extern MPI_User_function *MPIR_Op_table[MPIR_OP_N_BUILTIN];
extern MPIR_Op_check_dtype_fn *MPIR_Op_check_dtype_table[MPIR_OP_N_BUILTIN];
#define MPIR_OP_HDL_TO_FN(op) MPIR_Op_table[((op)&0xf)]
#define MPIR_OP_HDL_TO_DTYPE_FN(op) MPIR_Op_check_dtype_table[((op)&0xf)]

/* ---- user ops (op_create.c, op_free.c, op_commutative.c) ------------- */
MPICH_API_PUBLIC int MPI_Op_create(MPI_User_function * user_fn, int commute, MPI_Op * op);
MPICH_API_PUBLIC int PMPI_Op_create(MPI_User_function * user_fn, int commute, MPI_Op * op);
MPICH_API_PUBLIC int MPI_Op_free(MPI_Op * op);
MPICH_API_PUBLIC int PMPI_Op_free(MPI_Op * op);
MPICH_API_PUBLIC int MPI_Op_commutative(MPI_Op op, int *commute);
MPICH_API_PUBLIC int PMPI_Op_commutative(MPI_Op op, int *commute);
int MPIR_Op_is_commutative(MPI_Op op);

/* ---- errors ------------------------------------------------------------ */
#define MPI_MAX_ERROR_STRING 512
MPICH_API_PUBLIC int MPI_Error_class(int errorcode, int *errorclass);
MPICH_API_PUBLIC int MPI_Error_string(int errorcode, char *string, int *resultlen);

/* ---- extensions -------------------------------------------------------- */
/* Stream-ordered variant: enqueue the combine on `hip_stream` (a hipStream_t,
 * NULL = the calling thread's library stream) and return without waiting.
 * Both buffers must be device-accessible (hipMalloc / managed / mapped);
 * host-only pointers give MPI_ERR_BUFFER.  Same validation and error classes
 * as MPI_Reduce_local; user ops give MPI_ERR_OP (they run on the host). */
MPICH_API_PUBLIC int MPIX_Reduce_local_stream(const void *inbuf, void *inoutbuf, int count, MPI_Datatype datatype,
                             MPI_Op op, void *hip_stream);
/* Multi-operand local reduction: outbuf = fold of n device buffers, in the
 * association a reduction schedule would produce by calling MPIR_Reduce_local
 * step by step (bit-identical to doing exactly that):
 *   MPIX_ORDER_TREE  (n a power of two <= 64): ((b0+b1)+(b2+b3))+((b4+b5)+(b6+b7)) --
 *       recursive halving, reduce_intra_reduce_scatter_gather.c:186-249;
 *   MPIX_ORDER_CHAIN (1 <= n <= 64): ((b0+b1)+b2)+... -- pairwise,
 *       reduce_scatter_block_intra_pairwise.c:97-134.
 * Passes over HBM: one for TREE (any n) and for CHAIN with n <= 8; CHAIN with
 * n > 8 folds 7 more operands per pass into outbuf, ceil((n-1)/7) passes.
 * In each step the left operand is the step's inoutbuf.  outbuf may be
 * inbufs[0] exactly; any other overlap of outbuf with an operand is
 * MPI_ERR_BUFFER.  hip_stream NULL: synchronous on the library stream;
 * otherwise enqueued on that stream without waiting.  Builtin ops and basic
 * types with the same validation as MPI_Reduce_local. */
#define MPIX_ORDER_TREE  0
#define MPIX_ORDER_CHAIN 1
MPICH_API_PUBLIC int MPIX_Reduce_local_multi(const void *const *inbufs, int n, void *outbuf, int count,
                            MPI_Datatype datatype, MPI_Op op, int order, void *hip_stream);
MPICH_API_PUBLIC int MPIX_Reduce_local_set_errhandler(MPI_Errhandler errhandler);
MPICH_API_PUBLIC int MPIX_Reduce_local_get_errhandler(MPI_Errhandler * errhandler);

#ifdef __cplusplus
}
#endif
#endif /* MPI_REDUCE_LOCAL_H_INCLUDED */

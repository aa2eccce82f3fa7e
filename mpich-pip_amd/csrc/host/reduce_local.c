/*
 * reduce_local.c -- MPI_Reduce_local / PMPI_Reduce_local / MPIR_Reduce_local,
 * the stream-ordered MPIX variant, user-defined ops and error reporting.
 *
 * Reference: src/mpi/coll/reduce_local/reduce_local.c (MPIR_Reduce_local
 * :35-122, MPI_Reduce_local :155-219), src/include/mpir_err.h (ERRTEST_OP
 * :499-510, ERRTEST_ALIAS_COLL :277-285, ERRTEST_NAMED_BUF_INPLACE :440-446),
 * src/mpi/coll/op/op_create.c, op_free.c, op_commutative.c.
 *
 * Validation order, error classes, the count==0 early exit, the op_errno
 * reset/read protocol and the builtin/user dispatch are the reference's.
 * Differences, all documented in DESIGN.md:
 *   - the library is always "initialized" (no MPI_Init in this drop-in);
 *   - error codes are MPICH-format codes with an error stack (errutil.c; libmpi's
 *     own MPIR_Err_* routines when compiled into it);
 *   - the error handler that MPI_Reduce_local reaches through
 *     MPIR_Err_return_comm(NULL, ...) is set by MPIX_Reduce_local_set_errhandler
 *     (default MPI_ERRORS_ARE_FATAL, as for COMM_WORLD in the reference);
 *   - a builtin-kind op handle with table index 0 or 15 returns MPI_ERR_OP
 *     instead of calling through the table's NULL slot.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mpir_op_objects.h"
#include "mpir_op_types.h"

/* ---- handles and user ops: the MPIR_Op object store (op_objects.c) ----- */
#define HANDLE_KIND_INVALID  MPIR_HANDLE_KIND_INVALID
#define HANDLE_KIND_BUILTIN  MPIR_HANDLE_KIND_BUILTIN
#define HANDLE_GET_KIND(a)     MPIR_HANDLE_GET_KIND(a)
#define HANDLE_GET_MPI_KIND(a) MPIR_HANDLE_GET_MPI_KIND(a)

/* A live user-defined op: MPIR_Op_get_ptr + MPIR_Op_valid_ptr
 * (reduce_local.c:172-177), plus a check the reference does not make --
 * that the object is allocated (its handle is this handle, its reference
 * count positive) -- so a freed or never-created handle returns
 * MPI_ERR_OP instead of calling through a stale function pointer. */
static MPIR_Op *user_op_get(MPI_Op op)
{
    MPIR_Op *p;
    if (HANDLE_GET_MPI_KIND(op) != MPIR_OP_OBJ_KIND || HANDLE_GET_KIND(op) == HANDLE_KIND_BUILTIN)
        return NULL;
    p = MPIR_Op_get_ptr_fn(op);
    if (!p || p->handle != op || __atomic_load_n(&p->ref_count, __ATOMIC_ACQUIRE) <= 0 ||
        p->kind < MPIR_OP_KIND__USER_NONCOMMUTE)
        return NULL;
    return p;
}

/* ---- error handling ----------------------------------------------------- */
/* COMM_WORLD's handler as MPIR_Err_return_comm(NULL, ...) sees it: fatal,
 * unless MPIR_CVAR_REDUCE_LOCAL_ERRHANDLER=return (for the LD_PRELOAD shim,
 * whose MPIX_ setter the application cannot reach) or the setter says so */
static MPI_Errhandler reduce_local_errhandler = 0;

static MPI_Errhandler default_errhandler(void)
{
    const char *e = getenv("MPIR_CVAR_REDUCE_LOCAL_ERRHANDLER");
    return (e && !strcmp(e, "return")) ? MPI_ERRORS_RETURN : MPI_ERRORS_ARE_FATAL;
}

int MPIX_Reduce_local_set_errhandler(MPI_Errhandler errhandler)
{
    if (errhandler != MPI_ERRORS_ARE_FATAL && errhandler != MPI_ERRORS_RETURN)
        return MPI_ERR_ARG;
    __atomic_store_n(&reduce_local_errhandler, errhandler, __ATOMIC_RELAXED);
    return MPI_SUCCESS;
}

int MPIX_Reduce_local_get_errhandler(MPI_Errhandler * errhandler)
{
    MPI_Errhandler h = __atomic_load_n(&reduce_local_errhandler, __ATOMIC_RELAXED);
    *errhandler = h ? h : default_errhandler();
    return MPI_SUCCESS;
}

/* The innermost level of an error stack: a bare class raised inside this
 * library (its text in the thread's detail slot) becomes an MPICH error code
 * (MPIR_Err_create_code, errutil.c here or libmpi's own).  A code that already
 * carries a stack passes through. */
int MPIR_Err_wrap_detail(const char *fcname, int line, int mpi_errno)
{
    const char *detail;
    if (mpi_errno == MPI_SUCCESS || (mpi_errno & ~0x7f) != 0)
        return mpi_errno;
    detail = MPIR_Err_last_detail();
    if (!detail[0])
        return MPIR_Err_create_code(MPI_SUCCESS, MPIR_ERR_RECOVERABLE, fcname, line, mpi_errno, "**other", NULL);
    return MPIR_Err_create_code(MPI_SUCCESS, MPIR_ERR_RECOVERABLE, fcname, line, mpi_errno, "**other", "%s", detail);
}

/* The MPI-level error exit of every entry point but MPI_Reduce_local's own:
 * wrap, then MPIR_Err_return_comm(NULL, ...) (errutil.c:238) -- COMM_WORLD's
 * handler, fatal by default. */
int MPIR_Err_return_at(const char *fcname, int line, int mpi_errno)
{
    return MPIR_Err_return_comm(NULL, fcname, MPIR_Err_wrap_detail(fcname, line, mpi_errno));
}

#define err_return MPIR_Err_return

static int alias_check_enabled(void)
{
    /* MPIR_CVAR_COLL_ALIAS_CHECK (mpir_err.h:157-171), default 1.  Racing
     * first calls store the same value; the atomics make that well defined. */
    static int cached = -1;
    int c = __atomic_load_n(&cached, __ATOMIC_RELAXED);
    if (c < 0) {
        const char *v = getenv("MPIR_CVAR_COLL_ALIAS_CHECK");
        c = v ? (atoi(v) != 0) : 1;
        __atomic_store_n(&cached, c, __ATOMIC_RELAXED);
    }
    return c;
}

/* The validation block of MPI_Reduce_local (reduce_local.c:166-191). */
static int validate(const void *inbuf, void *inoutbuf, int count, MPI_Datatype datatype, MPI_Op op)
{
    int mpi_errno;
    /* MPIR_ERRTEST_OP (mpir_err.h:499-510) */
    if (op == MPI_OP_NULL) {
        MPIR_Err_set_detail("Null MPI_Op");
        return MPI_ERR_OP;
    }
    if (op == MPI_NO_OP || op == MPI_REPLACE) {
        MPIR_Err_set_detail("MPI_Op operation is not allowed in this routine");
        return MPI_ERR_OP;
    }
    if (HANDLE_GET_MPI_KIND(op) != MPIR_OP_OBJ_KIND || HANDLE_GET_KIND(op) == HANDLE_KIND_INVALID) {
        MPIR_Err_set_detail("Invalid MPI_Op");
        return MPI_ERR_OP;
    }
    if (HANDLE_GET_KIND(op) != HANDLE_KIND_BUILTIN) {
        if (!user_op_get(op)) {         /* MPIR_Op_valid_ptr */
            MPIR_Err_set_detail("Invalid MPI_Op");
            return MPI_ERR_OP;
        }
    } else {
        MPIR_Op_check_dtype_fn *chk = MPIR_OP_HDL_TO_DTYPE_FN(op);
        if (!chk) {
            MPIR_Err_set_detail("Invalid MPI_Op");
            return MPI_ERR_OP;
        }
        mpi_errno = chk(datatype);
        if (mpi_errno != MPI_SUCCESS)
            return mpi_errno;
    }
    if (count != 0 && alias_check_enabled() && inbuf == inoutbuf) {
        MPIR_Err_set_detail("Buffers must not be aliased");
        return MPI_ERR_BUFFER;
    }
    if (count > 0 && inbuf == MPI_IN_PLACE) {
        MPIR_Err_set_detail("buffer 'inbuf' cannot be MPI_IN_PLACE");
        return MPI_ERR_BUFFER;
    }
    if (count > 0 && inoutbuf == MPI_IN_PLACE) {
        MPIR_Err_set_detail("buffer 'inoutbuf' cannot be MPI_IN_PLACE");
        return MPI_ERR_BUFFER;
    }
    return MPI_SUCCESS;
}

/* ---- user op on device buffers: the function is host code, so device ----
 * ---- operands are staged through host memory around the call.      ---- */
static int call_user_op(MPI_User_function * fn, const void *inbuf, void *inoutbuf, int count,
                        MPI_Datatype datatype)
{
    int in_dev = MPIR_Hip_is_device_ptr(inbuf);
    int io_dev = MPIR_Hip_is_device_ptr(inoutbuf);
    const MPIR_Type_desc *d;
    size_t bytes;
    void *hin = NULL, *hio = NULL;
    int rc = MPI_SUCCESS;

    if (!in_dev && !io_dev) {
        fn((void *) inbuf, inoutbuf, &count, &datatype);
        return MPI_SUCCESS;
    }
    d = MPIR_Type_lookup(datatype);
    if (!d || count < 0) {
        MPIR_Err_set_detail("user MPI_Op on device buffers needs a basic datatype");
        return MPI_ERR_TYPE;
    }
    bytes = (size_t) count * MPIR_Hip_elem_size(d->elem);
    hin = in_dev ? malloc(bytes ? bytes : 1) : (void *) inbuf;
    hio = io_dev ? malloc(bytes ? bytes : 1) : inoutbuf;
    if (!hin || !hio) {
        rc = MPI_ERR_NO_MEM;
        goto done;
    }
    if ((in_dev && MPIR_Hip_memcpy(hin, inbuf, bytes)) || (io_dev && MPIR_Hip_memcpy(hio, inoutbuf, bytes))) {
        MPIR_Err_set_detail("staging for user MPI_Op: %s", MPIR_Hip_error_string());
        rc = MPI_ERR_OTHER;
        goto done;
    }
    fn(hin, hio, &count, &datatype);
    if (io_dev && MPIR_Hip_memcpy(inoutbuf, hio, bytes)) {
        MPIR_Err_set_detail("staging for user MPI_Op: %s", MPIR_Hip_error_string());
        rc = MPI_ERR_OTHER;
    }
  done:
    if (in_dev && hin)
        free(hin);
    if (io_dev && hio)
        free(hio);
    return rc;
}

/* ---- MPIR_Reduce_local (reduce_local.c:35-122) -------------------------- */
int MPIR_Reduce_local(const void *inbuf, void *inoutbuf, int count, MPI_Datatype datatype, MPI_Op op)
{
    int mpi_errno = MPI_SUCCESS;
    int *op_errno;
    MPI_User_function *uop;

    if (count == 0)
        return MPI_SUCCESS;

    op_errno = MPIR_Op_errno_ptr();
    *op_errno = MPI_SUCCESS;

    if (HANDLE_GET_KIND(op) == HANDLE_KIND_BUILTIN) {
        uop = MPIR_OP_HDL_TO_FN(op);
        if (!uop) {
            MPIR_Err_set_detail("Invalid MPI_Op");
            return MPI_ERR_OP;
        }
        (*uop) ((void *) inbuf, inoutbuf, &count, &datatype);
    } else {
        /* MPIR_Op_get_ptr; a C-language op calls function.c_function (:65-82) */
        MPIR_Op *op_ptr = user_op_get(op);
        uop = op_ptr ? (MPI_User_function *) op_ptr->function.c_function : NULL;
        if (!uop) {
            MPIR_Err_set_detail("Invalid MPI_Op");
            return MPI_ERR_OP;
        }
        mpi_errno = call_user_op(uop, inbuf, inoutbuf, count, datatype);
        if (mpi_errno)
            return mpi_errno;
    }

    if (*op_errno)
        mpi_errno = *op_errno;
    return mpi_errno;
}

/* ---- MPI_Reduce_local (reduce_local.c:155-219) -------------------------- */
/* The body of PMPI_Reduce_local, under an internal name the LD_PRELOAD shim
 * (preload.c) also calls. */
int MPIR_Reduce_local_checked(const void *inbuf, void *inoutbuf, int count, MPI_Datatype datatype, MPI_Op op)
{
    static const char FCNAME[] = "PMPI_Reduce_local";
    int mpi_errno;
    MPIR_Dropin_cs_enter(MPIR_DROPIN_CS_GLOBAL);         /* reduce_local.c:162 */
    mpi_errno = validate(inbuf, inoutbuf, count, datatype, op);
    if (mpi_errno == MPI_SUCCESS)
        mpi_errno = MPIR_Reduce_local(inbuf, inoutbuf, count, datatype, op);
    if (mpi_errno != MPI_SUCCESS) {
        /* fn_fail (reduce_local.c:208-217) */
        mpi_errno = MPIR_Err_wrap_detail(FCNAME, __LINE__, mpi_errno);
        mpi_errno = MPIR_Err_create_code(mpi_errno, MPIR_ERR_RECOVERABLE, FCNAME, __LINE__, MPI_ERR_OTHER,
                                         "**mpi_reduce_local", "**mpi_reduce_local %p %p %d %D %O", inbuf,
                                         inoutbuf, count, datatype, op);
        mpi_errno = MPIR_Err_return_comm(NULL, FCNAME, mpi_errno);
    }
    MPIR_Dropin_cs_exit(MPIR_DROPIN_CS_GLOBAL);          /* reduce_local.c:205 */
    return mpi_errno;
}

#ifndef MPIR_PRELOAD_SHIM
int PMPI_Reduce_local(const void *inbuf, void *inoutbuf, int count, MPI_Datatype datatype, MPI_Op op)
{
    return MPIR_Reduce_local_checked(inbuf, inoutbuf, count, datatype, op);
}

/* profiling interface: MPI_ is a weak alias of PMPI_ (reduce_local.c:10-20) */
int MPI_Reduce_local(const void *inbuf, void *inoutbuf, int count, MPI_Datatype datatype, MPI_Op op)
    __attribute__ ((weak, alias("PMPI_Reduce_local")));
#endif

/* ---- MPIX_Reduce_local_stream: enqueue on a HIP stream, no wait -------- */
static int reduce_local_stream(const void *inbuf, void *inoutbuf, int count, MPI_Datatype datatype,
                               MPI_Op op, void *hip_stream);

/* the MPIX entry points validate user-op handles like MPI_Reduce_local does,
 * so they hold the same GLOBAL section */
int MPIX_Reduce_local_stream(const void *inbuf, void *inoutbuf, int count, MPI_Datatype datatype,
                             MPI_Op op, void *hip_stream)
{
    int rc;
    MPIR_Dropin_cs_enter(MPIR_DROPIN_CS_GLOBAL);
    rc = reduce_local_stream(inbuf, inoutbuf, count, datatype, op, hip_stream);
    MPIR_Dropin_cs_exit(MPIR_DROPIN_CS_GLOBAL);
    return rc;
}

static int reduce_local_stream(const void *inbuf, void *inoutbuf, int count, MPI_Datatype datatype,
                               MPI_Op op, void *hip_stream)
{
    int mpi_errno = validate(inbuf, inoutbuf, count, datatype, op);
    int opidx, elem, rc;
    if (mpi_errno != MPI_SUCCESS)
        return err_return("MPIX_Reduce_local_stream", mpi_errno);
    if (count <= 0)
        return MPI_SUCCESS;
    if (HANDLE_GET_KIND(op) != HANDLE_KIND_BUILTIN) {
        MPIR_Err_set_detail("user MPI_Op functions run on the host; use MPI_Reduce_local");
        return err_return("MPIX_Reduce_local_stream", MPI_ERR_OP);
    }
    opidx = op & 0xf;
    elem = MPIR_Op_resolve_elem(opidx, datatype);
    if (!elem) {        /* compute switch `default:` (LAND/LOR on floats) */
        MPIR_Err_set_detail("MPI_Op operation not defined for this datatype");
        return err_return("MPIX_Reduce_local_stream", MPI_ERR_OP);
    }
    rc = MPIR_Hip_reduce(inbuf, inoutbuf, (uint64_t) count, opidx, elem, hip_stream, 0);
    if (rc == MPIR_HIP_EBUFFER) {
        MPIR_Err_set_detail("MPIX_Reduce_local_stream needs device-resident buffers on one device");
        return err_return("MPIX_Reduce_local_stream", MPI_ERR_BUFFER);
    }
    if (rc != MPIR_HIP_OK) {
        MPIR_Op_report_hip_error("MPIX_Reduce_local_stream", rc);
        return err_return("MPIX_Reduce_local_stream", *MPIR_Op_errno_ptr());
    }
    return MPI_SUCCESS;
}

/* ---- MPIX_Reduce_local_multi: fused schedule steps (see the header) ---- */
static int reduce_local_multi(const void *const *inbufs, int n, void *outbuf, int count,
                              MPI_Datatype datatype, MPI_Op op, int order, void *hip_stream);

int MPIX_Reduce_local_multi(const void *const *inbufs, int n, void *outbuf, int count,
                            MPI_Datatype datatype, MPI_Op op, int order, void *hip_stream)
{
    int rc;
    MPIR_Dropin_cs_enter(MPIR_DROPIN_CS_GLOBAL);
    rc = reduce_local_multi(inbufs, n, outbuf, count, datatype, op, order, hip_stream);
    MPIR_Dropin_cs_exit(MPIR_DROPIN_CS_GLOBAL);
    return rc;
}

static int reduce_local_multi(const void *const *inbufs, int n, void *outbuf, int count,
                              MPI_Datatype datatype, MPI_Op op, int order, void *hip_stream)
{
    static const char *fc = "MPIX_Reduce_local_multi";
    int mpi_errno, opidx, elem, rc, j;
    if (n < 1 || n > 64 || !inbufs || (order != MPIX_ORDER_TREE && order != MPIX_ORDER_CHAIN)) {
        MPIR_Err_set_detail("invalid operand count or order");
        return err_return(fc, MPI_ERR_ARG);
    }
    if (order == MPIX_ORDER_TREE && (n & (n - 1))) {
        MPIR_Err_set_detail("MPIX_ORDER_TREE needs a power-of-two operand count");
        return err_return(fc, MPI_ERR_ARG);
    }
    for (j = 0; j < n; j++) {
        mpi_errno = validate(inbufs[j], outbuf, j == 0 ? 0 : count, datatype, op);
        if (mpi_errno != MPI_SUCCESS)
            return err_return(fc, mpi_errno);
    }
    if (count <= 0)
        return MPI_SUCCESS;
    if (HANDLE_GET_KIND(op) != HANDLE_KIND_BUILTIN) {
        MPIR_Err_set_detail("user MPI_Op functions run on the host; use MPI_Reduce_local");
        return err_return(fc, MPI_ERR_OP);
    }
    opidx = op & 0xf;
    elem = MPIR_Op_resolve_elem(opidx, datatype);
    if (!elem) {
        MPIR_Err_set_detail("MPI_Op operation not defined for this datatype");
        return err_return(fc, MPI_ERR_OP);
    }
    /* outbuf may be inbufs[0] exactly; any other overlap is refused whatever
     * MPIR_CVAR_COLL_ALIAS_CHECK says: the CHAIN path for n > 8 writes outbuf
     * between passes, before later operands are read */
    {
        const uintptr_t ob = (uintptr_t) outbuf;
        const uintptr_t nb = (uintptr_t) count * MPIR_Hip_elem_size(elem);
        for (j = 0; j < n; j++) {
            const uintptr_t ib = (uintptr_t) inbufs[j];
            if ((j > 0 || ib != ob) && ib < ob + nb && ob < ib + nb) {
                MPIR_Err_set_detail("inbufs[%d] overlaps outbuf (only inbufs[0] may be outbuf, exactly)", j);
                return err_return(fc, MPI_ERR_BUFFER);
            }
        }
    }
    rc = MPIR_Hip_combine(inbufs, n, outbuf, (uint64_t) count, opidx, elem,
                          order == MPIX_ORDER_TREE ? MPIR_HIP_ORDER_TREE : MPIR_HIP_ORDER_CHAIN,
                          hip_stream, hip_stream == NULL);
    if (rc == MPIR_HIP_EBUFFER) {
        MPIR_Err_set_detail("%s needs device-resident buffers on one device", fc);
        return err_return(fc, MPI_ERR_BUFFER);
    }
    if (rc != MPIR_HIP_OK) {
        MPIR_Op_report_hip_error(fc, rc);
        return err_return(fc, *MPIR_Op_errno_ptr());
    }
    return MPI_SUCCESS;
}

/* ---- MPI_Op_create / MPI_Op_free / MPI_Op_commutative ------------------ */
int PMPI_Op_create(MPI_User_function * user_fn, int commute, MPI_Op * op)
{
    int mpi_errno;
    MPIR_Dropin_cs_enter(MPIR_DROPIN_CS_GLOBAL);         /* op_create.c:151 */
    mpi_errno = MPIR_Op_create_impl(user_fn, commute, op);
    if (mpi_errno != MPI_SUCCESS)
        mpi_errno = err_return("PMPI_Op_create", mpi_errno);
    MPIR_Dropin_cs_exit(MPIR_DROPIN_CS_GLOBAL);
    return mpi_errno;
}

int MPI_Op_create(MPI_User_function * user_fn, int commute, MPI_Op * op)
    __attribute__ ((weak, alias("PMPI_Op_create")));

/* op_free.c:79-122: a predefined op is "**permop" */
int PMPI_Op_free(MPI_Op * op)
{
    int mpi_errno = MPI_SUCCESS;
    MPIR_Dropin_cs_enter(MPIR_DROPIN_CS_GLOBAL);         /* op_free.c:86 */
    if (HANDLE_GET_KIND(*op) == HANDLE_KIND_BUILTIN && HANDLE_GET_MPI_KIND(*op) == MPIR_OP_OBJ_KIND) {
        MPIR_Err_set_detail("Cannot free permanent MPI_Op");       /* "**permop" */
        mpi_errno = err_return("PMPI_Op_free", MPI_ERR_OP);
    } else if (!user_op_get(*op)) {
        MPIR_Err_set_detail("Invalid MPI_Op");
        mpi_errno = err_return("PMPI_Op_free", MPI_ERR_OP);
    } else {
        MPIR_Op_free_impl(op);
    }
    MPIR_Dropin_cs_exit(MPIR_DROPIN_CS_GLOBAL);          /* op_free.c:120 */
    return mpi_errno;
}

int MPI_Op_free(MPI_Op * op) __attribute__ ((weak, alias("PMPI_Op_free")));

/* op_commutative.c:39-53 */
int MPIR_Op_is_commutative(MPI_Op op)
{
    MPIR_Op *op_ptr;
    if (HANDLE_GET_KIND(op) == HANDLE_KIND_BUILTIN)
        return 1;
    op_ptr = MPIR_Op_get_ptr_fn(op);
    return !(op_ptr && op_ptr->kind == MPIR_OP_KIND__USER_NONCOMMUTE);
}

/* op_commutative.c:101-140 */
int PMPI_Op_commutative(MPI_Op op, int *commute)
{
    MPIR_Op *op_ptr = NULL;
    int mpi_errno;
    MPIR_Dropin_cs_enter(MPIR_DROPIN_CS_GLOBAL);         /* op_commutative.c:109 */
    if (HANDLE_GET_KIND(op) != HANDLE_KIND_BUILTIN)
        op_ptr = user_op_get(op);
    else if (HANDLE_GET_MPI_KIND(op) == MPIR_OP_OBJ_KIND)
        op_ptr = MPIR_Op_get_ptr_fn(op);
    if (!op_ptr) {
        MPIR_Err_set_detail("Invalid MPI_Op");
        mpi_errno = err_return("PMPI_Op_commutative", MPI_ERR_OP);
    } else {
        mpi_errno = MPIR_Op_commutative(op_ptr, commute);
    }
    MPIR_Dropin_cs_exit(MPIR_DROPIN_CS_GLOBAL);          /* op_commutative.c:136 */
    return mpi_errno;
}

int MPI_Op_commutative(MPI_Op op, int *commute) __attribute__ ((weak, alias("PMPI_Op_commutative")));

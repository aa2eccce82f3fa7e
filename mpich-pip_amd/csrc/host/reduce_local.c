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
 *   - error codes are the bare error classes (MPI_Error_class(c) == c);
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

#include "mpir_op_types.h"

/* ---- handle layout (src/include/mpir_objects.h:150,163-205) ------------ */
#define HANDLE_KIND_INVALID  0x0
#define HANDLE_KIND_BUILTIN  0x1
#define HANDLE_KIND_DIRECT   0x2
#define HANDLE_KIND_INDIRECT 0x3
#define HANDLE_GET_KIND(a)     (((unsigned)(a) & 0xc0000000u) >> 30)
#define HANDLE_GET_MPI_KIND(a) (((unsigned)(a) & 0x3c000000u) >> 26)
#define MPIR_OP_OBJ_KIND 0x6

/* ---- user op objects (op_create.c:73-104) ------------------------------ */
#define MPIR_OP_KIND__USER_NONCOMMUTE 32
#define MPIR_OP_KIND__USER 33
#define MAX_USER_OPS 4096
#define OP_PREALLOC 16          /* MPIR_OP_PREALLOC (op_create.c:27) */

typedef struct {
    int in_use;
    int kind;
    MPI_User_function *fn;
} user_op_t;

static user_op_t user_ops[MAX_USER_OPS];
static pthread_mutex_t user_ops_lock = PTHREAD_MUTEX_INITIALIZER;

/* direct handles 0x98000000|i for the first 16 objects, indirect
 * 0xd8000000|(block<<12)|index beyond (mpir_objects.h:183-205) */
static MPI_Op user_op_handle(int slot)
{
    if (slot < OP_PREALLOC)
        return (MPI_Op) (0x98000000u | (unsigned) slot);
    slot -= OP_PREALLOC;
    return (MPI_Op) (0xd8000000u | ((unsigned) (slot / 1024) << 12) | (unsigned) (slot % 1024));
}

static user_op_t *user_op_get(MPI_Op op)
{
    unsigned h = (unsigned) op;
    int slot;
    if (HANDLE_GET_MPI_KIND(h) != MPIR_OP_OBJ_KIND)
        return NULL;
    if (HANDLE_GET_KIND(h) == HANDLE_KIND_DIRECT) {
        slot = (int) (h & 0x03ffffffu);
        if (slot >= OP_PREALLOC)
            return NULL;
    } else if (HANDLE_GET_KIND(h) == HANDLE_KIND_INDIRECT) {
        slot = OP_PREALLOC + (int) (((h & 0x03fff000u) >> 12) * 1024 + (h & 0xfffu));
        if (slot >= MAX_USER_OPS)
            return NULL;
    } else {
        return NULL;
    }
    return user_ops[slot].in_use ? &user_ops[slot] : NULL;
}

/* ---- error handling ----------------------------------------------------- */
static MPI_Errhandler reduce_local_errhandler = MPI_ERRORS_ARE_FATAL;

static const char *class_string(int cls)
{
    switch (cls) {
    case MPI_SUCCESS:
        return "No MPI error";
    case MPI_ERR_BUFFER:
        return "Invalid buffer pointer";
    case MPI_ERR_COUNT:
        return "Invalid count";
    case MPI_ERR_TYPE:
        return "Invalid datatype";
    case 5:     /* MPI_ERR_COMM */
        return "Invalid communicator";
    case 7:     /* MPI_ERR_ROOT */
        return "Invalid root";
    case MPI_ERR_OP:
        return "Invalid MPI_Op";
    case MPI_ERR_ARG:
        return "Invalid argument";
    case MPI_ERR_OTHER:
        return "Other MPI error";
    case MPI_ERR_INTERN:
        return "Internal MPI error!";
    case MPI_ERR_NO_MEM:
        return "Out of memory";
    default:
        return "Unknown error class";
    }
}

int MPI_Error_class(int errorcode, int *errorclass)
{
    *errorclass = errorcode & 0x7f;     /* ERROR_CLASS_MASK (dynerrutil.c:40) */
    return MPI_SUCCESS;
}

int MPI_Error_string(int errorcode, char *string, int *resultlen)
{
    const char *detail = MPIR_Err_last_detail();
    int n;
    if (errorcode != MPI_SUCCESS && detail[0])
        n = snprintf(string, MPI_MAX_ERROR_STRING, "%s, error stack:\n%s",
                     class_string(errorcode & 0x7f), detail);
    else
        n = snprintf(string, MPI_MAX_ERROR_STRING, "%s", class_string(errorcode & 0x7f));
    if (n >= MPI_MAX_ERROR_STRING)
        n = MPI_MAX_ERROR_STRING - 1;
    *resultlen = n;
    return MPI_SUCCESS;
}

int MPIX_Reduce_local_set_errhandler(MPI_Errhandler errhandler)
{
    if (errhandler != MPI_ERRORS_ARE_FATAL && errhandler != MPI_ERRORS_RETURN)
        return MPI_ERR_ARG;
    reduce_local_errhandler = errhandler;
    return MPI_SUCCESS;
}

int MPIX_Reduce_local_get_errhandler(MPI_Errhandler * errhandler)
{
    *errhandler = reduce_local_errhandler;
    return MPI_SUCCESS;
}

/* MPIR_Err_return_comm(NULL, fcname, errcode) (errutil.c:238) */
int MPIR_Err_return(const char *fcname, int mpi_errno)
{
    if (reduce_local_errhandler == MPI_ERRORS_ARE_FATAL) {
        fprintf(stderr, "Fatal error in %s: %s, error stack:\n%s: %s\n", fcname,
                class_string(mpi_errno & 0x7f), fcname, MPIR_Err_last_detail());
        fflush(stderr);
        exit(1);
    }
    return mpi_errno;
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
        pthread_mutex_lock(&user_ops_lock);
        user_op_t *u = user_op_get(op);
        pthread_mutex_unlock(&user_ops_lock);
        if (!u) {       /* MPIR_Op_valid_ptr */
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
        user_op_t *u;
        pthread_mutex_lock(&user_ops_lock);
        u = user_op_get(op);
        uop = u ? u->fn : NULL;
        pthread_mutex_unlock(&user_ops_lock);
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
int PMPI_Reduce_local(const void *inbuf, void *inoutbuf, int count, MPI_Datatype datatype, MPI_Op op)
{
    int mpi_errno = validate(inbuf, inoutbuf, count, datatype, op);
    if (mpi_errno == MPI_SUCCESS)
        mpi_errno = MPIR_Reduce_local(inbuf, inoutbuf, count, datatype, op);
    if (mpi_errno != MPI_SUCCESS)
        mpi_errno = err_return("PMPI_Reduce_local", mpi_errno);
    return mpi_errno;
}

/* profiling interface: MPI_ is a weak alias of PMPI_ (reduce_local.c:10-20) */
int MPI_Reduce_local(const void *inbuf, void *inoutbuf, int count, MPI_Datatype datatype, MPI_Op op)
    __attribute__ ((weak, alias("PMPI_Reduce_local")));

/* ---- MPIX_Reduce_local_stream: enqueue on a HIP stream, no wait -------- */
int MPIX_Reduce_local_stream(const void *inbuf, void *inoutbuf, int count, MPI_Datatype datatype,
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
int MPIX_Reduce_local_multi(const void *const *inbufs, int n, void *outbuf, int count,
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
    int slot;
    pthread_mutex_lock(&user_ops_lock);
    for (slot = 0; slot < MAX_USER_OPS; slot++)
        if (!user_ops[slot].in_use)
            break;
    if (slot == MAX_USER_OPS) {
        pthread_mutex_unlock(&user_ops_lock);
        MPIR_Err_set_detail("Out of memory (MPI_Op)");
        return MPI_ERR_OTHER;   /* op_create.c:80-86 "**nomem" */
    }
    user_ops[slot].in_use = 1;
    user_ops[slot].kind = commute ? MPIR_OP_KIND__USER : MPIR_OP_KIND__USER_NONCOMMUTE;
    user_ops[slot].fn = user_fn;
    pthread_mutex_unlock(&user_ops_lock);
    *op = user_op_handle(slot);
    return MPI_SUCCESS;
}

int MPI_Op_create(MPI_User_function * user_fn, int commute, MPI_Op * op)
    __attribute__ ((weak, alias("PMPI_Op_create")));

int PMPI_Op_free(MPI_Op * op)
{
    user_op_t *u;
    pthread_mutex_lock(&user_ops_lock);
    u = user_op_get(*op);
    if (!u) {
        pthread_mutex_unlock(&user_ops_lock);
        if (HANDLE_GET_KIND(*op) == HANDLE_KIND_BUILTIN && HANDLE_GET_MPI_KIND(*op) == MPIR_OP_OBJ_KIND) {
            MPIR_Err_set_detail("Cannot free permanent MPI_Op");       /* op_free.c "**permop" */
            return err_return("PMPI_Op_free", MPI_ERR_OP);
        }
        MPIR_Err_set_detail("Invalid MPI_Op");
        return err_return("PMPI_Op_free", MPI_ERR_OP);
    }
    u->in_use = 0;
    u->fn = NULL;
    pthread_mutex_unlock(&user_ops_lock);
    *op = MPI_OP_NULL;
    return MPI_SUCCESS;
}

int MPI_Op_free(MPI_Op * op) __attribute__ ((weak, alias("PMPI_Op_free")));

int MPIR_Op_is_commutative(MPI_Op op)
{
    user_op_t *u;
    int kind;
    if (HANDLE_GET_KIND(op) == HANDLE_KIND_BUILTIN)
        return 1;
    pthread_mutex_lock(&user_ops_lock);
    u = user_op_get(op);
    kind = u ? u->kind : MPIR_OP_KIND__USER;
    pthread_mutex_unlock(&user_ops_lock);
    return kind == MPIR_OP_KIND__USER_NONCOMMUTE ? 0 : 1;
}

int PMPI_Op_commutative(MPI_Op op, int *commute)
{
    if (HANDLE_GET_KIND(op) != HANDLE_KIND_BUILTIN) {
        user_op_t *u;
        pthread_mutex_lock(&user_ops_lock);
        u = user_op_get(op);
        pthread_mutex_unlock(&user_ops_lock);
        if (!u) {
            MPIR_Err_set_detail("Invalid MPI_Op");
            return err_return("PMPI_Op_commutative", MPI_ERR_OP);
        }
    } else if (HANDLE_GET_MPI_KIND(op) != MPIR_OP_OBJ_KIND) {
        MPIR_Err_set_detail("Invalid MPI_Op");
        return err_return("PMPI_Op_commutative", MPI_ERR_OP);
    }
    *commute = MPIR_Op_is_commutative(op);
    return MPI_SUCCESS;
}

int MPI_Op_commutative(MPI_Op op, int *commute) __attribute__ ((weak, alias("PMPI_Op_commutative")));

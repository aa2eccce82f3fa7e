/*
 * mock_libmpi.c -- stands in for the parts of an MPICH 3.3 libmpi that stay
 * when INTEGRATION.md's Option 1 is applied: the collective schedules
 * (unchanged callers of MPIR_Reduce_local and of the inline MPIR_Op_get_ptr /
 * reference-count macros) and MPICH's own error routines.  The test compiles
 * it TOGETHER WITH the library's host sources (DROPIN_SRC) into one shared
 * object with -fvisibility=hidden, exactly as MPICH builds libmpi
 * (configure.ac:1443, mpi.h.in:13), and links libmpir_hip.so.
 *
 * What it proves (tests/test_integration_cpu.py):
 *   - the schedules bind to the drop-in MPIR_Reduce_local / MPIR_Op_table
 *     inside libmpi although neither is exported;
 *   - a user op made by the public MPI_Op_create is found by the inline
 *     handle macros (allreduce.c:419, mpidu_sched.c:800) and survives
 *     MPI_Op_free while a schedule holds a reference;
 *   - MPICH's strong MPIR_Err_create_code / MPIR_Err_return_comm /
 *     MPI_Error_class take over the library's weak standalone ones.
 */
#include <stdio.h>

#include "mpir_op_objects.h"
#include "mpir_op_types.h"

/* ---- "MPICH's" error routines (errutil.c:238, :848): strong definitions,
 * codes tagged 0x00100000 so the test can tell them from the weak ones */
static int mock_err_calls, mock_return_calls;
int MPIR_Err_create_code(int lastcode, int fatal, const char fcname[], int line, int error_class,
                         const char generic_msg[], const char specific_msg[], ...)
{
    (void) fatal, (void) fcname, (void) line, (void) generic_msg, (void) specific_msg;
    mock_err_calls++;
    if (error_class == MPI_ERR_OTHER && lastcode != MPI_SUCCESS)
        error_class = lastcode & 0x7f;
    return error_class | 0x00100000;
}

int MPIR_Err_return_comm(void *comm_ptr, const char fcname[], int errcode)
{
    (void) comm_ptr, (void) fcname;
    mock_return_calls++;
    return errcode;
}

int MPI_Error_class(int errorcode, int *errorclass)
{
    *errorclass = errorcode & 0x7f;
    return MPI_SUCCESS;
}

/* ---- a schedule step, the way unchanged libmpi code is written ---------- */
/* MPIR_Op_get_ptr -> MPIR_Getb_ptr (mpir_objects.h:441-460, 487) */
static MPIR_Op *op_get_ptr(MPI_Op a)
{
    switch (MPIR_HANDLE_GET_KIND(a)) {
    case MPIR_HANDLE_KIND_BUILTIN:
        return MPIR_Op_builtin + ((unsigned) a & 0x000000ffu);
    case MPIR_HANDLE_KIND_DIRECT:
        return MPIR_Op_direct + MPIR_HANDLE_INDEX(a);
    case MPIR_HANDLE_KIND_INDIRECT:
        if ((int) MPIR_HANDLE_BLOCK(a) >= MPIR_Op_mem.indirect_size)
            return NULL;
        return (MPIR_Op *) (void *) ((char *) (*MPIR_Op_mem.indirect)[MPIR_HANDLE_BLOCK(a)] +
                                     MPIR_HANDLE_BLOCK_INDEX(a) * MPIR_Op_mem.size);
    default:
        return NULL;
    }
}

/* public, like an MPI_ entry point: an "Ireduce" that holds the op
 * (MPIR_Op_add_ref_if_not_builtin, mpidu_sched.c:800), lets the caller free
 * it, then runs its reduce vertex (mpidu_sched.c:288) and releases
 * (MPIR_Op_release_if_not_builtin). Returns the reduce's code. */
__attribute__((visibility("default")))
int mock_sched_reduce(const void *in, void *inout, int count, MPI_Datatype dt, MPI_Op op, MPI_Op * user_handle)
{
    int rc, in_use;
    MPIR_Op *p = NULL;
    if (MPIR_HANDLE_GET_KIND(op) != MPIR_HANDLE_KIND_BUILTIN) {
        p = op_get_ptr(op);
        if (!p)
            return -1;
        p->ref_count++;
    }
    if (user_handle)
        MPI_Op_free(user_handle);       /* the application frees its handle early */
    rc = MPIR_Reduce_local(in, inout, count, dt, op);
    if (p) {
        in_use = --p->ref_count;
        if (!in_use) {                  /* MPIR_Handle_obj_free (mpir_handlemem.h:334-385) */
            ((MPIR_Handle_common *) (void *) p)->next = MPIR_Op_mem.avail;
            MPIR_Op_mem.avail = (MPIR_Handle_common *) (void *) p;
        }
    }
    return rc;
}

/* public: the schedules' view of the builtin table (allreduce.c:121-139) */
__attribute__((visibility("default")))
int mock_table_ok(void)
{
    return MPIR_Op_table[3] == MPIR_SUM && MPIR_OP_HDL_TO_DTYPE_FN(MPI_SUM) == MPIR_SUM_check_dtype &&
        MPIR_SUM_check_dtype(MPI_FLOAT) == MPI_SUCCESS && MPIR_SUM_check_dtype(MPI_BYTE) != MPI_SUCCESS;
}

/* public: the op's state after the schedule, and the error-routine counts */
__attribute__((visibility("default")))
int mock_op_refcount(MPI_Op op)
{
    MPIR_Op *p = op_get_ptr(op);
    return p ? p->ref_count : -1;
}

__attribute__((visibility("default")))
void mock_err_counts(int *created, int *returned)
{
    *created = mock_err_calls;
    *returned = mock_return_calls;
}

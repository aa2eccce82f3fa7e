/*
 * mock_libmpi.c -- stands in for the parts of an MPICH 3.3 libmpi that stay
 * when INTEGRATION.md's Option 1 is applied: the collective schedules
 * (unchanged callers of MPIR_Reduce_local and of the inline MPIR_Op_get_ptr /
 * reference-count macros), MPICH's per-thread state and critical sections
 * (tests/progs/mock_mpich/mpiimpl.h) and MPICH's own error routines.  The test
 * compiles it TOGETHER WITH the library's host sources (DROPIN_SRC) and
 * csrc/host/mpich_glue.c, with -DMPIR_DROPIN_IN_LIBMPI, into one shared object
 * with -fvisibility=hidden, exactly as MPICH builds libmpi (configure.ac:1443,
 * mpi.h.in:13), and links libmpir_hip.so.  One build per thread granularity
 * (MOCK_GRANULARITY 1 GLOBAL, 2 POBJ, 3 VCI).
 *
 * What it proves (tests/test_integration_cpu.py):
 *   - the schedules bind to the drop-in MPIR_Reduce_local / MPIR_Op_table
 *     inside libmpi although neither is exported;
 *   - a user op made by the public MPI_Op_create is found by the inline
 *     handle macros (allreduce.c:419, mpidu_sched.c:800) and survives
 *     MPI_Op_free while a schedule holds a reference;
 *   - MPICH's strong MPIR_Err_create_code / MPIR_Err_return_comm /
 *     MPI_Error_class take over the library's weak standalone ones;
 *   - an op error raised inside the drop-in lands in MPIR_Per_thread.op_errno,
 *     where a schedule that discards MPIR_Reduce_local's return value finds it
 *     (mock_sched_rsg_reduce, the shape of reduce_intra_reduce_scatter_gather.c);
 *   - MPI_Op_create / MPI_Op_free and libmpi's inline releases of
 *     schedule-held ops serialise on MPICH's own critical sections
 *     (mock_progress_*: a "progress engine" thread releasing ops while other
 *     threads create and free).
 */
#define _GNU_SOURCE             /* PTHREAD_RECURSIVE_MUTEX_INITIALIZER_NP */
#include <stdio.h>
#include <stdlib.h>

#include "mpiimpl.h"            /* tests/progs/mock_mpich/ */
#include "mpir_op_objects.h"
#include "mpir_op_types.h"

/* ---- "MPICH's" per-thread state and mutexes (mpir_thread.h, initthread.c) */
__thread MPIR_Per_thread_t MPIR_Per_thread;
MPID_Thread_tls_t MPIR_Per_thread_key;
MPIR_Thread_info_t MPIR_ThreadInfo;
MPID_Thread_mutex_t MPIR_THREAD_GLOBAL_ALLFUNC_MUTEX = { PTHREAD_RECURSIVE_MUTEX_INITIALIZER_NP, 1 };
#if MOCK_GRANULARITY == 2
MPID_Thread_mutex_t MPIR_THREAD_POBJ_HANDLE_MUTEX = { PTHREAD_MUTEX_INITIALIZER, 0 };
#else
MPID_Thread_mutex_t MPIR_THREAD_POBJ_HANDLE_MUTEX = { PTHREAD_RECURSIVE_MUTEX_INITIALIZER_NP, 1 };
#endif
int mock_cs_global_enters, mock_cs_handle_enters;

/* ---- "MPICH's" world and its node communicator (MPIR_Comm_commit) -------- */
MPIR_Process_t MPIR_Process;
static MPIR_Comm mock_world, mock_node;

/* n > 0: a node-aware world whose node communicator holds n ranks; 0: none */
__attribute__((visibility("default")))
void mock_set_node_ranks(int n)
{
    mock_node.local_size = n;
    mock_world.local_size = 2 * n;
    mock_world.node_comm = n > 0 ? &mock_node : NULL;
    MPIR_Process.comm_world = &mock_world;
}

/* MPI_Init_thread(MPI_THREAD_MULTIPLE) sets this (initthread.c) */
__attribute__((visibility("default")))
void mock_set_threaded(int on)
{
    MPIR_ThreadInfo.isThreaded = on;
}

__attribute__((visibility("default")))
void mock_cs_counts(int *global, int *handle)
{
    *global = __atomic_load_n(&mock_cs_global_enters, __ATOMIC_RELAXED);
    *handle = __atomic_load_n(&mock_cs_handle_enters, __ATOMIC_RELAXED);
}

/* ---- "MPICH's" error routines (errutil.c:238, :848): strong definitions,
 * codes tagged 0x00100000 so the test can tell them from the weak ones */
static int mock_err_calls, mock_return_calls;
int MPIR_Err_create_code(int lastcode, int fatal, const char fcname[], int line, int error_class,
                         const char generic_msg[], const char specific_msg[], ...)
{
    (void) fatal, (void) fcname, (void) line, (void) generic_msg, (void) specific_msg;
    __atomic_add_fetch(&mock_err_calls, 1, __ATOMIC_RELAXED);
    if (error_class == MPI_ERR_OTHER && lastcode != MPI_SUCCESS)
        error_class = lastcode & 0x7f;
    return error_class | 0x00100000;
}

int MPIR_Err_return_comm(void *comm_ptr, const char fcname[], int errcode)
{
    (void) comm_ptr, (void) fcname;
    __atomic_add_fetch(&mock_return_calls, 1, __ATOMIC_RELAXED);
    return errcode;
}

int MPI_Error_class(int errorcode, int *errorclass)
{
    *errorclass = errorcode & 0x7f;
    return MPI_SUCCESS;
}

/* ---- the op store as unchanged libmpi code touches it ------------------- */
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

/* MPIR_Op_add_ref_if_not_builtin (mpidu_sched.c:800; a lock-free ref count) */
static void op_add_ref(MPIR_Op * p)
{
    __atomic_add_fetch(&p->ref_count, 1, __ATOMIC_RELAXED);
}

/* MPIR_Op_release_if_not_builtin -> MPIR_Handle_obj_free (mpir_handlemem.h:334-385).
 * The spin between reading and writing the list head stands for a thread
 * preempted there: it widens the window in which an unserialised create
 * would pop the same head (the test's teeth -- with the drop-in's private
 * mutex instead of MPICH's sections the avail list ends up corrupt). */
static void op_release(MPIR_Op * p)
{
    if (__atomic_sub_fetch(&p->ref_count, 1, __ATOMIC_ACQ_REL) == 0) {
        MPID_THREAD_CS_ENTER(POBJ, MPIR_THREAD_POBJ_HANDLE_MUTEX);
        MPID_THREAD_CS_ENTER(VCI, MPIR_THREAD_POBJ_HANDLE_MUTEX);
        ((MPIR_Handle_common *) (void *) p)->next = MPIR_Op_mem.avail;
        for (volatile int spin = 0; spin < 2000; spin++);
        MPIR_Op_mem.avail = (MPIR_Handle_common *) (void *) p;
        MPID_THREAD_CS_EXIT(VCI, MPIR_THREAD_POBJ_HANDLE_MUTEX);
        MPID_THREAD_CS_EXIT(POBJ, MPIR_THREAD_POBJ_HANDLE_MUTEX);
    }
}

/* ---- a schedule step, the way unchanged libmpi code is written ---------- */
/* public, like an MPI_ entry point: an "Ireduce" that holds the op
 * (MPIR_Op_add_ref_if_not_builtin, mpidu_sched.c:800), lets the caller free
 * it, then runs its reduce vertex (mpidu_sched.c:288) and releases
 * (MPIR_Op_release_if_not_builtin). Returns the reduce's code. */
__attribute__((visibility("default")))
int mock_sched_reduce(const void *in, void *inout, int count, MPI_Datatype dt, MPI_Op op, MPI_Op * user_handle)
{
    int rc;
    MPIR_Op *p = NULL;
    if (MPIR_HANDLE_GET_KIND(op) != MPIR_HANDLE_KIND_BUILTIN) {
        p = op_get_ptr(op);
        if (!p)
            return -1;
        op_add_ref(p);
    }
    if (user_handle)
        MPI_Op_free(user_handle);       /* the application frees its handle early */
    rc = MPIR_Reduce_local(in, inout, count, dt, op);
    if (p)
        op_release(p);
    return rc;
}

/* public: the error protocol of reduce_intra_reduce_scatter_gather.c, the
 * long-message MPI_Reduce / SMP MPI_Allreduce schedule (config 4):
 *   per_thread->op_errno = 0                                   (:63-71)
 *   for each step: mpi_errno = MPIR_Reduce_local(tmp, recvbuf)  (:161, :241)
 *     -- the return value is never tested, and the next
 *        communication call overwrites it (the gather, :255-399)
 *   if (per_thread->op_errno) mpi_errno = op_errno; goto fn_fail (:401-412)
 * `steps` operand blocks are folded into inout one after another. */
__attribute__((visibility("default")))
int mock_sched_rsg_reduce(const void *const *tmp, int steps, void *inout, int count, MPI_Datatype dt, MPI_Op op)
{
    int mpi_errno = MPI_SUCCESS;
    {
        MPIR_Per_thread_t *per_thread = NULL;
        int err = 0;
        MPID_THREADPRIV_KEY_GET_ADDR(MPIR_ThreadInfo.isThreaded, MPIR_Per_thread_key,
                                     MPIR_Per_thread, per_thread, &err);
        MPIR_Assert(err == 0);
        per_thread->op_errno = 0;
    }
    for (int i = 0; i < steps; i++)
        mpi_errno = MPIR_Reduce_local(tmp[i], inout, count, dt, op);
    mpi_errno = MPI_SUCCESS;            /* the gather's MPIC_Send / MPIC_Recv */
    {
        MPIR_Per_thread_t *per_thread = NULL;
        int err = 0;
        MPID_THREADPRIV_KEY_GET_ADDR(MPIR_ThreadInfo.isThreaded, MPIR_Per_thread_key,
                                     MPIR_Per_thread, per_thread, &err);
        MPIR_Assert(err == 0);
        if (per_thread->op_errno)
            mpi_errno = per_thread->op_errno;
    }
    return mpi_errno;
}

/* public: the slot the schedules read, as libmpi sees it */
__attribute__((visibility("default")))
int mock_per_thread_op_errno(void)
{
    return MPIR_Per_thread.op_errno;
}

/* ---- a progress engine releasing schedule-held ops ---------------------- */
/* Under MPI_THREAD_MULTIPLE a nonblocking collective's reference to a user op
 * is dropped by whichever thread completes it inside the progress engine --
 * under the GLOBAL critical section of the MPI call it runs in (GLOBAL
 * granularity), or only under the handle mutex of MPIR_Handle_obj_free (POBJ,
 * VCI).  mock_progress_post is an "Ireduce" (holds a reference, then returns),
 * mock_progress_poll the progress engine completing posted ones. */
#define MOCK_QUEUE 65536       /* more than the test ever posts */
static MPIR_Op *posted[MOCK_QUEUE];
static int post_head, post_tail;
static pthread_mutex_t post_lock = PTHREAD_MUTEX_INITIALIZER;

__attribute__((visibility("default")))
int mock_progress_post(MPI_Op op)
{
    int ok = 0;
    MPID_THREAD_CS_ENTER(GLOBAL, MPIR_THREAD_GLOBAL_ALLFUNC_MUTEX);
    MPIR_Op *p = op_get_ptr(op);
    pthread_mutex_lock(&post_lock);
    if (p && post_tail - post_head < MOCK_QUEUE) {
        op_add_ref(p);
        posted[post_tail++ % MOCK_QUEUE] = p;
        ok = 1;
    }
    pthread_mutex_unlock(&post_lock);
    MPID_THREAD_CS_EXIT(GLOBAL, MPIR_THREAD_GLOBAL_ALLFUNC_MUTEX);
    return ok;
}

/* completes up to `max` posted operations; returns how many */
__attribute__((visibility("default")))
int mock_progress_poll(int max)
{
    int done = 0;
    MPID_THREAD_CS_ENTER(GLOBAL, MPIR_THREAD_GLOBAL_ALLFUNC_MUTEX);
    while (done < max) {
        MPIR_Op *p = NULL;
        pthread_mutex_lock(&post_lock);
        if (post_head < post_tail)
            p = posted[post_head++ % MOCK_QUEUE];
        pthread_mutex_unlock(&post_lock);
        if (!p)
            break;
        op_release(p);
        done++;
    }
    MPID_THREAD_CS_EXIT(GLOBAL, MPIR_THREAD_GLOBAL_ALLFUNC_MUTEX);
    return done;
}

/* the avail list after the run: every object of every block on it exactly
 * once (no lost, duplicated or foreign entries, no cycle); returns the number
 * of objects on the list, -1 if it is corrupt */
__attribute__((visibility("default")))
int mock_avail_check(int *total_objects)
{
    const int total = MPIR_Op_mem.direct_size + MPIR_Op_mem.indirect_size * MPIR_HANDLE_NUM_INDICES;
    char *seen = calloc((size_t) total + 1, 1);
    int n = 0;
    *total_objects = total;
    for (MPIR_Handle_common * h = MPIR_Op_mem.avail; h; h = (MPIR_Handle_common *) h->next) {
        MPIR_Op *p = op_get_ptr(h->handle);
        int idx;
        if ((void *) p != (void *) h || n > total) {
            free(seen);
            return -1;
        }
        idx = MPIR_HANDLE_GET_KIND(h->handle) == MPIR_HANDLE_KIND_DIRECT ? (int) MPIR_HANDLE_INDEX(h->handle) :
            MPIR_Op_mem.direct_size + (int) MPIR_HANDLE_BLOCK(h->handle) * MPIR_HANDLE_NUM_INDICES +
            (int) MPIR_HANDLE_BLOCK_INDEX(h->handle);
        if (idx < 0 || idx >= total || seen[idx]++) {
            free(seen);
            return -1;
        }
        n++;
    }
    free(seen);
    return n;
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

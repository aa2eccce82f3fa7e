/*
 * mock_app.c -- an application linked against tests/progs/mock_libmpi.c's
 * libmockmpi.so (the drop-in compiled into a hidden-visibility "libmpi" with
 * -DMPIR_DROPIN_IN_LIBMPI and csrc/host/mpich_glue.c).  Host buffers only:
 * runs without a GPU (the host combine needs no device).
 *
 * It also interposes MPIR_Hip_reduce, the device layer's entry point
 * (libmpir_hip.so), to make a chosen combine step fail the way a HIP runtime
 * failure does (MPIR_HIP_ERUNTIME) -- the executable's definition comes first
 * in the lookup order, and passes every other call on to the real one.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "mpi_reduce_local.h"

int mock_sched_reduce(const void *in, void *inout, int count, MPI_Datatype dt, MPI_Op op, MPI_Op * user_handle);
int mock_sched_rsg_reduce(const void *const *tmp, int steps, void *inout, int count, MPI_Datatype dt, MPI_Op op);
int mock_per_thread_op_errno(void);
int mock_op_refcount(MPI_Op op);
void mock_err_counts(int *created, int *returned);
int mock_table_ok(void);
void mock_set_threaded(int on);
void mock_cs_counts(int *global, int *handle);
int mock_progress_post(MPI_Op op);
int mock_progress_poll(int max);
int mock_avail_check(int *total_objects);
void mock_set_node_ranks(int n);

#define CHECK(c) do { if (!(c)) { fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); return 1; } } while (0)

/* ---- fault injection at the device layer -------------------------------- */
static int hip_calls, fault_first = -1, fault_last = -1;

int MPIR_Hip_reduce(const void *inbuf, void *inoutbuf, uint64_t count, int op, int elem, void *hip_stream, int sync)
{
    static int (*real)(const void *, void *, uint64_t, int, int, void *, int);
    const int k = hip_calls++;
    if (fault_first >= 0 && k >= fault_first && (fault_last < 0 || k <= fault_last))
        return 2;               /* MPIR_HIP_ERUNTIME */
    if (!real)
        real = (int (*)(const void *, void *, uint64_t, int, int, void *, int)) dlsym(RTLD_NEXT, "MPIR_Hip_reduce");
    return real(inbuf, inoutbuf, count, op, elem, hip_stream, sync);
}

static void twice_plus(void *in, void *inout, int *len, MPI_Datatype * dt)
{
    int *a = (int *) in, *b = (int *) inout;
    (void) dt;
    for (int i = 0; i < *len; i++)
        b[i] = 2 * b[i] + a[i];
}

static void nop_op(void *in, void *inout, int *len, MPI_Datatype * dt)
{
    (void) in, (void) inout, (void) len, (void) dt;
}

static int error_class(int rc)
{
    int cls = -1;
    MPI_Error_class(rc, &cls);
    return cls;
}

/* ---- op_errno through an unchanged schedule ----------------------------- */
static int check_op_errno(void)
{
    float t0[4] = { 1, 2, 3, 4 }, t1[4] = { 10, 20, 30, 40 }, t2[4] = { 100, 200, 300, 400 };
    float acc[4] = { 0.5f, 0.5f, 0.5f, 0.5f };
    const void *steps[3] = { t0, t1, t2 };

    /* a clean schedule: every step combined, nothing in op_errno */
    CHECK(mock_sched_rsg_reduce(steps, 3, acc, 4, MPI_FLOAT, MPI_SUM) == MPI_SUCCESS);
    CHECK(acc[0] == 111.5f && acc[3] == 444.5f);
    CHECK(mock_per_thread_op_errno() == MPI_SUCCESS);

    /* LAND on MPI_FLOAT passes check_dtype (opland.c:105-106) and fails in the
     * kernel's switch: each step's return is discarded, the schedule finds
     * MPI_ERR_OP in MPIR_Per_thread.op_errno (reduce_intra_reduce_scatter_gather.c:401-412) */
    CHECK(mock_sched_rsg_reduce(steps, 3, acc, 4, MPI_FLOAT, MPI_LAND) == MPI_ERR_OP);
    CHECK(mock_per_thread_op_errno() == MPI_ERR_OP);
    CHECK(acc[0] == 111.5f);            /* inout untouched, as in the reference */

    /* a device-layer failure from the second step on (a faulted device stays
     * faulted): MPI_ERR_OTHER reaches the schedule the same way */
    hip_calls = 0;
    fault_first = 1;
    fault_last = -1;
    CHECK(mock_sched_rsg_reduce(steps, 3, acc, 4, MPI_FLOAT, MPI_SUM) == MPI_ERR_OTHER);
    CHECK(mock_per_thread_op_errno() == MPI_ERR_OTHER);
    CHECK(acc[0] == 112.5f);            /* the first step ran */

    /* MPIR_Reduce_local resets op_errno on entry (reduce_local.c:51-59), so in
     * the reference a failure confined to a middle step is overwritten by the
     * next step's reset and the schedule returns success; the drop-in keeps
     * that protocol unchanged */
    hip_calls = 0;
    fault_first = 1;
    fault_last = 1;
    CHECK(mock_sched_rsg_reduce(steps, 3, acc, 4, MPI_FLOAT, MPI_SUM) == MPI_SUCCESS);
    fault_first = fault_last = -1;

    /* the public entry point reports the same failure through its error stack */
    hip_calls = 0;
    fault_first = 0;
    {
        int rc = MPI_Reduce_local(t0, acc, 4, MPI_FLOAT, MPI_SUM);
        CHECK(error_class(rc) == MPI_ERR_OTHER);
    }
    fault_first = -1;
    return 0;
}

/* ---- create / free / progress-engine releases on many threads ----------- */
#define WORKERS 8
#define ITERS 4000
static volatile int workers_done;
static int worker_errors;

static void *worker(void *arg)
{
    (void) arg;
    for (int i = 0; i < ITERS; i++) {
        MPI_Op op;
        int commute = -1;
        if (MPI_Op_create(nop_op, i & 1, &op) != MPI_SUCCESS) {
            __atomic_add_fetch(&worker_errors, 1, __ATOMIC_RELAXED);
            continue;
        }
        /* an "Ireduce" holds the op; the application frees its handle at
         * once; the progress engine drops the schedule's reference later */
        if (!mock_progress_post(op))
            __atomic_add_fetch(&worker_errors, 1, __ATOMIC_RELAXED);
        if (MPI_Op_commutative(op, &commute) != MPI_SUCCESS || commute != (i & 1))
            __atomic_add_fetch(&worker_errors, 1, __ATOMIC_RELAXED);
        if (MPI_Op_free(&op) != MPI_SUCCESS || op != MPI_OP_NULL)
            __atomic_add_fetch(&worker_errors, 1, __ATOMIC_RELAXED);
        /* some ops freed by the application first, some by the engine first */
        if ((i & 3) == 0)
            mock_progress_poll(2);
    }
    __atomic_add_fetch(&workers_done, 1, __ATOMIC_RELEASE);
    return NULL;
}

static void *progress(void *arg)
{
    (void) arg;
    while (__atomic_load_n(&workers_done, __ATOMIC_ACQUIRE) < WORKERS)
        mock_progress_poll(8);
    while (mock_progress_poll(64) > 0);
    return NULL;
}

static int check_threads(void)
{
    pthread_t w[WORKERS], pr;
    int total = 0, n, global = 0, handle = 0;
    mock_set_threaded(1);               /* MPI_Init_thread(MPI_THREAD_MULTIPLE) */
    CHECK(pthread_create(&pr, NULL, progress, NULL) == 0);
    for (int i = 0; i < WORKERS; i++)
        CHECK(pthread_create(&w[i], NULL, worker, NULL) == 0);
    for (int i = 0; i < WORKERS; i++)
        pthread_join(w[i], NULL);
    pthread_join(pr, NULL);
    CHECK(worker_errors == 0);
    n = mock_avail_check(&total);
    /* every object back on the avail list exactly once */
    CHECK(n >= 0 && n == total && total >= 16);
    mock_cs_counts(&global, &handle);
    CHECK(global > 0 || handle > 0);    /* MPICH's own sections were taken */
    printf("threads: %d creates, %d objects in store, global CS %d, handle CS %d\n", WORKERS * ITERS, total,
           global, handle);
    mock_set_threaded(0);
    return 0;
}

int main(void)
{
    int in[3] = { 1, 2, 3 }, io[3] = { 5, 6, 7 }, created = 0, returned = 0, rc;
    MPI_Op op, handle;
    int (*set_local_ranks)(int) = (int (*)(int)) dlsym(RTLD_DEFAULT, "MPIR_Hip_set_local_ranks");

    /* before MPI_Init's world exists the op layer passes nothing; then the
     * node communicator's size reaches the device layer at the next combine */
    CHECK(set_local_ranks != NULL);
    CHECK(mock_sched_reduce(in, io, 3, MPI_INT, MPI_SUM, NULL) == MPI_SUCCESS);
    CHECK(set_local_ranks(0) == 0);
    mock_set_node_ranks(3);
    CHECK(mock_sched_reduce(in, io, 3, MPI_INT, MPI_SUM, NULL) == MPI_SUCCESS);
    CHECK(set_local_ranks(3) == 3);
    io[0] = 5, io[1] = 6, io[2] = 7;

    CHECK(MPI_Op_create(twice_plus, 0, &op) == MPI_SUCCESS);
    handle = op;
    /* the schedule holds the op, the application frees it, the reduce still runs */
    CHECK(mock_sched_reduce(in, io, 3, MPI_INT, op, &handle) == MPI_SUCCESS);
    CHECK(handle == MPI_OP_NULL);
    CHECK(io[0] == 11 && io[1] == 14 && io[2] == 17);
    CHECK(mock_op_refcount(op) == 0);                  /* released by the schedule */
    /* a freed op is refused by the public entry point ... */
    rc = MPI_Reduce_local(in, io, 3, MPI_INT, op);
    CHECK(error_class(rc) == MPI_ERR_OP);
    /* ... and the failure went through libmpi's (strong) error routines */
    mock_err_counts(&created, &returned);
    CHECK((rc & 0x00100000) != 0 && created >= 2 && returned == 1);
    /* builtin ops: the schedules' MPIR_Op_table is the drop-in's */
    CHECK(mock_table_ok());
    CHECK(mock_sched_reduce(in, io, 0, MPI_INT, MPI_SUM, NULL) == MPI_SUCCESS);
    /* builtin op on host buffers, no GPU needed */
    CHECK(mock_sched_reduce(in, io, 3, MPI_INT, MPI_SUM, NULL) == MPI_SUCCESS);
    CHECK(io[0] == 12 && io[1] == 16 && io[2] == 20);
    if (check_op_errno())
        return 1;
    if (check_threads())
        return 1;
    puts("mock libmpi ok");
    return 0;
}

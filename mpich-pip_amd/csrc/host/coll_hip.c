/*
 * coll_hip.c -- device reduction collectives over RCCL / an in-process
 * loopback, built on the gfx950 MPIR_Reduce_local kernels.  See
 * include/mpix_hip_coll.h for the contract.
 *
 * Reference schedules reproduced (bit-identical results):
 *   Allreduce, one node: allreduce_intra_smp.c (MPIR_Reduce to node root via
 *     reduce_intra_reduce_scatter_gather.c:130-250, then MPIR_Bcast).
 *     Non-power-of-two pre-fold :138-170 (odd rank r < 2*rem sends to r-1,
 *     even computes x_r (+) x_{r+1}); recursive halving :186-249 leaves newrank
 *     n owning block bitrev(n), reduced as ((y0+y1)+(y2+y3))+... with
 *     y_j = contribution of newrank n ^ j (tests/test_schedule_fused_gpu.py).
 *   Reduce_scatter_block: reduce_scatter_block_intra_pairwise.c:75-134:
 *     block r = ((x_r + x_{r-1}) + x_{r-2}) + ... .
 * MI355X form: the log2(p) Sendrecv+Reduce_local rounds become one all-to-all
 * (every xGMI link busy at once) + one fused combine pass + one allgather.
 */
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include "mpix_hip_coll.h"
#include "mpir_op_types.h"

#define COMM_RCCL 1
#define COMM_LOOPBACK 2
#define MAX_XFER 256
#define REDUCE_SHORT_MSG_SIZE 2048            /* reduce.c:14-17 */
#define RSB_COMMUTATIVE_LONG_MSG_SIZE 524288  /* reduce_scatter.c:14-17 */

typedef struct {
    void *buf;
    size_t bytes;
    int peer;
} xfer_t;

/* ------------------------------------------------------------ RCCL (dlopen) */
static struct {
    int loaded;
    void *so;
    ncclResult_t (*GetUniqueId)(ncclUniqueId *);
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int);
    ncclResult_t (*CommDestroy)(ncclComm_t);
    ncclResult_t (*AllReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
    ncclResult_t (*ReduceScatter)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                                  hipStream_t);
    ncclResult_t (*Reduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, int, ncclComm_t,
                           hipStream_t);
    ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
    ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
    ncclResult_t (*GroupStart)(void);
    ncclResult_t (*GroupEnd)(void);
    const char *(*GetErrorString)(ncclResult_t);
} rccl;
static pthread_mutex_t rccl_lock = PTHREAD_MUTEX_INITIALIZER;

static int rccl_load(void)
{
    static const char *names[] = { "librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so" };
    /* TEST ONLY: a stand-in library that records the calls
     * (tests/progs/rccl_stub.c, tests/test_rccl_sequence_cpu.py) */
    const char *test_lib = getenv("MPIR_TEST_RCCL_LIBRARY");
    size_t i;
    pthread_mutex_lock(&rccl_lock);
    if (rccl.loaded) {
        pthread_mutex_unlock(&rccl_lock);
        return rccl.loaded > 0;
    }
    if (test_lib && *test_lib)
        rccl.so = dlopen(test_lib, RTLD_NOW | RTLD_GLOBAL);
    for (i = 0; i < sizeof(names) / sizeof(names[0]) && !rccl.so && !(test_lib && *test_lib); i++)
        rccl.so = dlopen(names[i], RTLD_NOW | RTLD_GLOBAL);
    if (rccl.so) {
#define SYM(f, n) *(void **) (&rccl.f) = dlsym(rccl.so, n)
        SYM(GetUniqueId, "ncclGetUniqueId");
        SYM(CommInitRank, "ncclCommInitRank");
        SYM(CommDestroy, "ncclCommDestroy");
        SYM(AllReduce, "ncclAllReduce");
        SYM(ReduceScatter, "ncclReduceScatter");
        SYM(Reduce, "ncclReduce");
        SYM(Send, "ncclSend");
        SYM(Recv, "ncclRecv");
        SYM(GroupStart, "ncclGroupStart");
        SYM(GroupEnd, "ncclGroupEnd");
        SYM(GetErrorString, "ncclGetErrorString");
#undef SYM
    }
    rccl.loaded = (rccl.so && rccl.GetUniqueId && rccl.CommInitRank && rccl.Send && rccl.Recv &&
                   rccl.GroupStart && rccl.GroupEnd && rccl.AllReduce && rccl.ReduceScatter && rccl.Reduce) ? 1 : -1;
    pthread_mutex_unlock(&rccl_lock);
    return rccl.loaded > 0;
}

static long cvar_long(const char *name, long dflt)
{
    const char *v = getenv(name);
    return v && *v ? strtol(v, NULL, 0) : dflt;
}

/* ------------------------------------------------------------ communicators */
typedef struct loop_hub {
    int size;
    int refs;
    pthread_barrier_t bar;
    pthread_mutex_t lock;
    struct {
        int nsend;
        xfer_t sends[MAX_XFER];
        hipEvent_t ready;
    } slot[64];
} loop_hub_t;

#define MAX_PIPE 16            /* chunks of a pipelined exchange (pipe_chunks) */

struct MPIX_Hip_comm_s {
    int kind, rank, size, device;
    hipStream_t stream;
    void *scratch;
    size_t scratch_bytes;
    ncclComm_t nccl;
    loop_hub_t *hub;
    /* pipelined schedules (pipe_chunks): the folds' stream, one event per
     * chunk's exchange and one per chunk's fold (created on first use) */
    hipStream_t fold_stream;
    hipEvent_t xev[MAX_PIPE], fev[MAX_PIPE];
};

static int hip_fail(const char *fc, hipError_t e)
{
    MPIR_Err_set_detail("%s: HIP error %s", fc, hipGetErrorString(e));
    return MPIR_Err_return(fc, MPI_ERR_OTHER);
}

static int comm_init_common(struct MPIX_Hip_comm_s *c)
{
    hipError_t e = hipGetDevice(&c->device);
    if (e == hipSuccess)
        e = hipStreamCreate(&c->stream);
    return e == hipSuccess ? 0 : (int) e;
}

int MPIX_Hip_comm_get_unique_id(void *id)
{
    ncclUniqueId u;
    ncclResult_t r;
    if (!rccl_load()) {
        MPIR_Err_set_detail("RCCL (librccl.so.1) could not be loaded");
        return MPIR_Err_return("MPIX_Hip_comm_get_unique_id", MPI_ERR_OTHER);
    }
    r = rccl.GetUniqueId(&u);
    if (r != ncclSuccess) {
        MPIR_Err_set_detail("ncclGetUniqueId: %s", rccl.GetErrorString ? rccl.GetErrorString(r) : "?");
        return MPIR_Err_return("MPIX_Hip_comm_get_unique_id", MPI_ERR_OTHER);
    }
    memcpy(id, &u, sizeof(u));
    return MPI_SUCCESS;
}

int MPIX_Hip_comm_create(const void *id, int size, int rank, MPIX_Hip_comm * comm)
{
    static const char *fc = "MPIX_Hip_comm_create";
    struct MPIX_Hip_comm_s *c;
    ncclUniqueId u;
    ncclResult_t r;
    int e;
    if (size < 1 || rank < 0 || rank >= size || size > 64) {
        MPIR_Err_set_detail("%s: invalid size/rank", fc);
        return MPIR_Err_return(fc, MPI_ERR_ARG);
    }
    if (!rccl_load()) {
        MPIR_Err_set_detail("RCCL (librccl.so.1) could not be loaded");
        return MPIR_Err_return(fc, MPI_ERR_OTHER);
    }
    c = calloc(1, sizeof(*c));
    c->kind = COMM_RCCL;
    c->rank = rank;
    c->size = size;
    if ((e = comm_init_common(c)) != 0) {
        free(c);
        return hip_fail(fc, (hipError_t) e);
    }
    memcpy(&u, id, sizeof(u));
    r = rccl.CommInitRank(&c->nccl, size, u, rank);
    if (r != ncclSuccess) {
        MPIR_Err_set_detail("ncclCommInitRank: %s", rccl.GetErrorString ? rccl.GetErrorString(r) : "?");
        (void) hipStreamDestroy(c->stream);
        free(c);
        return MPIR_Err_return(fc, MPI_ERR_OTHER);
    }
    *comm = c;
    return MPI_SUCCESS;
}

int MPIX_Hip_comm_create_loopback(int size, MPIX_Hip_comm * comms)
{
    static const char *fc = "MPIX_Hip_comm_create_loopback";
    loop_hub_t *hub;
    int r, e;
    if (size < 1 || size > 64) {
        MPIR_Err_set_detail("%s: size must be 1..64", fc);
        return MPIR_Err_return(fc, MPI_ERR_ARG);
    }
    hub = calloc(1, sizeof(*hub));
    hub->size = size;
    hub->refs = size;
    pthread_barrier_init(&hub->bar, NULL, (unsigned) size);
    pthread_mutex_init(&hub->lock, NULL);
    for (r = 0; r < size; r++) {
        struct MPIX_Hip_comm_s *c = calloc(1, sizeof(*c));
        c->kind = COMM_LOOPBACK;
        c->rank = r;
        c->size = size;
        c->hub = hub;
        if ((e = comm_init_common(c)) != 0)
            return hip_fail(fc, (hipError_t) e);
        if ((e = hipEventCreateWithFlags(&hub->slot[r].ready, hipEventDisableTiming)) != hipSuccess)
            return hip_fail(fc, (hipError_t) e);
        comms[r] = c;
    }
    return MPI_SUCCESS;
}

int MPIX_Hip_comm_free(MPIX_Hip_comm * comm)
{
    struct MPIX_Hip_comm_s *c = *comm;
    if (!c)
        return MPI_SUCCESS;
    (void) hipStreamSynchronize(c->stream);
    if (c->kind == COMM_RCCL && c->nccl && rccl.CommDestroy)
        rccl.CommDestroy(c->nccl);
    if (c->kind == COMM_LOOPBACK) {
        loop_hub_t *hub = c->hub;
        int last;
        pthread_mutex_lock(&hub->lock);
        last = --hub->refs == 0;
        pthread_mutex_unlock(&hub->lock);
        if (last) {
            int r;
            for (r = 0; r < hub->size; r++)
                (void) hipEventDestroy(hub->slot[r].ready);
            pthread_barrier_destroy(&hub->bar);
            pthread_mutex_destroy(&hub->lock);
            free(hub);
        }
    }
    if (c->scratch)
        (void) hipFree(c->scratch);
    if (c->fold_stream) {
        int k;
        (void) hipStreamSynchronize(c->fold_stream);
        for (k = 0; k < MAX_PIPE; k++) {
            (void) hipEventDestroy(c->xev[k]);
            (void) hipEventDestroy(c->fev[k]);
        }
        (void) hipStreamDestroy(c->fold_stream);
    }
    (void) hipStreamDestroy(c->stream);
    free(c);
    *comm = NULL;
    return MPI_SUCCESS;
}

int MPIX_Hip_comm_rank(MPIX_Hip_comm comm, int *rank)
{
    *rank = comm->rank;
    return MPI_SUCCESS;
}

int MPIX_Hip_comm_size(MPIX_Hip_comm comm, int *size)
{
    *size = comm->size;
    return MPI_SUCCESS;
}

static int comm_scratch(struct MPIX_Hip_comm_s *c, size_t bytes, char **out)
{
    if (c->scratch_bytes < bytes) {
        hipError_t e;
        if (c->scratch) {
            (void) hipStreamSynchronize(c->stream);
            (void) hipDeviceSynchronize();
            (void) hipFree(c->scratch);
        }
        c->scratch = NULL;
        c->scratch_bytes = 0;
        e = hipMalloc(&c->scratch, bytes);
        if (e != hipSuccess)
            return (int) e;
        c->scratch_bytes = bytes;
    }
    *out = c->scratch;
    return 0;
}

/* ------------------------------------------------------------ transport:
 * one group of point-to-point transfers that progress together (all xGMI
 * links at once); completes in stream order. */
static int group_exchange(struct MPIX_Hip_comm_s *c, const xfer_t *sends, int nsend, const xfer_t *recvs,
                          int nrecv, hipStream_t s)
{
    int i, j;
    if (c->kind == COMM_RCCL) {
        ncclResult_t r = rccl.GroupStart();
        for (i = 0; i < nsend && r == ncclSuccess; i++)
            if (sends[i].bytes)
                r = rccl.Send(sends[i].buf, sends[i].bytes, ncclUint8, sends[i].peer, c->nccl, s);
        for (i = 0; i < nrecv && r == ncclSuccess; i++)
            if (recvs[i].bytes)
                r = rccl.Recv(recvs[i].buf, recvs[i].bytes, ncclUint8, recvs[i].peer, c->nccl, s);
        {
            ncclResult_t r2 = rccl.GroupEnd();
            if (r == ncclSuccess)
                r = r2;
        }
        if (r != ncclSuccess) {
            MPIR_Err_set_detail("RCCL grouped send/recv: %s", rccl.GetErrorString ? rccl.GetErrorString(r) : "?");
            return MPI_ERR_OTHER;
        }
        return MPI_SUCCESS;
    } else {
        /* loopback: post sends + a ready event; every receiver copies from the
         * matching sender once that event has fired; barrier both sides so no
         * sender reuses a buffer before its readers are done */
        loop_hub_t *hub = c->hub;
        hipError_t e;
        if (nsend > MAX_XFER)
            return MPI_ERR_INTERN;
        hub->slot[c->rank].nsend = nsend;
        memcpy(hub->slot[c->rank].sends, sends, sizeof(xfer_t) * (size_t) nsend);
        e = hipEventRecord(hub->slot[c->rank].ready, s);
        pthread_barrier_wait(&hub->bar);
        for (i = 0; i < nrecv && e == hipSuccess; i++) {
            int peer = recvs[i].peer, found = 0;
            for (j = 0; j < hub->slot[peer].nsend; j++) {
                const xfer_t *x = &hub->slot[peer].sends[j];
                if (x->peer == c->rank) {
                    if (x->bytes != recvs[i].bytes) {
                        MPIR_Err_set_detail("loopback: size mismatch %zu vs %zu", x->bytes, recvs[i].bytes);
                        pthread_barrier_wait(&hub->bar);
                        return MPI_ERR_INTERN;
                    }
                    e = hipStreamWaitEvent(s, hub->slot[peer].ready, 0);
                    if (e == hipSuccess && x->bytes)
                        e = hipMemcpyAsync(recvs[i].buf, x->buf, x->bytes, hipMemcpyDeviceToDevice, s);
                    found = 1;
                    break;
                }
            }
            if (!found && recvs[i].bytes) {
                MPIR_Err_set_detail("loopback: no matching send from %d", peer);
                pthread_barrier_wait(&hub->bar);
                return MPI_ERR_INTERN;
            }
        }
        if (e == hipSuccess)
            e = hipStreamSynchronize(s);
        pthread_barrier_wait(&hub->bar);
        if (e != hipSuccess) {
            MPIR_Err_set_detail("loopback transfer: %s", hipGetErrorString(e));
            return MPI_ERR_OTHER;
        }
        return MPI_SUCCESS;
    }
}

/* ------------------------------------------------------------ pipelining
 * The reference-order schedules move every block first and fold after (the
 * reference's rounds are step-serial too, allreduce_intra_reduce_scatter_
 * allgather.c:170-260, reduce_scatter_block_intra_pairwise.c:97-134).  For
 * large blocks the exchange is cut into chunks -- byte ranges [k * chunk, ...)
 * of every transfer, one group per chunk on every rank -- and chunk k's fold
 * runs on the communicator's fold stream while chunk k+1 moves: the folds
 * hide behind the transfers.  Element-wise folds over the same operands in the
 * same order: the results are bit-identical to the unchunked schedule.  The
 * pipelined folds keep their LDS cap: beside RCCL's kernel the capped fold
 * leaves it faster than the uncapped one (a one-rank all_reduce 56.9 against
 * 71.2 us, 21.8 alone), and in the pipeline the two are within
 * 1 % (tools/archive/pipeline_overlap.cpp, profiles/r06/pipeline_overlap.log); a caller
 * that wants the other choice has MPIR_Hip_combine_set_flags.
 * MPIR_CVAR_DEVICE_COLL_PIPELINE_KB: the chunk (default 32768 = 32 MiB; 0 =
 * never pipeline); a schedule pipelines when its largest block spans at least
 * two chunks, in at most MAX_PIPE chunks. */
static int pipe_chunks(size_t block_bytes, size_t * chunk)
{
    long kb = cvar_long("MPIR_CVAR_DEVICE_COLL_PIPELINE_KB", 32768);
    size_t ch, n;
    if (kb <= 0)
        return 1;
    ch = ((size_t) kb << 10) & ~(size_t) 255;
    if (ch < 256 || block_bytes < 2 * ch)
        return 1;
    n = (block_bytes + ch - 1) / ch;
    if (n > MAX_PIPE) {
        ch = ((block_bytes + MAX_PIPE - 1) / MAX_PIPE + 255) & ~(size_t) 255;
        n = (block_bytes + ch - 1) / ch;
    }
    *chunk = ch;
    return (int) n;
}

static int pipe_init(struct MPIX_Hip_comm_s *c)
{
    hipError_t e = hipSuccess;
    int k;
    if (c->fold_stream)
        return MPI_SUCCESS;
    for (k = 0; k < MAX_PIPE && e == hipSuccess; k++) {
        e = hipEventCreateWithFlags(&c->xev[k], hipEventDisableTiming);
        if (e == hipSuccess)
            e = hipEventCreateWithFlags(&c->fev[k], hipEventDisableTiming);
    }
    if (e == hipSuccess)
        e = hipStreamCreate(&c->fold_stream);
    if (e != hipSuccess) {
        MPIR_Err_set_detail("pipelined schedule: %s", hipGetErrorString(e));
        return MPI_ERR_OTHER;
    }
    return MPI_SUCCESS;
}

/* chunk k of a transfer list: [k * chunk, min((k + 1) * chunk, bytes)) of each
 * (empty past its end: both sides compute it from the same block size) */
static void chunk_of(const xfer_t *x, int n, int k, size_t chunk, xfer_t *out)
{
    int i;
    for (i = 0; i < n; i++) {
        size_t off = (size_t) k * chunk;
        out[i].peer = x[i].peer;
        out[i].buf = (char *) x[i].buf + (off < x[i].bytes ? off : x[i].bytes);
        out[i].bytes = off < x[i].bytes ? (x[i].bytes - off < chunk ? x[i].bytes - off : chunk) : 0;
    }
}

/* The fold of one chunk: `len` bytes at byte offset `off` of the schedule's
 * output, on stream fs. */
typedef int (*chunk_fold_fn)(void *ctx, size_t off, size_t len, hipStream_t fs);

/* Exchange `sends` / `recvs` in nchunk groups on s; after group k, fold(k)
 * on the fold stream, ordered after it by xev[k]; fev[k] marks fold k done.
 * `out_bytes` is the fold's output length (its chunks are [k * chunk, ...)). */
static int exchange_fold_pipelined(struct MPIX_Hip_comm_s *c, const xfer_t *sends, int nsend, const xfer_t *recvs,
                                   int nrecv, int nchunk, size_t chunk, size_t out_bytes, hipStream_t s,
                                   chunk_fold_fn fold, void *ctx)
{
    xfer_t sk[MAX_XFER], rk[MAX_XFER];
    int k, rc = MPI_SUCCESS;
    hipError_t e = hipSuccess;
    for (k = 0; k < nchunk && rc == MPI_SUCCESS; k++) {
        size_t off = (size_t) k * chunk;
        chunk_of(sends, nsend, k, chunk, sk);
        chunk_of(recvs, nrecv, k, chunk, rk);
        if ((rc = group_exchange(c, sk, nsend, rk, nrecv, s)) != MPI_SUCCESS)
            break;
        if ((e = hipEventRecord(c->xev[k], s)) != hipSuccess ||
            (e = hipStreamWaitEvent(c->fold_stream, c->xev[k], 0)) != hipSuccess)
            break;
        if (off < out_bytes &&
            (rc = fold(ctx, off, out_bytes - off < chunk ? out_bytes - off : chunk, c->fold_stream)) != MPI_SUCCESS)
            break;
        if ((e = hipEventRecord(c->fev[k], c->fold_stream)) != hipSuccess)
            break;
    }
    if (e != hipSuccess) {
        MPIR_Err_set_detail("pipelined schedule: %s", hipGetErrorString(e));
        return MPI_ERR_OTHER;
    }
    return rc;
}

/* ------------------------------------------------------------ helpers */
/* Byte stride between staging slots.  Slots at a power-of-two stride (equal
 * blocks of a power-of-two message) put the P operand streams of a fused
 * combine on the same HBM channels at the same moment: 8 x 32 MiB TREE8 fp32
 * ran at 0.689 of the HBM peak with a 32 MiB stride, 0.767 with 32 MiB +
 * 4352 B (4 KiB + 256), 0.717 with + 256 B only (rocprofv3 kernel trace,
 * tools/multi_gap_ab.hip, profiles/archive/r01s3_multi_skew_ab.log).  The best
 * skew depends on the block size (the address bits the blocks themselves set):
 * around 128 MiB blocks (config 5's 8 x 128 MiB CHAIN8) 6400 B ran 1.3-4.5
 * points above 4352 B in seven sweeps on five boxes, at 32 / 64 MiB 0.3-1 point
 * below it, at 256 MiB within a point (tools/archive/fold_skew.hip, chain_shape.hip
 * slabskew; profiles/r05/fold_skew*.log, slabskew.log).  The skew keeps the
 * 256 B alignment (fused kernels need the operands equal mod 16). */
static size_t stage_stride(size_t bytes)
{
    size_t st = (bytes + 255) & ~(size_t) 255;
    if (st >= ((size_t) 96 << 20) && st < ((size_t) 192 << 20))
        return st + 6400;
    return st >= ((size_t) 1 << 20) ? st + 4352 : st;
}

static int pof2_of(int p)
{
    int q = 1;
    while (q * 2 <= p)
        q *= 2;
    return q;
}

static int bitrev(int n, int bits)
{
    int r = 0, i;
    for (i = 0; i < bits; i++)
        if (n & (1 << i))
            r |= 1 << (bits - 1 - i);
    return r;
}

static void cnts_disps(long count, int pof2, long *cnts, long *disps)
{
    int i;
    for (i = 0; i < pof2; i++)
        cnts[i] = count / pof2 + (i < count % pof2 ? 1 : 0);
    disps[0] = 0;
    for (i = 1; i < pof2; i++)
        disps[i] = disps[i - 1] + cnts[i - 1];
}

/* MPIR_Allreduce_intra_auto's branch (allreduce.c:145-217) from the CVARs a
 * user can set (defaults in brackets): MPIR_CVAR_ENABLE_SMP_COLLECTIVES [1],
 * MPIR_CVAR_ENABLE_SMP_ALLREDUCE [1], MPIR_CVAR_MAX_SMP_ALLREDUCE_MSG_SIZE [0],
 * MPIR_CVAR_ALLREDUCE_SHORT_MSG_SIZE [2048].  The device communicator is taken
 * as node-aware (one node).  Note the reference's nbytes: it is 0 unless
 * MAX_SMP_ALLREDUCE_MSG_SIZE is set (:159), so the flat branch then always picks
 * recursive doubling. */
#define FLAT_NO 0
#define FLAT_RECURSIVE_DOUBLING 1
#define FLAT_RABENSEIFNER 2
static int allreduce_flat_choice(size_t bytes, long count, int pof2)
{
    const long max_smp = cvar_long("MPIR_CVAR_MAX_SMP_ALLREDUCE_MSG_SIZE", 0);
    const long nbytes = max_smp ? (long) bytes : 0;
    if (cvar_long("MPIR_CVAR_ENABLE_SMP_COLLECTIVES", 1) && cvar_long("MPIR_CVAR_ENABLE_SMP_ALLREDUCE", 1) &&
        nbytes <= max_smp)
        return FLAT_NO;
    if (nbytes <= cvar_long("MPIR_CVAR_ALLREDUCE_SHORT_MSG_SIZE", 2048) || count < pof2)
        return FLAT_RECURSIVE_DOUBLING;
    return FLAT_RABENSEIFNER;
}

/* real rank of newrank m after the pre-fold: the keeper of pair m is the even
 * rank 2m (reduce_intra_reduce_scatter_gather.c) or the odd rank 2m+1
 * (allreduce_intra_reduce_scatter_allgather.c, allreduce_intra_recursive_doubling.c) */
static int real_of(int m, int rem, int odd_keeps)
{
    return m < rem ? 2 * m + (odd_keeps ? 1 : 0) : m + rem;
}

/* ------------------------------------------------------------ short messages
 * MPICH switches algorithm on message size.  For these the device form keeps
 * the reference's association and operand order but not its rounds: ONE
 * exchange brings a rank every operand it needs, then the schedule's fold runs
 * on the device (tests/test_schedule_small_cpu.py pins the fold plans against
 * step-by-step simulations of the reference). */
static int hip_err(const char *fc, hipError_t e)
{
    MPIR_Err_set_detail("%s: HIP error %s", fc, hipGetErrorString(e));
    return MPI_ERR_OTHER;
}

static int fold_tree(const void *const *ys, int n, void *out, long count, int opidx, int elem, hipStream_t s,
                     const char *fc)
{
    int rc = MPIR_Hip_combine(ys, n, out, (uint64_t) count, opidx, elem, MPIR_HIP_ORDER_TREE, s, 0);
    if (rc) {
        MPIR_Op_report_hip_error(fc, rc);
        return MPI_ERR_OTHER;
    }
    return MPI_SUCCESS;
}

static int fold_step(const void *src, void *dst, long count, int opidx, int elem, hipStream_t s, const char *fc)
{
    int rc = MPIR_Hip_reduce(src, dst, (uint64_t) count, opidx, elem, s, 0);
    if (rc) {
        MPIR_Op_report_hip_error(fc, rc);
        return MPI_ERR_OTHER;
    }
    return MPI_SUCCESS;
}

/* MPI_Allreduce, count*size <= 2048 or count < pof2: MPIR_Reduce takes the
 * binomial tree to root 0 (reduce.c:214-225, reduce_intra_binomial.c:93-140:
 * relrank r folds in the accumulation of r|mask as the second operand), then
 * MPIR_Bcast.  Here: an allgather of the p inputs into slots 0..p-1, then every
 * rank folds them in the binomial order itself, so all ranks hold root 0's bytes. */
static int allreduce_short(struct MPIX_Hip_comm_s *c, const void *sendbuf, void *recvbuf, long count,
                           size_t esz, int opidx, int elem, hipStream_t s, const char *fc)
{
    int p = c->size, q, nx = 0, rc = MPI_SUCCESS, mask;
    size_t bytes = (size_t) count * esz, slot = stage_stride(bytes);
    xfer_t sends[MAX_XFER], recvs[MAX_XFER];
    const void *ys[64];
    char *scr = NULL, *own;
    hipError_t e;
    if (comm_scratch(c, (size_t) p * slot, &scr)) {
        MPIR_Err_set_detail("%s: scratch allocation failed", fc);
        return MPI_ERR_NO_MEM;
    }
    own = scr + (size_t) c->rank * slot;
    e = hipMemcpyAsync(own, sendbuf == MPI_IN_PLACE ? recvbuf : sendbuf, bytes, hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess)
        return hip_err(fc, e);
    for (q = 0; q < p; q++) {
        if (q == c->rank)
            continue;
        sends[nx].buf = own;
        sends[nx].bytes = bytes;
        sends[nx].peer = q;
        recvs[nx].buf = scr + (size_t) q * slot;
        recvs[nx].bytes = bytes;
        recvs[nx++].peer = q;
    }
    if ((rc = group_exchange(c, sends, nx, recvs, nx, s)) != MPI_SUCCESS)
        return rc;
    if ((p & (p - 1)) == 0) {
        /* power of two: the binomial tree IS the pairwise tree ((x0+x1)+(x2+x3))+... */
        for (q = 0; q < p; q++)
            ys[q] = scr + (size_t) q * slot;
        return fold_tree(ys, p, recvbuf, count, opidx, elem, s, fc);
    }
    for (mask = 1; mask < p; mask <<= 1)
        for (q = 0; q + mask < p; q += 2 * mask)
            if ((rc = fold_step(scr + (size_t) (q + mask) * slot, scr + (size_t) q * slot, count, opidx, elem,
                                s, fc)) != MPI_SUCCESS)
                return rc;
    e = hipMemcpyAsync(recvbuf, scr, bytes, hipMemcpyDeviceToDevice, s);
    return e == hipSuccess ? MPI_SUCCESS : hip_err(fc, e);
}

/* MPI_Allreduce, flat branch, recursive doubling
 * (allreduce_intra_recursive_doubling.c): even r < 2*rem sends to r+1, which
 * computes Y = x_{r} (+) x_{r-1}; then at mask 1, 2, 4, ... newrank n folds in
 * the partial of n ^ mask second, so n ends with the tree over z_j = Y_{n ^ j};
 * an excluded even rank receives the result of its odd neighbour.  Here: an
 * allgather of the p inputs, the rem pre-fold steps, one tree combine per rank. */
static int allreduce_recursive_doubling(struct MPIX_Hip_comm_s *c, const void *sendbuf, void *recvbuf,
                                        long count, size_t esz, int opidx, int elem, hipStream_t s,
                                        const char *fc)
{
    int p = c->size, q, nx = 0, rc = MPI_SUCCESS, pof2 = pof2_of(p), rem = p - pof2, n, j, m;
    size_t bytes = (size_t) count * esz, slot = stage_stride(bytes);
    xfer_t sends[MAX_XFER], recvs[MAX_XFER];
    const void *ys[64];
    char *scr = NULL, *own;
    hipError_t e;
    if (comm_scratch(c, (size_t) p * slot, &scr)) {
        MPIR_Err_set_detail("%s: scratch allocation failed", fc);
        return MPI_ERR_NO_MEM;
    }
    own = scr + (size_t) c->rank * slot;
    e = hipMemcpyAsync(own, sendbuf == MPI_IN_PLACE ? recvbuf : sendbuf, bytes, hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess)
        return hip_err(fc, e);
    for (q = 0; q < p; q++) {
        if (q == c->rank)
            continue;
        sends[nx].buf = own;
        sends[nx].bytes = bytes;
        sends[nx].peer = q;
        recvs[nx].buf = scr + (size_t) q * slot;
        recvs[nx].bytes = bytes;
        recvs[nx++].peer = q;
    }
    if ((rc = group_exchange(c, sends, nx, recvs, nx, s)) != MPI_SUCCESS)
        return rc;
    for (m = 0; m < rem; m++)
        if ((rc = fold_step(scr + (size_t) (2 * m) * slot, scr + (size_t) (2 * m + 1) * slot, count, opidx,
                            elem, s, fc)) != MPI_SUCCESS)
            return rc;
    n = c->rank < 2 * rem ? c->rank / 2 : c->rank - rem;
    for (j = 0; j < pof2; j++)
        ys[j] = scr + (size_t) real_of(n ^ j, rem, 1) * slot;
    return fold_tree(ys, pof2, recvbuf, count, opidx, elem, s, fc);
}

/* MPI_Reduce_scatter(_block), total bytes < 524288: recursive halving
 * (reduce_scatter_block_intra_recursive_halving.c; reduce_scatter_intra_
 * recursive_halving.c is the same schedule with per-rank counts).  Block r is
 * finished by newrank n = r/2 (r < 2*rem) or r - rem, as
 *   Y_m = x_{2m+1} (+) x_{2m} for m < rem (pre-fold :163-195), else x_{m+rem};
 *   tree ((z0+z1)+(z2+z3))+... over z_k = Y_{n ^ bitrev(k)} (halving :197-283,
 *   mask = pof2/2 first, received data second).
 * Here: one all-to-all of blocks (every rank gets x_q's block r from each q),
 * the rem pre-fold steps, one tree combine into recvbuf. */
static int reduce_scatter_short(struct MPIX_Hip_comm_s *c, const char *src, void *recvbuf, const long *cnts,
                                const long *disps, size_t esz, int opidx, int elem, hipStream_t s, const char *fc)
{
    int p = c->size, q, nx = 0, rc = MPI_SUCCESS, pof2 = pof2_of(p), rem = p - pof2, bits = 0, n, k, m;
    long rcount = cnts[c->rank];
    size_t nb = (size_t) rcount * esz, slot = stage_stride(nb);
    xfer_t sends[MAX_XFER], recvs[MAX_XFER];
    const void *ys[64];
    char *scr = NULL;
    hipError_t e;
    while ((1 << bits) < pof2)
        bits++;
    if (comm_scratch(c, (size_t) p * slot + 256, &scr)) {
        MPIR_Err_set_detail("%s: scratch allocation failed", fc);
        return MPI_ERR_NO_MEM;
    }
    /* own block into its slot: the pre-fold updates slots in place */
    if (nb) {
        e = hipMemcpyAsync(scr + (size_t) c->rank * slot, src + (size_t) disps[c->rank] * esz, nb,
                           hipMemcpyDeviceToDevice, s);
        if (e != hipSuccess)
            return hip_err(fc, e);
    }
    for (q = 0; q < p; q++) {
        if (q == c->rank)
            continue;
        sends[nx].buf = (void *) (src + (size_t) disps[q] * esz);
        sends[nx].bytes = (size_t) cnts[q] * esz;
        sends[nx].peer = q;
        recvs[nx].buf = scr + (size_t) q * slot;
        recvs[nx].bytes = nb;
        recvs[nx++].peer = q;
    }
    if ((rc = group_exchange(c, sends, nx, recvs, nx, s)) != MPI_SUCCESS)
        return rc;
    if (!rcount)
        return MPI_SUCCESS;
    for (m = 0; m < rem; m++)
        if ((rc = fold_step(scr + (size_t) (2 * m) * slot, scr + (size_t) (2 * m + 1) * slot, rcount, opidx,
                            elem, s, fc)) != MPI_SUCCESS)
            return rc;
    n = c->rank < 2 * rem ? c->rank / 2 : c->rank - rem;
    for (k = 0; k < pof2; k++) {
        int y = n ^ bitrev(k, bits);
        ys[k] = scr + (size_t) (y < rem ? 2 * y + 1 : y + rem) * slot;
    }
    return fold_tree(ys, pof2, recvbuf, rcount, opidx, elem, s, fc);
}

/* the pipelined folds: operands and output shifted by the chunk's offset */
typedef struct {
    const void *const *ys;
    int n, order, opidx, elem;
    char *out;
    size_t esz;
    const char *fc;
} fold_ctx_t;

static int chunk_fold(void *ctx, size_t off, size_t len, hipStream_t fs)
{
    const fold_ctx_t *f = ctx;
    const void *ys[64];
    int i, rc;
    for (i = 0; i < f->n; i++)
        ys[i] = (const char *) f->ys[i] + off;
    rc = MPIR_Hip_combine(ys, f->n, f->out + off, (uint64_t) (len / f->esz), f->opidx, f->elem, f->order, fs, 0);
    if (rc) {
        MPIR_Op_report_hip_error(f->fc, rc);
        return MPI_ERR_OTHER;
    }
    return MPI_SUCCESS;
}

/* validation shared by the collectives (MPIR_ERRTEST_OP + check_dtype) */
static int coll_check(const char *fc, const void *sendbuf, void *recvbuf, int count, MPI_Datatype dt, MPI_Op op,
                      MPIX_Hip_comm comm, int *elem)
{
    unsigned kind = ((unsigned) op & 0xc0000000u) >> 30, mpikind = ((unsigned) op & 0x3c000000u) >> 26;
    int opidx = op & 0xf, rc;
    if (!comm) {
        MPIR_Err_set_detail("%s: null communicator", fc);
        return MPI_ERR_ARG;
    }
    if (count < 0) {
        MPIR_Err_set_detail("%s: negative count", fc);
        return MPI_ERR_COUNT;
    }
    if (op == MPI_OP_NULL || op == MPI_NO_OP || op == MPI_REPLACE || kind != 1 || mpikind != 6 ||
        opidx < 1 || opidx > 12) {
        MPIR_Err_set_detail("%s: builtin reduction MPI_Op required", fc);
        return MPI_ERR_OP;
    }
    if ((rc = MPIR_Op_check_dtype_table[opidx] (dt)) != MPI_SUCCESS)
        return rc;
    *elem = MPIR_Op_resolve_elem(opidx, dt);
    if (!*elem) {
        MPIR_Err_set_detail("MPI_Op operation not defined for this datatype");
        return MPI_ERR_OP;
    }
    if (count > 0 && sendbuf == recvbuf) {
        MPIR_Err_set_detail("%s: Buffers must not be aliased", fc);
        return MPI_ERR_BUFFER;
    }
    return MPI_SUCCESS;
}

static int want_rccl(struct MPIX_Hip_comm_s *c, int algorithm, int elem, int opidx, ncclDataType_t * t,
                     ncclRedOp_t * o)
{
    const char *v;
    if (c->kind != COMM_RCCL || algorithm == MPIX_HIP_ALG_REFERENCE_ORDER)
        return 0;
    if (algorithm == MPIX_HIP_ALG_AUTO && (v = getenv("MPIR_CVAR_DEVICE_COLL_ALGORITHM")) &&
        !strcmp(v, "reference"))
        return 0;
    switch (elem) {
    case MPIR_HIP_I8: *t = ncclInt8; break;
    case MPIR_HIP_U8: *t = ncclUint8; break;
    case MPIR_HIP_I32: *t = ncclInt32; break;
    case MPIR_HIP_U32: *t = ncclUint32; break;
    case MPIR_HIP_I64: *t = ncclInt64; break;
    case MPIR_HIP_U64: *t = ncclUint64; break;
    case MPIR_HIP_F16: *t = ncclFloat16; break;
    case MPIR_HIP_F32: *t = ncclFloat32; break;
    case MPIR_HIP_F64: *t = ncclFloat64; break;
    default: return 0;
    }
    switch (opidx) {
    case MPIR_HIP_OP_SUM: *o = ncclSum; break;
    case MPIR_HIP_OP_PROD: *o = ncclProd; break;
    case MPIR_HIP_OP_MAX: *o = ncclMax; break;
    case MPIR_HIP_OP_MIN: *o = ncclMin; break;
    default: return 0;
    }
    return 1;
}

#define HIPTRY(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
        MPIR_Err_set_detail("%s: %s", #x, hipGetErrorString(e_)); rc = MPI_ERR_OTHER; goto done; } } while (0)
#define TRY(x) do { if ((rc = (x)) != MPI_SUCCESS) goto done; } while (0)

/* The reduce-scatter phase of reduce_intra_reduce_scatter_gather.c on `work`
 * (count elements, this rank's contribution): the non-power-of-two pre-fold
 * (:138-170: odd r < 2*rem sends everything to r-1, which computes x_r (+) x_{r+1}),
 * then the recursive halving (:186-249) as ONE all-to-all of blocks and ONE
 * fused tree combine: newrank n owns block bitrev(n), reduced as
 * ((y0+y1)+(y2+y3))+... with y_j = the block from newrank n ^ j.
 * `scr` holds rsg_scratch_bytes(): (pof2-1) slots of stage_stride(cnts[0]
 * elements), then `count` elements for the pre-fold partner's vector.
 * Returns this rank's newrank in *newrank (-1: excluded by the pre-fold). */

static size_t rsg_scratch_bytes(int pof2, const long *cnts, size_t esz, size_t bytes)
{
    return (size_t) (pof2 > 1 ? pof2 - 1 : 1) * stage_stride((size_t) cnts[0] * esz) + bytes + 256;
}

static int rsg_phase(struct MPIX_Hip_comm_s *c, char *work, long count, size_t esz, int opidx, int elem,
                     hipStream_t s, const char *fc, char *scr, const long *cnts, const long *disps, int odd_keeps,
                     int *newrank, int *nchunk, size_t *chunk)
{
    int p = c->size, pof2 = pof2_of(p), rem = p - pof2, bits = 0, nsend = 0, nrecv = 0, rc, i;
    size_t bytes = (size_t) count * esz, blk = stage_stride((size_t) cnts[0] * esz);
    xfer_t sends[MAX_XFER], recvs[MAX_XFER];
    while ((1 << bits) < pof2)
        bits++;
    /* pre-fold; every rank takes part in the transfer group (empty for ranks >= 2*rem).
     * The keeper folds its partner's vector in as the second operand. */
    if (rem > 0 && c->rank >= 2 * rem)
        if ((rc = group_exchange(c, NULL, 0, NULL, 0, s)) != MPI_SUCCESS)
            return rc;
    if (c->rank < 2 * rem) {
        const int keeper = (c->rank % 2) == (odd_keeps ? 1 : 0);
        if (!keeper) {
            xfer_t x = { work, bytes, odd_keeps ? c->rank + 1 : c->rank - 1 };
            if ((rc = group_exchange(c, &x, 1, NULL, 0, s)) != MPI_SUCCESS)
                return rc;
            *newrank = -1;
        } else {
            char *tmp = scr + (size_t) (pof2 > 1 ? pof2 - 1 : 1) * blk;
            xfer_t x = { tmp, bytes, odd_keeps ? c->rank - 1 : c->rank + 1 };
            if ((rc = group_exchange(c, NULL, 0, &x, 1, s)) != MPI_SUCCESS)
                return rc;
            if ((rc = fold_step(tmp, work, count, opidx, elem, s, fc)) != MPI_SUCCESS)
                return rc;
            *newrank = c->rank / 2;
        }
    } else
        *newrank = c->rank - rem;

    /* all-to-all of blocks: the owner receives y_j into scratch slot j-1;
     * chunked, with the tree folded chunk by chunk behind it, when the blocks
     * are large (pipe_chunks: every rank derives the same chunk count from
     * the largest block, cnts[0]) */
    *nchunk = pof2 > 1 ? pipe_chunks((size_t) cnts[0] * esz, chunk) : 1;
    if (*nchunk > 1 && (rc = pipe_init(c)) != MPI_SUCCESS)
        return rc;
    if (*newrank >= 0 && pof2 > 1) {
        int n = *newrank, mb = bitrev(n, bits), m;
        const void *ys[64];
        for (m = 0; m < pof2; m++) {
            int real, b;
            if (m == n)
                continue;
            real = real_of(m, rem, odd_keeps);
            b = bitrev(m, bits);
            sends[nsend].buf = work + disps[b] * esz;
            sends[nsend].bytes = (size_t) cnts[b] * esz;
            sends[nsend++].peer = real;
            recvs[nrecv].buf = scr + (size_t) ((n ^ m) - 1) * blk;
            recvs[nrecv].bytes = (size_t) cnts[mb] * esz;
            recvs[nrecv++].peer = real;
        }
        ys[0] = work + disps[mb] * esz;
        for (i = 1; i < pof2; i++)
            ys[i] = scr + (size_t) (i - 1) * blk;
        if (*nchunk > 1) {
            fold_ctx_t f = { ys, pof2, MPIR_HIP_ORDER_TREE, opidx, elem, work + disps[mb] * esz, esz, fc };
            return exchange_fold_pipelined(c, sends, nsend, recvs, nrecv, *nchunk, *chunk, (size_t) cnts[mb] * esz,
                                           s, chunk_fold, &f);
        }
        if ((rc = group_exchange(c, sends, nsend, recvs, nrecv, s)) != MPI_SUCCESS)
            return rc;
        if (cnts[mb] && (rc = fold_tree(ys, pof2, work + disps[mb] * esz, cnts[mb], opidx, elem, s, fc)))
            return rc;
    } else if (pof2 > 1) {
        /* excluded rank: matches the group calls of the participants (no transfers) */
        if (*nchunk > 1)
            return exchange_fold_pipelined(c, NULL, 0, NULL, 0, *nchunk, *chunk, 0, s, chunk_fold, NULL);
        if ((rc = group_exchange(c, NULL, 0, NULL, 0, s)) != MPI_SUCCESS)
            return rc;
    }
    return MPI_SUCCESS;
}

/* ------------------------------------------------------------ Allreduce */
int MPIX_Allreduce_hip(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
                       MPIX_Hip_comm comm, int algorithm, void *hip_stream)
{
    static const char *fc = "MPIX_Allreduce_hip";
    struct MPIX_Hip_comm_s *c = comm;
    int elem = 0, opidx = op & 0xf, rc, p, pof2, rem, newrank = -1, bits, i, flat, odd_keeps, nchunk = 1, k;
    size_t esz, bytes, chunk = 0;
    hipStream_t s;
    ncclDataType_t nt;
    ncclRedOp_t no;
    long cnts[64] = {0}, disps[64] = {0};
    xfer_t sends[MAX_XFER], recvs[MAX_XFER];
    int nsend = 0, nrecv = 0, cur = 0;
    char *scr = NULL;

    rc = coll_check(fc, sendbuf, recvbuf, count, datatype, op, comm, &elem);
    if (rc)
        return MPIR_Err_return(fc, rc);
    if (count == 0)
        return MPI_SUCCESS;
    if (hipGetDevice(&cur) == hipSuccess && cur != c->device)
        (void) hipSetDevice(c->device);
    s = hip_stream ? (hipStream_t) hip_stream : c->stream;
    esz = MPIR_Hip_elem_size(elem);
    bytes = (size_t) count * esz;
    p = c->size;

    if (want_rccl(c, algorithm, elem, opidx, &nt, &no)) {
        ncclResult_t r = rccl.AllReduce(sendbuf == MPI_IN_PLACE ? recvbuf : sendbuf, recvbuf, (size_t) count,
                                        nt, no, c->nccl, s);
        if (r != ncclSuccess) {
            MPIR_Err_set_detail("ncclAllReduce: %s", rccl.GetErrorString ? rccl.GetErrorString(r) : "?");
            rc = MPI_ERR_OTHER;
        }
        goto done_sync;
    }

    /* ---- reference order: MPIR_Allreduce_intra_auto (allreduce.c:145-217).  On one
     * node the SMP branch runs (allreduce_intra_smp.c: MPIR_Reduce with
     * MPIR_Reduce_intra_auto's choice, then MPIR_Bcast); with the SMP CVARs off
     * (or a comm with one rank per node) the flat branch runs */
    pof2 = pof2_of(p);
    if (p == 1) {
        if (sendbuf != MPI_IN_PLACE)
            HIPTRY(hipMemcpyAsync(recvbuf, sendbuf, bytes, hipMemcpyDeviceToDevice, s));
        goto done_sync;
    }
    flat = allreduce_flat_choice(bytes, count, pof2);
    if (flat == FLAT_RECURSIVE_DOUBLING) {
        TRY(allreduce_recursive_doubling(c, sendbuf, recvbuf, count, esz, opidx, elem, s, fc));
        goto done_sync;
    }
    odd_keeps = flat == FLAT_RABENSEIFNER;
    if (!flat && (bytes <= REDUCE_SHORT_MSG_SIZE || count < pof2)) {
        TRY(allreduce_short(c, sendbuf, recvbuf, count, esz, opidx, elem, s, fc));
        goto done_sync;
    }
    /* long: the reduce-scatter of reduce_intra_reduce_scatter_gather.c (SMP) or
     * allreduce_intra_reduce_scatter_allgather.c (flat, Rabenseifner) on recvbuf */
    if (sendbuf != MPI_IN_PLACE)
        HIPTRY(hipMemcpyAsync(recvbuf, sendbuf, bytes, hipMemcpyDeviceToDevice, s));
    rem = p - pof2;
    bits = 0;
    while ((1 << bits) < pof2)
        bits++;
    cnts_disps(count, pof2, cnts, disps);
    if (comm_scratch(c, rsg_scratch_bytes(pof2, cnts, esz, bytes), &scr)) {
        MPIR_Err_set_detail("%s: scratch allocation failed", fc);
        rc = MPI_ERR_NO_MEM;
        goto done;
    }
    TRY(rsg_phase(c, recvbuf, count, esz, opidx, elem, s, fc, scr, cnts, disps, odd_keeps, &newrank, &nchunk, &chunk));

    /* allgather of the reduced blocks to every rank (the gather + MPIR_Bcast of
     * allreduce_intra_smp.c move data only) */
    nsend = nrecv = 0;
    if (newrank >= 0) {
        int mb = bitrev(newrank, bits), q;
        for (q = 0; q < p; q++) {
            if (q == c->rank)
                continue;
            sends[nsend].buf = (char *) recvbuf + disps[mb] * esz;
            sends[nsend].bytes = (size_t) cnts[mb] * esz;
            sends[nsend++].peer = q;
        }
    }
    for (i = 0; i < pof2; i++) {
        int real = real_of(i, rem, odd_keeps), b = bitrev(i, bits);
        if (real == c->rank)
            continue;
        recvs[nrecv].buf = (char *) recvbuf + disps[b] * esz;
        recvs[nrecv].bytes = (size_t) cnts[b] * esz;
        recvs[nrecv++].peer = real;
    }
    if (nchunk > 1) {
        /* chunk k of the owners' blocks leaves once its fold is done */
        xfer_t sk[MAX_XFER], rk[MAX_XFER];
        for (k = 0; k < nchunk; k++) {
            HIPTRY(hipStreamWaitEvent(s, c->fev[k], 0));
            chunk_of(sends, nsend, k, chunk, sk);
            chunk_of(recvs, nrecv, k, chunk, rk);
            TRY(group_exchange(c, sk, nsend, rk, nrecv, s));
        }
    } else
        TRY(group_exchange(c, sends, nsend, recvs, nrecv, s));

  done_sync:
    if (rc == MPI_SUCCESS && !hip_stream)
        HIPTRY(hipStreamSynchronize(s));
  done:
    if (cur != c->device)
        (void) hipSetDevice(cur);
    return rc ? MPIR_Err_return(fc, rc) : MPI_SUCCESS;
}

/* ------------------------------------------------------------ Reduce
 * MPI_Reduce on one node: MPIR_Reduce_intra_smp (reduce_intra_smp.c) reduces
 * to the root over node_comm with MPIR_Reduce_intra_auto (reduce.c:170-225):
 *   count*size <= 2048 or count < pof2: binomial tree rooted at `root`
 *       (reduce_intra_binomial.c:93-140, commutative: relrank = rank - root);
 *       here a gather to the root, which folds the relranks in binomial order;
 *   else reduce_intra_reduce_scatter_gather.c: the reduce-scatter phase of the
 *       Allreduce (block values do not depend on the root), then the owners'
 *       blocks are gathered to the root. */
int MPIX_Reduce_hip(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype, MPI_Op op, int root,
                    MPIX_Hip_comm comm, int algorithm, void *hip_stream)
{
    static const char *fc = "MPIX_Reduce_hip";
    struct MPIX_Hip_comm_s *c = comm;
    int elem = 0, opidx = op & 0xf, rc, p, pof2, rem, newrank = -1, bits, i, isroot, cur = 0, nchunk = 1;
    size_t esz, bytes, slot, chunk = 0;
    hipStream_t s;
    ncclDataType_t nt;
    ncclRedOp_t no;
    long cnts[64] = {0}, disps[64] = {0};
    xfer_t sends[MAX_XFER], recvs[MAX_XFER];
    int nsend = 0, nrecv = 0;
    char *scr = NULL, *work;
    const void *own;

    if (comm && (root < 0 || root >= comm->size)) {
        MPIR_Err_set_detail("%s: Invalid root (value given was %d)", fc, root);
        return MPIR_Err_return(fc, MPI_ERR_ROOT);
    }
    isroot = comm && comm->rank == root;
    if (comm && !isroot && sendbuf == MPI_IN_PLACE && count > 0) {
        MPIR_Err_set_detail("%s: MPI_IN_PLACE is only valid at the root", fc);
        return MPIR_Err_return(fc, MPI_ERR_BUFFER);
    }
    /* recvbuf is significant at the root only (the alias check with it too) */
    rc = coll_check(fc, sendbuf, isroot ? recvbuf : NULL, count, datatype, op, comm, &elem);
    if (rc)
        return MPIR_Err_return(fc, rc);
    if (count == 0)
        return MPI_SUCCESS;
    if (hipGetDevice(&cur) == hipSuccess && cur != c->device)
        (void) hipSetDevice(c->device);
    s = hip_stream ? (hipStream_t) hip_stream : c->stream;
    esz = MPIR_Hip_elem_size(elem);
    bytes = (size_t) count * esz;
    p = c->size;
    own = sendbuf == MPI_IN_PLACE ? recvbuf : sendbuf;

    if (want_rccl(c, algorithm, elem, opidx, &nt, &no)) {
        ncclResult_t r = rccl.Reduce(own, isroot ? recvbuf : NULL, (size_t) count, nt, no, root, c->nccl, s);
        if (r != ncclSuccess) {
            MPIR_Err_set_detail("ncclReduce: %s", rccl.GetErrorString ? rccl.GetErrorString(r) : "?");
            rc = MPI_ERR_OTHER;
        }
        goto done_sync;
    }

    pof2 = pof2_of(p);
    if (p == 1) {
        if (sendbuf != MPI_IN_PLACE)
            HIPTRY(hipMemcpyAsync(recvbuf, sendbuf, bytes, hipMemcpyDeviceToDevice, s));
        goto done_sync;
    }
    if (bytes <= REDUCE_SHORT_MSG_SIZE || count < pof2) {
        /* binomial: slot rel holds x_{(rel + root) % p}; the tree folds relranks */
        int mask;
        slot = stage_stride(bytes);
        if (!isroot) {
            xfer_t x = { (void *) own, bytes, root };
            TRY(group_exchange(c, &x, 1, NULL, 0, s));
            goto done_sync;
        }
        if (comm_scratch(c, (size_t) p * slot, &scr)) {
            MPIR_Err_set_detail("%s: scratch allocation failed", fc);
            rc = MPI_ERR_NO_MEM;
            goto done;
        }
        HIPTRY(hipMemcpyAsync(scr, own, bytes, hipMemcpyDeviceToDevice, s));
        for (i = 1; i < p; i++) {
            recvs[nrecv].buf = scr + (size_t) i * slot;
            recvs[nrecv].bytes = bytes;
            recvs[nrecv++].peer = (i + root) % p;
        }
        TRY(group_exchange(c, NULL, 0, recvs, nrecv, s));
        if ((p & (p - 1)) == 0) {
            const void *ys[64];
            for (i = 0; i < p; i++)
                ys[i] = scr + (size_t) i * slot;
            TRY(fold_tree(ys, p, recvbuf, count, opidx, elem, s, fc));
            goto done_sync;
        }
        for (mask = 1; mask < p; mask <<= 1)
            for (i = 0; i + mask < p; i += 2 * mask)
                TRY(fold_step(scr + (size_t) (i + mask) * slot, scr + (size_t) i * slot, count, opidx, elem, s, fc));
        HIPTRY(hipMemcpyAsync(recvbuf, scr, bytes, hipMemcpyDeviceToDevice, s));
        goto done_sync;
    }

    /* long: reduce-scatter on `work` (recvbuf at the root, scratch elsewhere) */
    rem = p - pof2;
    bits = 0;
    while ((1 << bits) < pof2)
        bits++;
    cnts_disps(count, pof2, cnts, disps);
    slot = (rsg_scratch_bytes(pof2, cnts, esz, bytes) + 255) & ~(size_t) 255;
    if (comm_scratch(c, slot + (isroot ? 0 : bytes), &scr)) {
        MPIR_Err_set_detail("%s: scratch allocation failed", fc);
        rc = MPI_ERR_NO_MEM;
        goto done;
    }
    work = isroot ? (char *) recvbuf : scr + slot;
    if (work != own)
        HIPTRY(hipMemcpyAsync(work, own, bytes, hipMemcpyDeviceToDevice, s));
    TRY(rsg_phase(c, work, count, esz, opidx, elem, s, fc, scr, cnts, disps, 0, &newrank, &nchunk, &chunk));
    if (nchunk > 1)
        HIPTRY(hipStreamWaitEvent(s, c->fev[nchunk - 1], 0));       /* every fold done */

    /* gather of the owners' blocks to the root (reduce_intra_reduce_scatter_gather.c:256-410) */
    if (newrank >= 0 && !isroot) {
        int mb = bitrev(newrank, bits);
        sends[nsend].buf = work + disps[mb] * esz;
        sends[nsend].bytes = (size_t) cnts[mb] * esz;
        sends[nsend++].peer = root;
    }
    if (isroot) {
        for (i = 0; i < pof2; i++) {
            int real = real_of(i, rem, 0), b = bitrev(i, bits);
            if (real == c->rank)
                continue;
            recvs[nrecv].buf = (char *) recvbuf + disps[b] * esz;
            recvs[nrecv].bytes = (size_t) cnts[b] * esz;
            recvs[nrecv++].peer = real;
        }
    }
    TRY(group_exchange(c, sends, nsend, recvs, nrecv, s));

  done_sync:
    if (rc == MPI_SUCCESS && !hip_stream)
        HIPTRY(hipStreamSynchronize(s));
  done:
    if (cur != c->device)
        (void) hipSetDevice(cur);
    return rc ? MPIR_Err_return(fc, rc) : MPI_SUCCESS;
}

/* ------------------------------------------------------------ Reduce_scatter(_block)
 * One implementation for both: counts[q] elements of the result go to rank q.
 *   RCCL:  ncclReduceScatter (regular counts only).
 *   reference order (MPIR_Reduce_scatter(_block)_intra_auto, builtin ops are
 *   commutative): recursive halving below 524288 total bytes, else pairwise
 *   (reduce_scatter_block_intra_pairwise.c:97-134 /
 *   reduce_scatter_intra_pairwise.c): block r = ((x_r + x_{r-1}) + x_{r-2}) + ...
 *   as one all-to-all + one CHAIN combine. */
static int reduce_scatter_common(const char *fc, const void *sendbuf, void *recvbuf, const int *counts,
                                 MPI_Datatype datatype, MPI_Op op, MPIX_Hip_comm comm, int algorithm,
                                 void *hip_stream)
{
    struct MPIX_Hip_comm_s *c = comm;
    int elem = 0, opidx = op & 0xf, rc, p, i, cur = 0, regular = 1;
    long cnts[64] = {0}, disps[64] = {0}, total = 0;
    size_t esz, nb, slot;
    hipStream_t s;
    ncclDataType_t nt;
    ncclRedOp_t no;
    xfer_t sends[MAX_XFER], recvs[MAX_XFER];
    const void *ys[64];
    const char *src;
    char *scr = NULL;

    if (!comm) {
        MPIR_Err_set_detail("%s: null communicator", fc);
        return MPIR_Err_return(fc, MPI_ERR_ARG);
    }
    p = c->size;
    for (i = 0; i < p; i++) {
        if (counts[i] < 0) {
            MPIR_Err_set_detail("%s: negative count", fc);
            return MPIR_Err_return(fc, MPI_ERR_COUNT);
        }
        cnts[i] = counts[i];
        disps[i] = total;
        total += counts[i];
        regular &= counts[i] == counts[0];
    }
    /* op / type validation; the alias check applies when any data moves */
    rc = coll_check(fc, sendbuf, recvbuf, total > 0, datatype, op, comm, &elem);
    if (rc)
        return MPIR_Err_return(fc, rc);
    if (total == 0)
        return MPI_SUCCESS;
    if (hipGetDevice(&cur) == hipSuccess && cur != c->device)
        (void) hipSetDevice(c->device);
    s = hip_stream ? (hipStream_t) hip_stream : c->stream;
    esz = MPIR_Hip_elem_size(elem);
    nb = (size_t) cnts[c->rank] * esz;
    src = sendbuf == MPI_IN_PLACE ? (const char *) recvbuf : (const char *) sendbuf;

    if (regular && want_rccl(c, algorithm, elem, opidx, &nt, &no)) {
        ncclResult_t r;
        /* NCCL's in-place form is recvbuff == sendbuff + rank * recvcount */
        void *dst = sendbuf == MPI_IN_PLACE ? (char *) recvbuf + (size_t) c->rank * nb : recvbuf;
        r = rccl.ReduceScatter(src, dst, (size_t) cnts[0], nt, no, c->nccl, s);
        if (r != ncclSuccess) {
            MPIR_Err_set_detail("ncclReduceScatter: %s", rccl.GetErrorString ? rccl.GetErrorString(r) : "?");
            rc = MPI_ERR_OTHER;
            goto done;
        }
        if (sendbuf == MPI_IN_PLACE && c->rank)
            HIPTRY(hipMemcpyAsync(recvbuf, dst, nb, hipMemcpyDeviceToDevice, s));
        goto done_sync;
    }

    if (p > 1 && (size_t) total * esz < RSB_COMMUTATIVE_LONG_MSG_SIZE) {
        TRY(reduce_scatter_short(c, src, recvbuf, cnts, disps, esz, opidx, elem, s, fc));
        goto done_sync;
    }
    /* long: pairwise.  y_i = block r from rank r - i into scratch slot i-1; in
     * place, the own block is staged too when it overlaps the output. */
    slot = stage_stride(nb);
    if (comm_scratch(c, (size_t) p * slot + 256, &scr)) {
        MPIR_Err_set_detail("%s: scratch allocation failed", fc);
        rc = MPI_ERR_NO_MEM;
        goto done;
    }
    ys[0] = src + (size_t) disps[c->rank] * esz;
    if (sendbuf == MPI_IN_PLACE && disps[c->rank] > 0 && disps[c->rank] < cnts[c->rank]) {
        HIPTRY(hipMemcpyAsync(scr + (size_t) (p - 1) * slot, ys[0], nb, hipMemcpyDeviceToDevice, s));
        ys[0] = scr + (size_t) (p - 1) * slot;
    }
    for (i = 1; i < p; i++) {
        int dst = (c->rank + i) % p, from = (c->rank - i + p) % p;
        sends[i - 1].buf = (void *) (src + (size_t) disps[dst] * esz);
        sends[i - 1].bytes = (size_t) cnts[dst] * esz;
        sends[i - 1].peer = dst;
        recvs[i - 1].buf = scr + (size_t) (i - 1) * slot;
        recvs[i - 1].bytes = nb;
        recvs[i - 1].peer = from;
        ys[i] = scr + (size_t) (i - 1) * slot;
    }
    {
        /* large blocks: the exchange in chunks, chunk k's chain folded while
         * k+1 moves (pipe_chunks; every rank takes the chunk count from the
         * largest block) */
        size_t maxb = 0, chunk = 0;
        int nchunk;
        for (i = 0; i < p; i++)
            if ((size_t) cnts[i] * esz > maxb)
                maxb = (size_t) cnts[i] * esz;
        nchunk = p > 1 ? pipe_chunks(maxb, &chunk) : 1;
        if (nchunk > 1) {
            fold_ctx_t f = { ys, p, MPIR_HIP_ORDER_CHAIN, opidx, elem, recvbuf, esz, fc };
            TRY(pipe_init(c));
            TRY(exchange_fold_pipelined(c, sends, p - 1, recvs, p - 1, nchunk, chunk, nb, s, chunk_fold, &f));
            HIPTRY(hipStreamWaitEvent(s, c->fev[nchunk - 1], 0));
            goto done_sync;
        }
    }
    if (p > 1)
        TRY(group_exchange(c, sends, p - 1, recvs, p - 1, s));
    if (nb) {
        rc = MPIR_Hip_combine(ys, p, recvbuf, (uint64_t) cnts[c->rank], opidx, elem, MPIR_HIP_ORDER_CHAIN, s, 0);
        if (rc) {
            MPIR_Op_report_hip_error(fc, rc);
            rc = MPI_ERR_OTHER;
            goto done;
        }
    }

  done_sync:
    if (rc == MPI_SUCCESS && !hip_stream)
        HIPTRY(hipStreamSynchronize(s));
  done:
    if (cur != c->device)
        (void) hipSetDevice(cur);
    return rc ? MPIR_Err_return(fc, rc) : MPI_SUCCESS;
}

int MPIX_Reduce_scatter_block_hip(const void *sendbuf, void *recvbuf, int recvcount, MPI_Datatype datatype,
                                  MPI_Op op, MPIX_Hip_comm comm, int algorithm, void *hip_stream)
{
    int counts[64], i;
    if (!comm || recvcount < 0)
        return reduce_scatter_common("MPIX_Reduce_scatter_block_hip", sendbuf, recvbuf,
                                     (int[64]) { recvcount }, datatype, op, comm, algorithm, hip_stream);
    for (i = 0; i < comm->size; i++)
        counts[i] = recvcount;
    return reduce_scatter_common("MPIX_Reduce_scatter_block_hip", sendbuf, recvbuf, counts, datatype, op, comm,
                                 algorithm, hip_stream);
}

int MPIX_Reduce_scatter_hip(const void *sendbuf, void *recvbuf, const int recvcounts[], MPI_Datatype datatype,
                            MPI_Op op, MPIX_Hip_comm comm, int algorithm, void *hip_stream)
{
    if (!recvcounts) {
        MPIR_Err_set_detail("MPIX_Reduce_scatter_hip: recvcounts is NULL");
        return MPIR_Err_return("MPIX_Reduce_scatter_hip", MPI_ERR_ARG);
    }
    return reduce_scatter_common("MPIX_Reduce_scatter_hip", sendbuf, recvbuf, recvcounts, datatype, op, comm,
                                 algorithm, hip_stream);
}

/* ------------------------------------------------------------ Scan / Exscan
 * On one node MPI_Scan is MPIR_Scan_intra_smp over node_comm, i.e. the
 * recursive doubling of scan_intra_recursive_doubling.c:94-147; MPI_Exscan is
 * exscan_intra_recursive_doubling.c:105-170.  At mask m rank r receives the
 * partial scan of r ^ m and, when r > r ^ m, folds it into recvbuf as the
 * second operand.  That partial scan is the full tree T(d) over
 * z_j = x_{d ^ j}, j < m, d = r ^ m (each rank folds its partner's partial
 * scan in second), so rank r's result is the chain
 *     x_r (+) T(r ^ m_1) (+) T(r ^ m_2) ...      (m_i: set bits of r, increasing)
 * and the exscan is the same chain without x_r (tests/test_schedule_small_cpu.py
 * pins the plan against the step-by-step schedules).  MI355X form: every rank
 * sends its vector to all higher ranks in ONE exchange (all xGMI links at
 * once instead of log2(p) dependent rounds), then folds the trees and the
 * chain on the device.  RCCL has no scan; MPIX_HIP_ALG_RCCL runs this too. */
static int scan_common(const char *fc, const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype,
                       MPI_Op op, MPIX_Hip_comm comm, void *hip_stream, int exclusive)
{
    struct MPIX_Hip_comm_s *c = comm;
    int elem = 0, opidx = op & 0xf, rc, p, r, q, m, nx = 0, nr = 0, nparts = 0, cur = 0;
    size_t esz, bytes, slot;
    hipStream_t s;
    xfer_t sends[MAX_XFER], recvs[MAX_XFER];
    const void *chain[64], *ys[64];
    const void *own;
    char *scr = NULL;

    if (!comm) {
        MPIR_Err_set_detail("%s: null communicator", fc);
        return MPIR_Err_return(fc, MPI_ERR_ARG);
    }
    /* the exscan's recvbuf is not significant at rank 0 */
    rc = coll_check(fc, sendbuf, (exclusive && comm->rank == 0 && sendbuf != MPI_IN_PLACE) ? NULL : recvbuf, count,
                    datatype, op, comm, &elem);
    if (rc)
        return MPIR_Err_return(fc, rc);
    if (count == 0)
        return MPI_SUCCESS;
    if (hipGetDevice(&cur) == hipSuccess && cur != c->device)
        (void) hipSetDevice(c->device);
    s = hip_stream ? (hipStream_t) hip_stream : c->stream;
    esz = MPIR_Hip_elem_size(elem);
    bytes = (size_t) count * esz;
    slot = stage_stride(bytes);
    p = c->size;
    r = c->rank;
    own = sendbuf == MPI_IN_PLACE ? recvbuf : sendbuf;
    for (m = 1; m <= r; m <<= 1)
        nparts += (r & m) != 0;
    if (p > 1 && comm_scratch(c, (size_t) (r + nparts + 1) * slot, &scr)) {
        MPIR_Err_set_detail("%s: scratch allocation failed", fc);
        rc = MPI_ERR_NO_MEM;
        goto done;
    }
    /* every rank's vector to all higher ranks; x_q lands in slot q */
    for (q = 0; q < p; q++) {
        if (q > r) {
            sends[nx].buf = (void *) own;
            sends[nx].bytes = bytes;
            sends[nx++].peer = q;
        } else if (q < r) {
            recvs[nr].buf = scr + (size_t) q * slot;
            recvs[nr].bytes = bytes;
            recvs[nr++].peer = q;
        }
    }
    if (p > 1)
        TRY(group_exchange(c, sends, nx, recvs, nr, s));
    nx = 0;
    if (!exclusive)
        chain[nx++] = own;
    for (m = 1, q = 0; m <= r; m <<= 1) {
        int d, j;
        if (!(r & m))
            continue;
        d = r ^ m;
        if (m == 1) {
            chain[nx++] = scr + (size_t) d * slot;
        } else {
            char *t = scr + (size_t) (r + q++) * slot;
            for (j = 0; j < m; j++)
                ys[j] = scr + (size_t) (d ^ j) * slot;
            TRY(fold_tree(ys, m, t, count, opidx, elem, s, fc));
            chain[nx++] = t;
        }
    }
    if (nx > 0) {
        rc = MPIR_Hip_combine(chain, nx, recvbuf, (uint64_t) count, opidx, elem, MPIR_HIP_ORDER_CHAIN, s, 0);
        if (rc) {
            MPIR_Op_report_hip_error(fc, rc);
            rc = MPI_ERR_OTHER;
            goto done;
        }
    }
    if (!hip_stream)
        HIPTRY(hipStreamSynchronize(s));
  done:
    if (cur != c->device)
        (void) hipSetDevice(cur);
    return rc ? MPIR_Err_return(fc, rc) : MPI_SUCCESS;
}

int MPIX_Scan_hip(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
                  MPIX_Hip_comm comm, int algorithm, void *hip_stream)
{
    (void) algorithm;
    return scan_common("MPIX_Scan_hip", sendbuf, recvbuf, count, datatype, op, comm, hip_stream, 0);
}

int MPIX_Exscan_hip(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
                    MPIX_Hip_comm comm, int algorithm, void *hip_stream)
{
    (void) algorithm;
    return scan_common("MPIX_Exscan_hip", sendbuf, recvbuf, count, datatype, op, comm, hip_stream, 1);
}

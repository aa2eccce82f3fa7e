/*
 * pip_world.c -- the MPI runtime subset of include/mpi_pip.h (config 1 plumbing,
 * SURVEY.md §8f row 3).
 *
 * Ranks are the processes bin/mpiexec forks; they attach the POSIX shm
 * segment named by MPIR_PIP_SHM.  Each rank owns one mailbox slot plus a
 * PIP_CHUNK-byte data area in that segment; a message is a sequence of
 * chunks, each handed over with a release-store of dst + 1 into the slot's
 * `owner` word and returned with a release-store of 0 by the receiver.  Because every rank
 * issues the same collectives in the same order and pairs exchange FIFO, no
 * tags are needed.  A rank started without mpiexec is a singleton (size 1).
 *
 * The collective schedules are the reference's, step for step, so results
 * are bit-identical to MPICH's for the same inputs:
 *   Bcast   binomial               bcast_intra_binomial.c:68-163
 *   Reduce  MPIR_Reduce_intra_auto  reduce.c:170-225 -- on one node the SMP
 *           branch (:190-205) reduces over node_comm == this communicator, so
 *           the choice is: > MPIR_CVAR_REDUCE_SHORT_MSG_SIZE (2048) bytes,
 *           builtin op and count >= pof2 -> reduce-scatter + gather
 *           (reduce_intra_reduce_scatter_gather.c:40-400), else binomial
 *           (reduce_intra_binomial.c:100-160).
 *   Barrier dissemination           barrier_intra_dissemination.c:25-60
 * Every combine step is MPIR_Reduce_local(tmp, acc, ...) -- the HIP path.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "mpi_pip.h"
#include "mpir_op_types.h"
#include "pip_shm.h"

static struct {
    int initialized, finalized;
    int rank, size;
    pip_shm_t *shm;
    size_t shm_bytes;
} W;

static int err(const char *fc, int cls, const char *fmt, const char *arg)
{
    MPIR_Err_set_detail(fmt, arg);
    return MPIR_Err_return(fc, cls);
}

static inline void relax(void)
{
    __builtin_ia32_pause();
}

/* ------------------------------------------------------------ transport */
static char *slot_data(int r)
{
    return (char *) W.shm + PIP_DATA_OFFSET + (size_t) r * PIP_CHUNK;
}

/* Send `sbytes` to `dst` and receive up to `rbytes` from `src` concurrently
 * (either side may be absent: dst / src < 0).  Progresses both directions
 * chunk by chunk so a pairwise exchange of long messages cannot deadlock.
 * Every chunk carries the message's total length, so the receiver takes
 * exactly the message that was sent whatever it expected: a longer one is
 * drained to its end with the excess dropped, a shorter one ends early.
 * Returns the received message's length (0 with no receive side). */
static size_t sendrecv(const void *sbuf, size_t sbytes, int dst, void *rbuf, size_t rbytes, int src)
{
    pip_slot_t *mine = &W.shm->slot[W.rank];
    pip_slot_t *theirs = src >= 0 ? &W.shm->slot[src] : NULL;
    size_t soff = 0, roff = 0, rtotal = 0;
    int sdone = dst < 0, rdone = src < 0, sfirst = 1;
    while (!sdone || !rdone) {
        int moved = 0;
        if (!sdone && atomic_load_explicit(&mine->owner, memory_order_acquire) == 0) {
            size_t n = sbytes - soff < PIP_CHUNK ? sbytes - soff : PIP_CHUNK;
            if (n)
                memcpy(slot_data(W.rank), (const char *) sbuf + soff, n);
            mine->bytes = (uint32_t) n;
            mine->total = sbytes;
            atomic_store_explicit(&mine->owner, (uint32_t) dst + 1, memory_order_release);
            soff += n;
            sfirst = 0;
            sdone = soff >= sbytes && !sfirst;
            moved = 1;
        }
        if (!rdone && atomic_load_explicit(&theirs->owner, memory_order_acquire) == (uint32_t) W.rank + 1) {
            size_t n = theirs->bytes, keep = n;
            rtotal = (size_t) theirs->total;
            if (roff >= rbytes)
                keep = 0;               /* truncation: past the end of the receive buffer */
            else if (roff + n > rbytes)
                keep = rbytes - roff;
            if (keep)
                memcpy((char *) rbuf + roff, slot_data(src), keep);
            roff += n;
            atomic_store_explicit(&theirs->owner, 0, memory_order_release);
            rdone = roff >= rtotal;
            moved = 1;
        }
        if (!moved)
            relax();
    }
    /* the last outgoing chunk must be consumed before the buffer is reused */
    if (dst >= 0)
        while (atomic_load_explicit(&mine->owner, memory_order_acquire) != 0)
            relax();
    return rtotal;
}

/* A collective's first receive error, kept while the schedule runs on (as
 * MPICH's errflag does, so no peer is left waiting) and returned at its end:
 * a message longer than the receive buffer is MPI_ERR_TRUNCATE (MPIC_Recv,
 * ch3u_request.c:516), any other length mismatch MPI_ERR_OTHER
 * "**collective_size_mismatch" (bcast_intra_binomial.c:116-124). */
static __thread int coll_err;
static __thread char coll_why[160];

static void note_length(size_t got, size_t want)
{
    if (got == want || coll_err)
        return;
    coll_err = got > want ? MPI_ERR_TRUNCATE : MPI_ERR_OTHER;
    snprintf(coll_why, sizeof(coll_why), got > want ?
             "Message truncated; %zu bytes received but buffer size is %zu" :
             "message sizes do not match across processes in the collective routine: "
             "Received %zu but expected %zu", got, want);
}

static void exchange(const void *sbuf, size_t sbytes, int dst, void *rbuf, size_t rbytes, int src)
{
    size_t got = sendrecv(sbuf, sbytes, dst, rbuf, rbytes, src);
    if (src >= 0)
        note_length(got, rbytes);
}

static void send_to(const void *buf, size_t bytes, int dst)
{
    sendrecv(buf, bytes, dst, NULL, 0, -1);
}

static void recv_from(void *buf, size_t bytes, int src)
{
    note_length(sendrecv(NULL, 0, -1, buf, bytes, src), bytes);
}

/* the collective's result: its own error, else the first receive error */
static int coll_finish(const char *fc, int rc)
{
    int e = coll_err;
    coll_err = 0;
    if (rc)
        return rc;
    if (e) {
        MPIR_Err_set_detail("%s", coll_why);
        return MPIR_Err_return(fc, e);
    }
    return MPI_SUCCESS;
}

/* ------------------------------------------------------------ init / finalize */
int MPI_Init(int *argc, char ***argv)
{
    static const char *fc = "MPI_Init";
    const char *er = getenv("MPIR_PIP_RANK"), *es = getenv("MPIR_PIP_SIZE"), *name = getenv("MPIR_PIP_SHM");
    (void) argc;
    (void) argv;
    if (W.initialized)
        return err(fc, MPI_ERR_OTHER, "%s", "MPI_Init called twice");
    W.rank = 0;
    W.size = 1;
    if (er && es && name) {
        int fd;
        struct stat st;
        W.rank = atoi(er);
        W.size = atoi(es);
        if (W.size < 1 || W.size > PIP_MAX_RANKS || W.rank < 0 || W.rank >= W.size)
            return err(fc, MPI_ERR_OTHER, "bad MPIR_PIP_RANK/SIZE (%s)", es);
        fd = shm_open(name, O_RDWR, 0600);
        if (fd < 0)
            return err(fc, MPI_ERR_OTHER, "shm_open(%s) failed", name);
        if (fstat(fd, &st) != 0 || (size_t) st.st_size < PIP_DATA_OFFSET) {
            close(fd);
            return err(fc, MPI_ERR_OTHER, "shm segment %s too small", name);
        }
        W.shm_bytes = (size_t) st.st_size;
        W.shm = mmap(NULL, W.shm_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (W.shm == MAP_FAILED || W.shm->magic != PIP_MAGIC || (int) W.shm->size != W.size) {
            W.shm = NULL;
            return err(fc, MPI_ERR_OTHER, "shm segment %s is not an mpiexec world", name);
        }
    }
    W.initialized = 1;
    return MPI_Barrier(MPI_COMM_WORLD);
}

int MPI_Initialized(int *flag)
{
    *flag = W.initialized;
    return MPI_SUCCESS;
}

int MPI_Finalized(int *flag)
{
    *flag = W.finalized;
    return MPI_SUCCESS;
}

int MPI_Finalize(void)
{
    int rc;
    if (!W.initialized || W.finalized)
        return err("MPI_Finalize", MPI_ERR_OTHER, "%s", "MPI not initialized");
    rc = MPI_Barrier(MPI_COMM_WORLD);
    if (W.shm)
        munmap(W.shm, W.shm_bytes);
    W.shm = NULL;
    W.finalized = 1;
    return rc;
}

int MPI_Abort(MPI_Comm comm, int errorcode)
{
    (void) comm;
    fprintf(stderr, "application called MPI_Abort(MPI_COMM_WORLD, %d) - process %d\n", errorcode, W.rank);
    fflush(stderr);
    _exit(errorcode);
}

/* comm -> (rank, size); MPI_ERR_COMM for anything but WORLD / SELF */
static int comm_geom(const char *fc, MPI_Comm comm, int *rank, int *size)
{
    if (!W.initialized || W.finalized)
        return err(fc, MPI_ERR_OTHER, "%s", "MPI not initialized");
    if (comm == MPI_COMM_WORLD) {
        *rank = W.rank;
        *size = W.size;
    } else if (comm == MPI_COMM_SELF) {
        *rank = 0;
        *size = 1;
    } else {
        return err(fc, MPI_ERR_COMM, "%s", "Invalid communicator");
    }
    return MPI_SUCCESS;
}

int MPI_Comm_size(MPI_Comm comm, int *size)
{
    int r;
    return comm_geom("MPI_Comm_size", comm, &r, size);
}

int MPI_Comm_rank(MPI_Comm comm, int *rank)
{
    int s;
    return comm_geom("MPI_Comm_rank", comm, rank, &s);
}

int MPI_Get_processor_name(char *name, int *resultlen)
{
    if (gethostname(name, MPI_MAX_PROCESSOR_NAME) != 0)
        strcpy(name, "localhost");
    name[MPI_MAX_PROCESSOR_NAME - 1] = 0;
    *resultlen = (int) strlen(name);
    return MPI_SUCCESS;
}

double MPI_Wtime(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double) ts.tv_sec + 1e-9 * (double) ts.tv_nsec;
}

double MPI_Wtick(void)
{
    struct timespec ts;
    clock_getres(CLOCK_MONOTONIC, &ts);
    return (double) ts.tv_sec + 1e-9 * (double) ts.tv_nsec;
}

/* ------------------------------------------------------------ Barrier */
/* dissemination (barrier_intra_dissemination.c:37-55): in round k every rank
 * signals rank + 2^k and waits for rank - 2^k (zero-byte messages) */
int MPI_Barrier(MPI_Comm comm)
{
    int rank, size, mask, rc;
    if ((rc = comm_geom("MPI_Barrier", comm, &rank, &size)))
        return rc;
    if (size == 1)
        return MPI_SUCCESS;
    for (mask = 1; mask < size; mask <<= 1)
        exchange(NULL, 0, (rank + mask) % size, NULL, 0, (rank - mask + size) % size);
    return coll_finish("MPI_Barrier", MPI_SUCCESS);
}

/* ------------------------------------------------------------ helpers */
static size_t type_size(MPI_Datatype dt)
{
    const MPIR_Type_desc *d = MPIR_Type_lookup(dt);
    return d ? MPIR_Hip_elem_size(d->elem) : 0;
}

static int coll_args(const char *fc, MPI_Comm comm, int count, MPI_Datatype dt, int root, int *rank, int *size,
                     size_t *esz)
{
    int rc;
    if ((rc = comm_geom(fc, comm, rank, size)))
        return rc;
    if (count < 0)
        return err(fc, MPI_ERR_COUNT, "%s", "Negative count");
    if (!(*esz = type_size(dt)))
        return err(fc, MPI_ERR_TYPE, "%s", "Invalid datatype");
    if (root < 0 || root >= *size)
        return err(fc, MPI_ERR_ROOT, "%s", "Invalid root");
    return MPI_SUCCESS;
}

/* ------------------------------------------------------------ Bcast */
int MPI_Bcast(void *buffer, int count, MPI_Datatype datatype, int root, MPI_Comm comm)
{
    static const char *fc = "MPI_Bcast";
    int rank, size, rc, mask, rel;
    size_t esz, nbytes;
    if ((rc = coll_args(fc, comm, count, datatype, root, &rank, &size, &esz)))
        return rc;
    nbytes = (size_t) count * esz;
    if (size == 1 || nbytes == 0)
        return MPI_SUCCESS;
    rel = (rank - root + size) % size;
    /* receive from the parent (bcast_intra_binomial.c:95-128) */
    for (mask = 1; mask < size; mask <<= 1) {
        if (rel & mask) {
            recv_from(buffer, nbytes, (rank - mask + size) % size);
            break;
        }
    }
    /* forward to the children, largest subtree first (:142-163) */
    for (mask >>= 1; mask > 0; mask >>= 1)
        if (rel + mask < size)
            send_to(buffer, nbytes, (rank + mask) % size);
    return coll_finish(fc, MPI_SUCCESS);
}

/* ------------------------------------------------------------ Reduce */
static int local_reduce(const char *fc, const void *in, void *inout, int count, MPI_Datatype dt, MPI_Op op)
{
    int rc;
    if (count <= 0)
        return MPI_SUCCESS;
    rc = MPIR_Reduce_local(in, inout, count, dt, op);
    if (rc) {
        char why[256];
        snprintf(why, sizeof(why), "%s", MPIR_Err_last_detail());
        MPIR_Err_set_detail("MPIR_Reduce_local failed in %s: %s", fc, why);
    }
    return rc;
}

/* reduce_intra_binomial.c:100-160 */
static int reduce_binomial(void *acc, void *tmp, int count, size_t esz, MPI_Datatype dt, MPI_Op op, int root,
                           int rank, int size)
{
    const int commute = MPIR_Op_is_commutative(op);
    const size_t nbytes = (size_t) count * esz;
    const int lroot = commute ? root : 0, rel = (rank - lroot + size) % size;
    int mask, rc;
    for (mask = 1; mask < size; mask <<= 1) {
        if ((mask & rel) == 0) {
            int src = rel | mask;
            if (src < size) {
                recv_from(tmp, nbytes, (src + lroot) % size);
                if (commute) {
                    if ((rc = local_reduce("MPI_Reduce", tmp, acc, count, dt, op)))
                        return rc;
                } else {
                    /* the sender is above us: received data is the right operand */
                    if ((rc = local_reduce("MPI_Reduce", acc, tmp, count, dt, op)))
                        return rc;
                    memcpy(acc, tmp, nbytes);
                }
            }
        } else {
            send_to(acc, nbytes, ((rel & ~mask) + lroot) % size);
            break;
        }
    }
    if (!commute && root != 0) {
        if (rank == 0)
            send_to(acc, nbytes, root);
        else if (rank == root)
            recv_from(acc, nbytes, 0);
    }
    return MPI_SUCCESS;
}

/* reduce_intra_reduce_scatter_gather.c:105-400 (builtin, commutative ops) */
static int reduce_scatter_gather(void *acc_, void *tmp_, int count, size_t esz, MPI_Datatype dt, MPI_Op op,
                                 int root, int rank, int size)
{
    char *acc = acc_, *tmp = tmp_;
    int pof2 = 1, rem, newrank, newroot, mask, i, j, rc;
    int cnts[PIP_MAX_RANKS], disps[PIP_MAX_RANKS];
    int send_idx = 0, recv_idx = 0, last_idx = 0;
    while (pof2 * 2 <= size)
        pof2 *= 2;
    rem = size - pof2;
    for (i = 0; i < pof2; i++)
        cnts[i] = count / pof2 + (i < count % pof2 ? 1 : 0);
    disps[0] = 0;
    for (i = 1; i < pof2; i++)
        disps[i] = disps[i - 1] + cnts[i - 1];

    /* pre-fold: odd ranks < 2*rem send to rank-1 (:127-170) */
    if (rank < 2 * rem) {
        if (rank % 2) {
            send_to(acc, (size_t) count * esz, rank - 1);
            newrank = -1;
        } else {
            recv_from(tmp, (size_t) count * esz, rank + 1);
            if ((rc = local_reduce("MPI_Reduce", tmp, acc, count, dt, op)))
                return rc;
            newrank = rank / 2;
        }
    } else
        newrank = rank - rem;

    /* recursive halving reduce-scatter (:190-250) */
    if (newrank != -1) {
        send_idx = recv_idx = 0;
        last_idx = pof2;
        for (mask = 1; mask < pof2;) {
            int newdst = newrank ^ mask, dst = newdst < rem ? newdst * 2 : newdst + rem;
            int send_cnt = 0, recv_cnt = 0;
            if (newrank < newdst) {
                send_idx = recv_idx + pof2 / (mask * 2);
                for (i = send_idx; i < last_idx; i++)
                    send_cnt += cnts[i];
                for (i = recv_idx; i < send_idx; i++)
                    recv_cnt += cnts[i];
            } else {
                recv_idx = send_idx + pof2 / (mask * 2);
                for (i = send_idx; i < recv_idx; i++)
                    send_cnt += cnts[i];
                for (i = recv_idx; i < last_idx; i++)
                    recv_cnt += cnts[i];
            }
            exchange(acc + (size_t) disps[send_idx] * esz, (size_t) send_cnt * esz, dst,
                     tmp + (size_t) disps[recv_idx] * esz, (size_t) recv_cnt * esz, dst);
            if ((rc = local_reduce("MPI_Reduce", tmp + (size_t) disps[recv_idx] * esz,
                                   acc + (size_t) disps[recv_idx] * esz, recv_cnt, dt, op)))
                return rc;
            send_idx = recv_idx;
            mask <<= 1;
            if (mask < pof2)
                last_idx = recv_idx + pof2 / mask;
        }
    }

    /* gather to root (:252-400): an excluded odd root takes newrank 0's role */
    if (root < 2 * rem) {
        if (root % 2) {
            if (rank == root) {
                recv_from(acc, (size_t) cnts[0] * esz, 0);
                newrank = 0;
                send_idx = 0;
                last_idx = 2;
            } else if (newrank == 0) {
                send_to(acc, (size_t) cnts[0] * esz, root);
                newrank = -1;
            }
            newroot = 0;
        } else
            newroot = root / 2;
    } else
        newroot = root - rem;

    if (newrank != -1) {
        j = 0;
        for (mask = 1; mask < pof2; mask <<= 1)
            j++;
        mask >>= 1;
        j--;
        while (mask > 0) {
            int newdst = newrank ^ mask, dst = newdst < rem ? newdst * 2 : newdst + rem;
            int send_cnt = 0, recv_cnt = 0, ndtr, nrtr;
            if (newdst == 0 && root < 2 * rem && root % 2)
                dst = root;
            ndtr = (newdst >> j) << j;
            nrtr = (newroot >> j) << j;
            if (newrank < newdst) {
                if (mask != pof2 / 2)
                    last_idx = last_idx + pof2 / (mask * 2);
                recv_idx = send_idx + pof2 / (mask * 2);
                for (i = send_idx; i < recv_idx; i++)
                    send_cnt += cnts[i];
                for (i = recv_idx; i < last_idx; i++)
                    recv_cnt += cnts[i];
            } else {
                recv_idx = send_idx - pof2 / (mask * 2);
                for (i = send_idx; i < last_idx; i++)
                    send_cnt += cnts[i];
                for (i = recv_idx; i < send_idx; i++)
                    recv_cnt += cnts[i];
            }
            if (ndtr == nrtr) {
                /* newdst's half holds the root: send and exit */
                send_to(acc + (size_t) disps[send_idx] * esz, (size_t) send_cnt * esz, dst);
                break;
            }
            recv_from(acc + (size_t) disps[recv_idx] * esz, (size_t) recv_cnt * esz, dst);
            if (newrank > newdst)
                send_idx = recv_idx;
            mask >>= 1;
            j--;
        }
    }
    return MPI_SUCCESS;
}

int MPI_Reduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype, MPI_Op op, int root,
               MPI_Comm comm)
{
    static const char *fc = "MPI_Reduce";
    int rank, size, rc, pof2 = 1, builtin;
    size_t esz, nbytes;
    char *acc, *tmp, *own = NULL;
    if ((rc = coll_args(fc, comm, count, datatype, root, &rank, &size, &esz)))
        return rc;
    if (op == MPI_OP_NULL || op == MPI_NO_OP || ((unsigned) op & 0x3c000000u) >> 26 != 6)
        return err(fc, MPI_ERR_OP, "%s", "Invalid MPI_Op");
    builtin = ((unsigned) op & 0xc0000000u) >> 30 == 1;
    if (builtin && (rc = MPIR_Op_check_dtype_table[op & 0xf] (datatype)) != MPI_SUCCESS)
        return MPIR_Err_return(fc, rc);
    if (count == 0)
        return MPI_SUCCESS;
    nbytes = (size_t) count * esz;
    if (rank == root && sendbuf == recvbuf)
        return err(fc, MPI_ERR_BUFFER, "%s", "Buffers must not be aliased");
    /* the root accumulates in recvbuf; everyone else in a temporary */
    if (rank == root) {
        acc = recvbuf;
    } else {
        acc = own = malloc(nbytes);
        if (!own)
            return err(fc, MPI_ERR_NO_MEM, "%s", "out of memory");
    }
    if (sendbuf != MPI_IN_PLACE)
        memcpy(acc, sendbuf, nbytes);
    tmp = malloc(nbytes);
    if (!tmp) {
        free(own);
        return err(fc, MPI_ERR_NO_MEM, "%s", "out of memory");
    }
    while (pof2 * 2 <= size)
        pof2 *= 2;
    if (size == 1)
        rc = MPI_SUCCESS;
    else if (nbytes > 2048 && builtin && count >= pof2)     /* reduce.c:214-216 */
        rc = reduce_scatter_gather(acc, tmp, count, esz, datatype, op, root, rank, size);
    else
        rc = reduce_binomial(acc, tmp, count, esz, datatype, op, root, rank, size);
    free(tmp);
    free(own);
    return coll_finish(fc, rc ? MPIR_Err_return(fc, rc) : MPI_SUCCESS);
}

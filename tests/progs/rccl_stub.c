/*
 * rccl_stub.c -- TEST ONLY: a stand-in librccl that records every call the
 * device collectives make (csrc/host/coll_hip.c loads it through
 * MPIR_TEST_RCCL_LIBRARY), one line per call into $RCCL_STUB_LOG.<rank>, so a
 * CPU test can check that the N ranks' RCCL call sequences match one another
 * (tests/test_rccl_sequence_cpu.py).  It moves no data and touches no buffer.
 *
 * Lines:  init <rank> <nranks>
 *         group_start | group_end
 *         send <bytes> <type> <peer> | recv <bytes> <type> <peer>
 *         allreduce <count> <type> <op> | reduce_scatter <recvcount> <type> <op>
 *         reduce <count> <type> <op> <root> | destroy
 *         note <text>                       (from the harness: memcpy, combine, ...)
 */
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <rccl/rccl.h>

struct ncclComm {
    int rank, nranks;
};

static FILE *logf_;
static int depth;           /* group nesting, as NCCL allows it */

static void out(const char *fmt, ...)
{
    va_list ap;
    if (!logf_)
        return;
    va_start(ap, fmt);
    vfprintf(logf_, fmt, ap);
    va_end(ap);
    fputc('\n', logf_);
    fflush(logf_);
}

/* the harness's own events, in the same stream */
void rccl_stub_note(const char *text)
{
    out("note %s", text);
}

ncclResult_t ncclGetUniqueId(ncclUniqueId *id)
{
    memset(id, 0, sizeof(*id));
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t *comm, int nranks, ncclUniqueId id, int rank)
{
    char path[4096];
    const char *base = getenv("RCCL_STUB_LOG");
    (void) id;
    if (!base || nranks < 1 || rank < 0 || rank >= nranks)
        return ncclInvalidArgument;
    snprintf(path, sizeof path, "%s.%d", base, rank);
    logf_ = fopen(path, "w");
    if (!logf_)
        return ncclSystemError;
    *comm = calloc(1, sizeof(struct ncclComm));
    (*comm)->rank = rank;
    (*comm)->nranks = nranks;
    out("init %d %d", rank, nranks);
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm)
{
    out("destroy");
    free(comm);
    return ncclSuccess;
}

ncclResult_t ncclGroupStart(void)
{
    if (depth++ == 0)
        out("group_start");
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd(void)
{
    if (depth == 0)
        return ncclInvalidUsage;
    if (--depth == 0)
        out("group_end");
    return ncclSuccess;
}

ncclResult_t ncclSend(const void *buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t s)
{
    (void) buf;
    (void) s;
    if (peer < 0 || peer >= comm->nranks || peer == comm->rank)
        return ncclInvalidArgument;
    out("send %zu %d %d", count, (int) t, peer);
    return ncclSuccess;
}

ncclResult_t ncclRecv(void *buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t s)
{
    (void) buf;
    (void) s;
    if (peer < 0 || peer >= comm->nranks || peer == comm->rank)
        return ncclInvalidArgument;
    out("recv %zu %d %d", count, (int) t, peer);
    return ncclSuccess;
}

ncclResult_t ncclAllReduce(const void *sb, void *rb, size_t count, ncclDataType_t t, ncclRedOp_t op,
                           ncclComm_t comm, hipStream_t s)
{
    (void) sb;
    (void) rb;
    (void) comm;
    (void) s;
    out("allreduce %zu %d %d", count, (int) t, (int) op);
    return ncclSuccess;
}

ncclResult_t ncclReduceScatter(const void *sb, void *rb, size_t recvcount, ncclDataType_t t, ncclRedOp_t op,
                               ncclComm_t comm, hipStream_t s)
{
    (void) sb;
    (void) rb;
    (void) comm;
    (void) s;
    out("reduce_scatter %zu %d %d", recvcount, (int) t, (int) op);
    return ncclSuccess;
}

ncclResult_t ncclReduce(const void *sb, void *rb, size_t count, ncclDataType_t t, ncclRedOp_t op, int root,
                        ncclComm_t comm, hipStream_t s)
{
    (void) sb;
    (void) rb;
    (void) s;
    if (root < 0 || root >= comm->nranks)
        return ncclInvalidArgument;
    out("reduce %zu %d %d %d", count, (int) t, (int) op, root);
    return ncclSuccess;
}

const char *ncclGetErrorString(ncclResult_t r)
{
    return r == ncclSuccess ? "success" : "stub error";
}

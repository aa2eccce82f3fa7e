/*
 * mpix_hip_coll.h -- device reduction collectives built on the MI355X
 * MPI_Reduce_local.
 *
 * These are the device-collective hooks of the reference's ADI
 * (MPID_Allreduce, src/mpid/ch3/include/mpid_coll.h:58; ch4_coll.h:92; and
 * the MPIR_Reduce_scatter_block path, reduce_scatter_block.c:99-160) for
 * buffers that live in HBM, one rank per GPU.  The cross-rank step is RCCL
 * over xGMI.  Two algorithms:
 *
 *   MPIX_HIP_ALG_REFERENCE_ORDER -- results bit-identical to MPICH's own
 *       schedules (allreduce_intra_smp.c -> reduce_intra_reduce_scatter_gather.c
 *       + bcast; reduce_scatter_block_intra_pairwise.c).  MI355X-native form:
 *       one all-to-all of blocks over all xGMI links (grouped ncclSend/ncclRecv),
 *       then ONE fused pass (MPIX_Reduce_local_multi) that applies the
 *       schedule's log2(p) / p-1 combine steps in its exact association and
 *       operand order, then an allgather of the reduced blocks.
 *   MPIX_HIP_ALG_RCCL -- ncclAllReduce / ncclReduceScatter (RCCL's own
 *       reduction order: results within the tolerance documented in DESIGN.md).
 *   MPIX_HIP_ALG_AUTO -- RCCL where it has the (op, type), else reference order;
 *       overridable with MPIR_CVAR_DEVICE_COLL_ALGORITHM=reference|rccl.
 *
 * Communicators: MPIX_Hip_comm_create wraps ncclCommInitRank (the caller
 * broadcasts the 128-byte unique id out of band, as MPICH would over PMI);
 * MPIX_Hip_comm_create_loopback builds `size` in-process virtual ranks on the
 * current device (one host thread per rank; transfers are device copies) so
 * the schedule logic is testable on one GPU.  RCCL is loaded with dlopen on
 * first use: MPI_Reduce_local itself never depends on it.
 *
 * Streams: stream == NULL runs on the communicator's stream and returns with
 * the result complete; otherwise the collective is enqueued on that stream.
 */
#ifndef MPIX_HIP_COLL_H_INCLUDED
#define MPIX_HIP_COLL_H_INCLUDED

#include "mpi_reduce_local.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct MPIX_Hip_comm_s *MPIX_Hip_comm;

#ifndef MPI_ERR_ROOT
#define MPI_ERR_ROOT 7      /* mpi.h.in:792 */
#endif

#define MPIX_HIP_UNIQUE_ID_BYTES 128
#define MPIX_HIP_ALG_AUTO 0
#define MPIX_HIP_ALG_REFERENCE_ORDER 1
#define MPIX_HIP_ALG_RCCL 2

MPICH_API_PUBLIC int MPIX_Hip_comm_get_unique_id(void *id);
MPICH_API_PUBLIC int MPIX_Hip_comm_create(const void *id, int size, int rank, MPIX_Hip_comm * comm);
MPICH_API_PUBLIC int MPIX_Hip_comm_create_loopback(int size, MPIX_Hip_comm * comms);
MPICH_API_PUBLIC int MPIX_Hip_comm_free(MPIX_Hip_comm * comm);
MPICH_API_PUBLIC int MPIX_Hip_comm_rank(MPIX_Hip_comm comm, int *rank);
MPICH_API_PUBLIC int MPIX_Hip_comm_size(MPIX_Hip_comm comm, int *size);

/* MPI_Allreduce semantics (sendbuf may be MPI_IN_PLACE). */
MPICH_API_PUBLIC int MPIX_Allreduce_hip(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
                       MPIX_Hip_comm comm, int algorithm, void *hip_stream);
/* MPI_Reduce semantics (reduce.c:382; MPI_IN_PLACE at the root only; recvbuf
 * significant at the root only).  Reference order: reduce_intra_smp.c ->
 * MPIR_Reduce_intra_auto on the node (binomial tree rooted at `root` for
 * count*size <= 2048 or count < pof2, else reduce-scatter + gather);
 * MPIX_HIP_ALG_RCCL: ncclReduce. */
MPICH_API_PUBLIC int MPIX_Reduce_hip(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype, MPI_Op op, int root,
                    MPIX_Hip_comm comm, int algorithm, void *hip_stream);
/* MPI_Reduce_scatter_block semantics (sendbuf may be MPI_IN_PLACE). */
MPICH_API_PUBLIC int MPIX_Reduce_scatter_block_hip(const void *sendbuf, void *recvbuf, int recvcount, MPI_Datatype datatype,
                                  MPI_Op op, MPIX_Hip_comm comm, int algorithm, void *hip_stream);
/* MPI_Reduce_scatter semantics (reduce_scatter.c:383; rank q receives
 * recvcounts[q] elements; sendbuf may be MPI_IN_PLACE).  Reference order:
 * MPIR_Reduce_scatter_intra_auto (recursive halving below 524288 total bytes,
 * else pairwise); MPIX_HIP_ALG_RCCL: ncclReduceScatter when the counts are
 * all equal, else the reference order. */
MPICH_API_PUBLIC int MPIX_Reduce_scatter_hip(const void *sendbuf, void *recvbuf, const int recvcounts[], MPI_Datatype datatype,
                            MPI_Op op, MPIX_Hip_comm comm, int algorithm, void *hip_stream);

/* MPI_Scan / MPI_Exscan semantics (scan.c, exscan.c; sendbuf may be
 * MPI_IN_PLACE; the exscan's recvbuf at rank 0 is left untouched).  Reference
 * order of the recursive doubling (scan_intra_recursive_doubling.c,
 * exscan_intra_recursive_doubling.c); RCCL has no scan, so every algorithm
 * value runs the reference order. */
MPICH_API_PUBLIC int MPIX_Scan_hip(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
                  MPIX_Hip_comm comm, int algorithm, void *hip_stream);
MPICH_API_PUBLIC int MPIX_Exscan_hip(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
                    MPIX_Hip_comm comm, int algorithm, void *hip_stream);

#ifdef __cplusplus
}
#endif
#endif /* MPIX_HIP_COLL_H_INCLUDED */

/*
 * mpi_pip.h -- the MPI runtime subset that config 1 (examples/cpi.c under
 * `mpiexec -n 2`) needs around the hot path:
 * init/finalize, the world communicator, Bcast, Reduce, Barrier, Wtime.
 *
 * Ranks are processes started by mpich-pip_amd/bin/mpiexec (fork + exec);
 * they share one POSIX shared-memory segment that carries every transfer,
 * standing in for PiP's shared address space (pmip_cb.c:485-497).  Every
 * reduction step runs through MPIR_Reduce_local: the HIP kernels, or, for
 * host operands of at most MPIR_CVAR_REDUCE_LOCAL_HOST_MAX_KB, the same
 * functors compiled for the host (csrc/hip/kernel_table.hpp); a builtin op
 * with no HIP device is an error, never a CPU fallback.  Counts that differ
 * across ranks give MPI_ERR_TRUNCATE / MPI_ERR_OTHER on the receiving ranks.
 *
 * Reference interfaces replaced (file:line under the reference tree):
 *   MPI_Comm, MPI_COMM_WORLD/SELF/NULL     src/include/mpi.h.in:89,289-291
 *   MPI_MAX_PROCESSOR_NAME (128)           configure.ac:5506
 *   MPI_ERR_COMM 5, MPI_ERR_ROOT 7,        src/include/mpi.h.in:790-793
 *   MPI_ERR_TRUNCATE 14
 *   MPI_Init / MPI_Finalize                src/mpi/init/init.c:118, finalize.c
 *   MPI_Comm_size / MPI_Comm_rank          src/mpi/comm/comm_size.c, comm_rank.c
 *   MPI_Get_processor_name, MPI_Wtime      src/mpi/misc/getpname.c, src/mpi/timer/wtime.c
 *   MPI_Barrier                            src/mpi/coll/barrier/barrier_intra_dissemination.c
 *   MPI_Bcast   (binomial)                 src/mpi/coll/bcast/bcast_intra_binomial.c:68-163
 *   MPI_Reduce  (auto: binomial or reduce-scatter + gather)
 *                                          src/mpi/coll/reduce/reduce.c:170-225,
 *                                          reduce_intra_binomial.c:100-160,
 *                                          reduce_intra_reduce_scatter_gather.c:40-400
 */
#ifndef MPI_PIP_H_INCLUDED
#define MPI_PIP_H_INCLUDED

#include "mpi_reduce_local.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef int MPI_Comm;
#define MPI_COMM_NULL  ((MPI_Comm)0x04000000)
#define MPI_COMM_WORLD ((MPI_Comm)0x44000000)
#define MPI_COMM_SELF  ((MPI_Comm)0x44000001)

#define MPI_MAX_PROCESSOR_NAME 128
#define MPI_ERR_COMM  5
#define MPI_ERR_ROOT  7
#define MPI_ERR_TRUNCATE 14

MPICH_API_PUBLIC int MPI_Init(int *argc, char ***argv);
MPICH_API_PUBLIC int MPI_Initialized(int *flag);
MPICH_API_PUBLIC int MPI_Finalize(void);
MPICH_API_PUBLIC int MPI_Finalized(int *flag);
MPICH_API_PUBLIC int MPI_Abort(MPI_Comm comm, int errorcode);
MPICH_API_PUBLIC int MPI_Comm_size(MPI_Comm comm, int *size);
MPICH_API_PUBLIC int MPI_Comm_rank(MPI_Comm comm, int *rank);
MPICH_API_PUBLIC int MPI_Get_processor_name(char *name, int *resultlen);
MPICH_API_PUBLIC double MPI_Wtime(void);
MPICH_API_PUBLIC double MPI_Wtick(void);
MPICH_API_PUBLIC int MPI_Barrier(MPI_Comm comm);
MPICH_API_PUBLIC int MPI_Bcast(void *buffer, int count, MPI_Datatype datatype, int root, MPI_Comm comm);
MPICH_API_PUBLIC int MPI_Reduce(const void *sendbuf, void *recvbuf, int count, MPI_Datatype datatype, MPI_Op op, int root,
               MPI_Comm comm);

#ifdef __cplusplus
}
#endif
#endif /* MPI_PIP_H_INCLUDED */

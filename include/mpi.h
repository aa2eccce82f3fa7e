/*
 * mpi.h -- umbrella header: everything this library implements of the MPI
 * C API (MPICH 3.3 x86-64 ABI values).
 *   mpi_reduce_local.h  MPI_Reduce_local, MPI_Op_*, op tables, error classes
 *   mpi_pip.h           the runtime subset (Init, Comm_size/rank, Bcast, Reduce, ...)
 *   mpix_hip_coll.h     device-buffer Allreduce / Reduce_scatter_block (MPIX_)
 */
#ifndef MPI_H_INCLUDED
#define MPI_H_INCLUDED
#include "mpi_reduce_local.h"
#include "mpi_pip.h"
#include "mpix_hip_coll.h"
#endif

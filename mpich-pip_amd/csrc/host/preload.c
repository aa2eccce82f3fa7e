/*
 * preload.c -- the LD_PRELOAD form of the drop-in (Option 2).
 *
 * An installed MPICH 3.3 libmpi is built with -fvisibility=hidden
 * (configure.ac:1443, PAC_CHECK_VISIBILITY; only MPICH_API_PUBLIC symbols are
 * exported, mpi.h.in:13), so its collective schedules call their own
 * MPIR_Reduce_local and MPIR_Op_table directly, out of reach of symbol
 * interposition.  What a preloaded library CAN replace is the public
 * MPI_Reduce_local / PMPI_Reduce_local (reduce_local.c:11-20,155).  This shim
 * exports exactly those two symbols; everything else in
 * libmpich_reduce_local_preload.so is hidden, so libmpi keeps its own
 * MPI_Op_create and object store:
 *   - builtin op: the drop-in's validation and GPU combine
 *     (MPIR_Reduce_local_checked);
 *   - user-defined op: the handle belongs to libmpi's object store, so the
 *     call goes on to libmpi's PMPI_Reduce_local (dlsym RTLD_NEXT).
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdio.h>

#include "mpir_op_objects.h"
#include "mpir_op_types.h"

typedef int (*reduce_local_fn) (const void *, void *, int, MPI_Datatype, MPI_Op);

static int forward(const void *inbuf, void *inoutbuf, int count, MPI_Datatype datatype, MPI_Op op)
{
    /* racing first calls resolve the same symbol; the atomics make that well defined */
    static reduce_local_fn cached;
    reduce_local_fn next = __atomic_load_n(&cached, __ATOMIC_ACQUIRE);
    if (!next) {
        next = (reduce_local_fn) dlsym(RTLD_NEXT, "PMPI_Reduce_local");
        if (!next) {
            fprintf(stderr, "libmpich_reduce_local_preload: no PMPI_Reduce_local after the shim\n");
            return MPI_ERR_INTERN;
        }
        __atomic_store_n(&cached, next, __ATOMIC_RELEASE);
    }
    return next(inbuf, inoutbuf, count, datatype, op);
}

__attribute__ ((visibility("default")))
int PMPI_Reduce_local(const void *inbuf, void *inoutbuf, int count, MPI_Datatype datatype, MPI_Op op)
{
    if (MPIR_HANDLE_GET_KIND(op) != MPIR_HANDLE_KIND_BUILTIN)
        return forward(inbuf, inoutbuf, count, datatype, op);
    return MPIR_Reduce_local_checked(inbuf, inoutbuf, count, datatype, op);
}

__attribute__ ((visibility("default")))
int MPI_Reduce_local(const void *inbuf, void *inoutbuf, int count, MPI_Datatype datatype, MPI_Op op)
{
    return PMPI_Reduce_local(inbuf, inoutbuf, count, datatype, op);
}

/*
 * mpich_glue.c -- the drop-in's thread-safety hooks bound to MPICH's own
 * state, for INTEGRATION.md Option 1 (DROPIN_SRC compiled into libmpi with
 * -DMPIR_DROPIN_IN_LIBMPI).  This is the only file of the library that
 * includes MPICH's internal header; it is compiled with libmpi's own include
 * path and flags, and never in the standalone build (whose hooks are in
 * op_kernels.c and op_objects.c).
 *
 *   MPIR_Op_errno_ptr()   -> &MPIR_Per_thread.op_errno through
 *                            MPID_THREADPRIV_KEY_GET_ADDR (mpir_thread.h:61-82),
 *                            the slot the unchanged schedules reset and read
 *                            themselves (reduce_scatter_block_intra_pairwise.c:48-57,
 *                            153-162; reduce_intra_reduce_scatter_gather.c:63-71,
 *                            401-412; scan / exscan / reduce_scatter*), and
 *                            MPIR_Reduce_local's own reset / read
 *                            (reduce_local.c:51-59,107-117);
 *   MPIR_Dropin_local_ranks() -> MPIR_Process.comm_world->node_comm->local_size,
 *                            the ranks sharing this node's CPUs (sizes the
 *                            host combine's threads; op_kernels.c);
 *   MPIR_DROPIN_CS_GLOBAL -> MPID_THREAD_CS_ENTER/EXIT(GLOBAL,
 *                            MPIR_THREAD_GLOBAL_ALLFUNC_MUTEX), the section
 *                            MPI_Reduce_local, MPI_Op_create, MPI_Op_free and
 *                            MPI_Op_commutative hold (reduce_local.c:162,205,
 *                            op_create.c:151-164, op_free.c:86,120,
 *                            op_commutative.c:109,136);
 *   MPIR_DROPIN_CS_HANDLE -> MPID_THREAD_CS_ENTER/EXIT(POBJ | VCI,
 *                            MPIR_THREAD_POBJ_HANDLE_MUTEX), the section
 *                            MPIR_Handle_obj_alloc / MPIR_Handle_obj_free hold
 *                            around the avail list (mpir_handlemem.h:221-225,
 *                            338-384) -- libmpi's inline releases of
 *                            schedule-held ops take the same one.
 * Whichever granularity libmpi was configured with, the macros expand to the
 * same locking its own handle code does; under MPICH_THREAD_GRANULARITY
 * GLOBAL the POBJ / VCI ones are empty and the GLOBAL section is what
 * serialises a create against a progress-engine release.
 */
#include "mpiimpl.h"

int *MPIR_Op_errno_ptr(void)
{
    MPIR_Per_thread_t *per_thread = NULL;
    int err = 0;

    MPID_THREADPRIV_KEY_GET_ADDR(MPIR_ThreadInfo.isThreaded, MPIR_Per_thread_key,
                                 MPIR_Per_thread, per_thread, &err);
    MPIR_Assert(err == 0);
    return &per_thread->op_errno;
}

/* Ranks of MPI_COMM_WORLD on this node: MPICH's node communicator
 * (mpir_comm.h:148, built by MPIR_Comm_commit when the world is node-aware),
 * else 0 (unknown: the library reads the launcher's environment).  The op
 * layer hands it to MPIR_Hip_set_local_ranks() before its first combine, so the
 * host combine's threads are this rank's share of the node's CPUs. */
int MPIR_Dropin_local_ranks(void)
{
    MPIR_Comm *world = MPIR_Process.comm_world;
    if (world && world->node_comm)
        return world->node_comm->local_size;
    return 0;
}

/* which: 0 = GLOBAL, 1 = HANDLE (enum in mpir_op_types.h, not included here:
 * this file sees MPICH's mpi.h, not the drop-in's) */
void MPIR_Dropin_cs_enter(int which)
{
    if (which == 0) {
        MPID_THREAD_CS_ENTER(GLOBAL, MPIR_THREAD_GLOBAL_ALLFUNC_MUTEX);
    } else {
        MPID_THREAD_CS_ENTER(POBJ, MPIR_THREAD_POBJ_HANDLE_MUTEX);
        MPID_THREAD_CS_ENTER(VCI, MPIR_THREAD_POBJ_HANDLE_MUTEX);
    }
}

void MPIR_Dropin_cs_exit(int which)
{
    if (which == 0) {
        MPID_THREAD_CS_EXIT(GLOBAL, MPIR_THREAD_GLOBAL_ALLFUNC_MUTEX);
    } else {
        MPID_THREAD_CS_EXIT(VCI, MPIR_THREAD_POBJ_HANDLE_MUTEX);
        MPID_THREAD_CS_EXIT(POBJ, MPIR_THREAD_POBJ_HANDLE_MUTEX);
    }
}

/*
 * op_objects.c -- the MPIR_Op object store (include/mpir_op_objects.h).
 *
 * Reference: src/mpi/coll/op/op_create.c:27-104 (MPIR_Op_builtin,
 * MPIR_Op_direct, MPIR_Op_mem, MPIR_Op_create_impl), op_free.c:33-49
 * (MPIR_Op_free_impl), op_commutative.c:39-74, and the handle allocator
 * src/include/mpir_handlemem.h:88-172 (direct / indirect block set-up),
 * :233-321 (alloc), :334-385 (free), :390-422 (indirect lookup).
 *
 * The allocator keeps MPICH's representation exactly -- the avail list of
 * MPIR_Handle_common threaded through free objects, handles written into
 * each object when its block is set up, indirect blocks of
 * MPIR_HANDLE_NUM_INDICES objects in a table of MPIR_HANDLE_NUM_BLOCKS --
 * because unchanged MPICH code walks it with inline macros (MPIR_Getb_ptr,
 * MPIR_Handle_obj_free).  The avail list is guarded by the HANDLE section
 * and the MPI entry points (reduce_local.c) hold the GLOBAL one, as
 * MPIR_Handle_obj_alloc / _free and MPI_Op_create / _free do
 * (mpir_handlemem.h:221-225,338-384, op_create.c:151-164, op_free.c:86,120).
 * Standalone, HANDLE is this library's mutex and GLOBAL has nothing to guard;
 * compiled into libmpi (-DMPIR_DROPIN_IN_LIBMPI) both are MPICH's own
 * critical sections (mpich_glue.c), the ones libmpi's inline op releases take.
 */
#include <pthread.h>
#include <stdlib.h>

#include "mpir_op_objects.h"
#include "mpir_op_types.h"

MPIR_Op MPIR_Op_builtin[MPIR_OP_N_BUILTIN];
MPIR_Op MPIR_Op_direct[MPIR_OP_PREALLOC];
MPIR_Object_alloc_t MPIR_Op_mem = { 0, 0, 0, 0, MPIR_OP_OBJ_KIND, sizeof(MPIR_Op), MPIR_Op_direct,
    MPIR_OP_PREALLOC
};

#ifndef MPIR_DROPIN_IN_LIBMPI
static pthread_mutex_t op_mem_lock = PTHREAD_MUTEX_INITIALIZER;

void MPIR_Dropin_cs_enter(int which)
{
    if (which == MPIR_DROPIN_CS_HANDLE)
        pthread_mutex_lock(&op_mem_lock);
}

void MPIR_Dropin_cs_exit(int which)
{
    if (which == MPIR_DROPIN_CS_HANDLE)
        pthread_mutex_unlock(&op_mem_lock);
}
#endif

static unsigned make_handle(unsigned kind, unsigned bits)
{
    return (kind << 30) | ((unsigned) MPIR_OP_OBJ_KIND << 26) | bits;
}

/* MPIR_Handle_direct_init (mpir_handlemem.h:88-117): chain the direct block */
static MPIR_Handle_common *direct_init(void)
{
    char *p = (char *) MPIR_Op_mem.direct;
    MPIR_Handle_common *h = NULL;
    for (int i = 0; i < MPIR_Op_mem.direct_size; i++) {
        h = (MPIR_Handle_common *) (void *) p;
        p += MPIR_Op_mem.size;
        h->next = p;
        h->handle = (int) make_handle(MPIR_HANDLE_KIND_DIRECT, (unsigned) i);
    }
    if (h)
        h->next = NULL;
    return (MPIR_Handle_common *) MPIR_Op_mem.direct;
}

/* MPIR_Handle_indirect_init (mpir_handlemem.h:120-173): one more block */
static MPIR_Handle_common *indirect_init(void)
{
    char *block, *p;
    MPIR_Handle_common *h = NULL;
    if (!MPIR_Op_mem.indirect) {
        MPIR_Op_mem.indirect = calloc(MPIR_HANDLE_NUM_BLOCKS, sizeof(void *));
        if (!MPIR_Op_mem.indirect)
            return NULL;
        MPIR_Op_mem.indirect_size = 0;
    }
    if (MPIR_Op_mem.indirect_size >= MPIR_HANDLE_NUM_BLOCKS)
        return NULL;
    block = calloc(MPIR_HANDLE_NUM_INDICES, (size_t) MPIR_Op_mem.size);
    if (!block)
        return NULL;
    p = block;
    for (int i = 0; i < MPIR_HANDLE_NUM_INDICES; i++) {
        h = (MPIR_Handle_common *) (void *) p;
        p += MPIR_Op_mem.size;
        h->next = p;
        h->handle = (int) make_handle(MPIR_HANDLE_KIND_INDIRECT,
                                      ((unsigned) MPIR_Op_mem.indirect_size << 12) | (unsigned) i);
    }
    h->next = NULL;
    (*MPIR_Op_mem.indirect)[MPIR_Op_mem.indirect_size] = block;
    MPIR_Op_mem.indirect_size++;
    return (MPIR_Handle_common *) (void *) block;
}

/* MPIR_Handle_obj_alloc_unsafe (mpir_handlemem.h:233-321) */
static MPIR_Op *obj_alloc(void)
{
    MPIR_Handle_common *p;
    if (MPIR_Op_mem.avail) {
        p = MPIR_Op_mem.avail;
        MPIR_Op_mem.avail = (MPIR_Handle_common *) p->next;
    } else {
        if (!MPIR_Op_mem.initialized) {
            MPIR_Op_mem.initialized = 1;
            p = direct_init();
        } else {
            p = indirect_init();
        }
        if (p)
            MPIR_Op_mem.avail = (MPIR_Handle_common *) p->next;
    }
    return (MPIR_Op *) (void *) p;
}

/* MPIR_Handle_obj_free (mpir_handlemem.h:334-385) */
static void obj_free(MPIR_Op * op_ptr)
{
    MPIR_Handle_common *h = (MPIR_Handle_common *) (void *) op_ptr;
    h->next = MPIR_Op_mem.avail;
    MPIR_Op_mem.avail = h;
}

/* MPIR_Getb_ptr(Op, OP, a, 0xff, ptr) (mpir_objects.h:441-460, 487) and
 * MPIR_Handle_get_ptr_indirect (mpir_handlemem.h:390-422) */
MPIR_Op *MPIR_Op_get_ptr_fn(MPI_Op op)
{
    const unsigned a = (unsigned) op;
    switch (MPIR_HANDLE_GET_KIND(a)) {
    case MPIR_HANDLE_KIND_BUILTIN:
        return (a & 0xffu) < MPIR_OP_N_BUILTIN ? MPIR_Op_builtin + (a & 0xffu) : NULL;
    case MPIR_HANDLE_KIND_DIRECT:
        return MPIR_HANDLE_INDEX(a) < MPIR_OP_PREALLOC ? MPIR_Op_direct + MPIR_HANDLE_INDEX(a) : NULL;
    case MPIR_HANDLE_KIND_INDIRECT:{
            MPIR_Op *p = NULL;
            if (MPIR_HANDLE_GET_MPI_KIND(a) != (unsigned) MPIR_Op_mem.kind)
                return NULL;
            MPIR_Dropin_cs_enter(MPIR_DROPIN_CS_HANDLE);
            if ((int) MPIR_HANDLE_BLOCK(a) < MPIR_Op_mem.indirect_size &&
                MPIR_HANDLE_BLOCK_INDEX(a) < MPIR_HANDLE_NUM_INDICES)
                p = (MPIR_Op *) (void *) ((char *) (*MPIR_Op_mem.indirect)[MPIR_HANDLE_BLOCK(a)] +
                                          (size_t) MPIR_HANDLE_BLOCK_INDEX(a) * MPIR_Op_mem.size);
            MPIR_Dropin_cs_exit(MPIR_DROPIN_CS_HANDLE);
            return p;
        }
    default:
        return NULL;
    }
}

/* MPIR_Op_create_impl (op_create.c:73-104) */
int MPIR_Op_create_impl(MPI_User_function * user_fn, int commute, MPI_Op * op)
{
    MPIR_Op *op_ptr;
    MPIR_Dropin_cs_enter(MPIR_DROPIN_CS_HANDLE);     /* MPIR_Handle_obj_alloc */
    op_ptr = obj_alloc();
    if (op_ptr) {
        op_ptr->language = MPIR_LANG__C;
        op_ptr->kind = commute ? MPIR_OP_KIND__USER : MPIR_OP_KIND__USER_NONCOMMUTE;
        op_ptr->function.c_function = (void (*)(const void *, void *, const int *, const MPI_Datatype *)) user_fn;
        __atomic_store_n(&op_ptr->ref_count, 1, __ATOMIC_RELAXED);     /* MPIR_Object_set_ref */
    }
    MPIR_Dropin_cs_exit(MPIR_DROPIN_CS_HANDLE);
    if (!op_ptr) {
        MPIR_Err_set_detail("Out of memory (MPI_Op)");      /* "**nomem %s" */
        return MPI_ERR_OTHER;
    }
    *op = op_ptr->handle;       /* MPIR_OBJ_PUBLISH_HANDLE */
    return MPI_SUCCESS;
}

/* MPIR_Op_free_impl (op_free.c:33-49): release one reference
 * (MPIR_Op_ptr_release_ref, atomic like MPICH's lock-free ref counts), and
 * at zero MPIR_Handle_obj_free under the HANDLE section */
void MPIR_Op_free_impl(MPI_Op * op)
{
    MPIR_Op *op_ptr = MPIR_Op_get_ptr_fn(*op);
    if (op_ptr && __atomic_sub_fetch(&op_ptr->ref_count, 1, __ATOMIC_ACQ_REL) == 0) {
        MPIR_Dropin_cs_enter(MPIR_DROPIN_CS_HANDLE);
        obj_free(op_ptr);
        MPIR_Dropin_cs_exit(MPIR_DROPIN_CS_HANDLE);
    }
    *op = MPI_OP_NULL;
}

/* MPIR_Op_commutative (op_commutative.c:59-74) */
int MPIR_Op_commutative(MPIR_Op * op_ptr, int *commute)
{
    *commute = op_ptr->kind == MPIR_OP_KIND__USER_NONCOMMUTE ? 0 : 1;
    return MPI_SUCCESS;
}

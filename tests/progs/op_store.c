/*
 * op_store.c -- user-defined ops as unchanged MPICH code sees them.
 *
 * MPICH resolves an MPI_Op handle with the inline macro MPIR_Op_get_ptr
 * (src/include/mpir_objects.h:441-460,487) over the exported MPIR_Op_builtin /
 * MPIR_Op_direct / MPIR_Op_mem, bumps the reference count in place
 * (MPIR_Op_add_ref_if_not_builtin, mpir_op.h:161-169, used by
 * mpidu_sched.c:800) and frees through MPIR_Handle_obj_free
 * (mpir_handlemem.h:334-385, via MPIR_Op_release_if_not_builtin).  This
 * program restates those macros the way libmpi inlines them and checks them
 * against the library's MPI_Op_create / MPI_Op_free / MPIR_Reduce_local.
 * Host buffers only: runs without a GPU.
 */
#include <stdio.h>
#include <string.h>

#include "mpir_op_objects.h"

#define CHECK(c) do { if (!(c)) { fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); return 1; } } while (0)

/* MPIR_Getb_ptr(Op, OP, a, 0x000000ff, ptr), as libmpi expands it */
static MPIR_Op *getb_ptr(MPI_Op a)
{
    switch (MPIR_HANDLE_GET_KIND(a)) {
    case MPIR_HANDLE_KIND_BUILTIN:
        return MPIR_Op_builtin + ((unsigned) a & 0x000000ffu);
    case MPIR_HANDLE_KIND_DIRECT:
        return MPIR_Op_direct + MPIR_HANDLE_INDEX(a);
    case MPIR_HANDLE_KIND_INDIRECT:
        /* MPIR_Handle_get_ptr_indirect (mpir_handlemem.h:390-422) */
        if (MPIR_HANDLE_GET_MPI_KIND(a) != (unsigned) MPIR_Op_mem.kind)
            return NULL;
        if ((int) MPIR_HANDLE_BLOCK(a) >= MPIR_Op_mem.indirect_size)
            return NULL;
        return (MPIR_Op *) (void *) ((char *) (*MPIR_Op_mem.indirect)[MPIR_HANDLE_BLOCK(a)] +
                                     MPIR_HANDLE_BLOCK_INDEX(a) * MPIR_Op_mem.size);
    default:
        return NULL;
    }
}

/* MPIR_Op_ptr_release + MPIR_Handle_obj_free, as libmpi inlines them */
static void release_inline(MPIR_Op * p)
{
    if (--p->ref_count == 0) {
        MPIR_Handle_common *h = (MPIR_Handle_common *) (void *) p;
        h->next = MPIR_Op_mem.avail;
        MPIR_Op_mem.avail = h;
    }
}

static void twice_plus(void *in, void *inout, int *len, MPI_Datatype * dt)
{
    int *a = (int *) in, *b = (int *) inout;
    (void) dt;
    for (int i = 0; i < *len; i++)
        b[i] = 2 * b[i] + a[i];
}

static void plus(void *in, void *inout, int *len, MPI_Datatype * dt)
{
    int *a = (int *) in, *b = (int *) inout;
    (void) dt;
    for (int i = 0; i < *len; i++)
        b[i] += a[i];
}

int main(void)
{
    MPI_Op op, op2, kept;
    MPIR_Op *p;
    int in[4] = { 1, 2, 3, 4 }, io[4] = { 10, 20, 30, 40 }, commute = -1;

    MPIX_Reduce_local_set_errhandler(MPI_ERRORS_RETURN);
    CHECK(sizeof(MPIR_Op) == 24 && sizeof(MPIR_Handle_common) == 16 && sizeof(MPIR_Object_alloc_t) == 56);
    CHECK(MPIR_Op_mem.kind == MPIR_OP_OBJ_KIND && MPIR_Op_mem.size == (int) sizeof(MPIR_Op));
    CHECK(MPIR_Op_mem.direct == (void *) MPIR_Op_direct && MPIR_Op_mem.direct_size == MPIR_OP_PREALLOC);

    /* builtin ops resolve to the (zeroed) builtin objects: commutative */
    p = getb_ptr(MPI_SUM);
    CHECK(p == &MPIR_Op_builtin[3]);
    CHECK(MPIR_Op_commutative(p, &commute) == 0 && commute == 1);

    /* a user op: the object libmpi finds carries the function, kind, language, refcount */
    CHECK(MPI_Op_create(twice_plus, 0, &op) == MPI_SUCCESS);
    CHECK((unsigned) op == 0x98000000u);                 /* first direct handle */
    p = getb_ptr(op);
    CHECK(p == &MPIR_Op_direct[0] && p->handle == op);
    CHECK(p->function.c_function == (void (*)(const void *, void *, const int *, const MPI_Datatype *)) twice_plus);
    CHECK(p->kind == MPIR_OP_KIND__USER_NONCOMMUTE && p->language == MPIR_LANG__C && p->ref_count == 1);
    CHECK(MPIR_Op_is_commutative(op) == 0);
    CHECK(MPIR_Op_commutative(p, &commute) == 0 && commute == 0);

    /* a nonblocking schedule holds a reference (MPIR_Op_add_ref_if_not_builtin) ... */
    p->ref_count++;
    kept = op;
    /* ... so the user's MPI_Op_free leaves the object alive */
    CHECK(MPI_Op_free(&op) == MPI_SUCCESS && op == MPI_OP_NULL);
    CHECK(p->ref_count == 1);
    CHECK(MPIR_Reduce_local(in, io, 4, MPI_INT, kept) == MPI_SUCCESS);
    CHECK(io[0] == 21 && io[1] == 42 && io[2] == 63 && io[3] == 84);
    /* the schedule's release (inline MPIR_Handle_obj_free) returns it to the allocator */
    release_inline(p);
    CHECK(MPIR_Op_mem.avail == (MPIR_Handle_common *) (void *) p);
    CHECK(MPIR_Reduce_local(in, io, 4, MPI_INT, kept) == MPI_ERR_OP);   /* freed handle */
    /* and the next create reuses it, as MPICH's allocator does */
    CHECK(MPI_Op_create(plus, 1, &op2) == MPI_SUCCESS && op2 == kept);
    CHECK(p->kind == MPIR_OP_KIND__USER && p->ref_count == 1);

    /* past the 16 direct objects: indirect handles resolve through MPIR_Op_mem */
    {
        MPI_Op many[40];
        for (int i = 0; i < 40; i++)
            CHECK(MPI_Op_create(plus, 1, &many[i]) == MPI_SUCCESS);
        CHECK(MPIR_HANDLE_GET_KIND(many[39]) == MPIR_HANDLE_KIND_INDIRECT);
        CHECK(((unsigned) many[39] & 0xfc000000u) == 0xd8000000u);
        for (int i = 0; i < 40; i++) {
            MPIR_Op *q = getb_ptr(many[i]);
            CHECK(q && q->handle == many[i] && q->ref_count == 1 && q->kind == MPIR_OP_KIND__USER);
            CHECK(q == MPIR_Op_get_ptr_fn(many[i]));
        }
        memcpy(io, (int[4]) { 1, 1, 1, 1 }, sizeof io);
        CHECK(MPIR_Reduce_local(in, io, 4, MPI_INT, many[39]) == MPI_SUCCESS && io[3] == 5);
        for (int i = 0; i < 40; i++)
            CHECK(MPI_Op_free(&many[i]) == MPI_SUCCESS);
    }
    CHECK(MPI_Op_free(&op2) == MPI_SUCCESS);
    /* freeing a predefined op: "**permop" */
    op = MPI_MAX;
    {
        int cls = -1;
        CHECK(MPI_Error_class(MPI_Op_free(&op), &cls) == MPI_SUCCESS && cls == MPI_ERR_OP);
    }
    puts("op_store ok");
    return 0;
}

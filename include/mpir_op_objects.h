/*
 * mpir_op_objects.h -- the MPIR_Op object store, layout-compatible with
 * MPICH 3.3 so that unchanged libmpi code finds user-defined ops.
 *
 * Unchanged MPICH code resolves an MPI_Op handle to its object with the
 * inline macro MPIR_Op_get_ptr (src/include/mpir_objects.h:487, expanding
 * MPIR_Getb_ptr :441-460): builtin handles index MPIR_Op_builtin, direct
 * handles MPIR_Op_direct, indirect handles the blocks hanging off MPIR_Op_mem
 * (MPIR_Handle_get_ptr_indirect, src/include/mpir_handlemem.h:390-422).  The
 * call sites include allreduce.c:419, reduce.c:492, scan.c:248,
 * reduce_scatter_block.c:411, and mpidu_sched.c:800
 * (MPIR_Op_add_ref_if_not_builtin, which bumps ref_count in place), and
 * MPIR_Op_release_if_not_builtin frees through MPIR_Handle_obj_free, which
 * pushes the object onto MPIR_Op_mem.avail (mpir_handlemem.h:334-385).  This
 * library owns those three symbols, so its MPI_Op_create / MPI_Op_free /
 * MPIR_Reduce_local and that inline code work on the same objects.
 *
 * Layout (x86-64, C-only ch3 build, MPICH_THREAD_REFCOUNT NONE or LOCKFREE:
 * both give a 4-byte ref count; MPID_DEV_OP_DECL is not defined for ch3):
 *   MPIR_Op                 24 bytes: handle @0, ref_count @4, kind @8,
 *                           language @12, function @16      (mpir_op.h:102-110)
 *   MPIR_Handle_common      handle @0, ref_count @4, next @8 (mpir_objects.h:412-416)
 *   MPIR_Object_alloc_t     avail, initialized, indirect, indirect_size, kind,
 *                           size, direct, direct_size        (mpir_objects.h:420-430)
 * ch4 appends MPIDI_Devop_t to MPIR_Op (ch4/include/mpidpre.h:500): a ch4
 * build must add the same bytes here (MPIR_OP_DEV_BYTES).
 */
#ifndef MPIR_OP_OBJECTS_H_INCLUDED
#define MPIR_OP_OBJECTS_H_INCLUDED

#include "mpi_reduce_local.h"

#ifdef __cplusplus
extern "C" {
#endif

#ifndef MPIR_OP_DEV_BYTES
#define MPIR_OP_DEV_BYTES 0
#endif

/* handle layout (mpir_objects.h:144-205) */
#define MPIR_OP_OBJ_KIND        0x6     /* MPII_Object_kind MPIR_OP */
#define MPIR_HANDLE_KIND_INVALID  0x0
#define MPIR_HANDLE_KIND_BUILTIN  0x1
#define MPIR_HANDLE_KIND_DIRECT   0x2
#define MPIR_HANDLE_KIND_INDIRECT 0x3
#define MPIR_HANDLE_GET_KIND(a)     (((unsigned)(a) & 0xc0000000u) >> 30)
#define MPIR_HANDLE_GET_MPI_KIND(a) (((unsigned)(a) & 0x3c000000u) >> 26)
#define MPIR_HANDLE_INDEX(a)        ((unsigned)(a) & 0x03ffffffu)
#define MPIR_HANDLE_BLOCK(a)        (((unsigned)(a) & 0x03fff000u) >> 12)
#define MPIR_HANDLE_BLOCK_INDEX(a)  ((unsigned)(a) & 0x00000fffu)
#define MPIR_HANDLE_NUM_BLOCKS      8192
#define MPIR_HANDLE_NUM_INDICES     1024
#define MPIR_OP_PREALLOC            16          /* op_create.c:29-31 */

/* MPIR_Op_kind (mpir_op.h:25-43) */
#define MPIR_OP_KIND__USER_NONCOMMUTE 32
#define MPIR_OP_KIND__USER            33
/* MPIR_Lang_t (mpir_misc.h:40-48), C-only build */
#define MPIR_LANG__C 0

typedef int MPI_Fint;

typedef union MPIR_User_function {
    void (*c_function) (const void *, void *, const int *, const MPI_Datatype *);
    void (*f77_function) (const void *, void *, const MPI_Fint *, const MPI_Fint *);
} MPIR_User_function;

typedef struct MPIR_Op {
    int handle;
    int ref_count;
    int kind;                   /* MPIR_Op_kind */
    int language;               /* MPIR_Lang_t */
    MPIR_User_function function;
#if MPIR_OP_DEV_BYTES
    char dev[MPIR_OP_DEV_BYTES];
#endif
} MPIR_Op;

typedef struct MPIR_Handle_common {
    int handle;
    int ref_count;
    void *next;
} MPIR_Handle_common;

typedef struct MPIR_Object_alloc_t {
    MPIR_Handle_common *avail;
    int initialized;
    void *(*indirect)[];
    int indirect_size;
    int kind;                   /* MPII_Object_kind */
    int size;
    void *direct;
    int direct_size;
} MPIR_Object_alloc_t;

extern MPIR_Op MPIR_Op_builtin[MPIR_OP_N_BUILTIN];
extern MPIR_Op MPIR_Op_direct[MPIR_OP_PREALLOC];
extern MPIR_Object_alloc_t MPIR_Op_mem;

/* handle -> object, MPIR_Op_get_ptr semantics (NULL for an invalid kind or an
 * indirect block that was never allocated).  The object may be free. */
MPIR_Op *MPIR_Op_get_ptr_fn(MPI_Op op);

/* MPIR_Op_create_impl (op_create.c:73-104), MPIR_Op_free_impl (op_free.c:33-49),
 * MPIR_Op_commutative (op_commutative.c:39-60) */
int MPIR_Op_create_impl(MPI_User_function * user_fn, int commute, MPI_Op * op);
void MPIR_Op_free_impl(MPI_Op * op);
int MPIR_Op_commutative(MPIR_Op * op_ptr, int *commute);

#ifdef __cplusplus
}
#endif
#endif /* MPIR_OP_OBJECTS_H_INCLUDED */

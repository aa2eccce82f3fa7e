/*
 * mpir_op_types.h -- the (MPI_Op x MPI_Datatype) matrix as data.
 *
 * The reference expresses the matrix as X-macro type groups expanded into
 * switch statements (src/include/mpir_op_util.h:263-364) plus a per-op list of
 * which groups each kernel and each check_dtype accepts (src/mpi/coll/op/op*.c).
 * Here each basic datatype carries its group bits and its device element
 * class, and each op carries two group masks: the groups its compute switch
 * handles and the groups its check_dtype accepts.  The two differ only for
 * LAND/LOR, whose check_dtype accepts FLOATING_POINT while the compute switch
 * has no float case (opland.c:105-106, oplor.c:105-106): float LAND/LOR pass
 * validation and then fail through op_errno, exactly like the reference.
 */
#ifndef MPIR_OP_TYPES_H_INCLUDED
#define MPIR_OP_TYPES_H_INCLUDED

#include "mpi_reduce_local.h"
#include "mpir_hip_reduce.h"

/* type groups (mpir_op_util.h:263-364), for a C-only x86-64 build */
#define G_C_INTEGER        0x001u   /* int, long, short, ..., int8_t..uint64_t */
#define G_C_INTEGER_EXTRA  0x002u   /* char */
#define G_FORTRAN_INTEGER  0x004u   /* MPI_AINT, MPI_OFFSET, MPI_COUNT */
#define G_FLOATING_POINT   0x008u   /* float, double */
#define G_FLOATING_EXTRA   0x010u   /* MPIX_C_FLOAT16 */
#define G_LOGICAL          0x020u   /* MPI_C_BOOL */
#define G_COMPLEX          0x040u   /* MPI_C_FLOAT_COMPLEX, MPI_C_DOUBLE_COMPLEX */
#define G_BYTE             0x080u   /* MPI_BYTE */
#define G_LOC_PAIR         0x100u   /* MPI_2INT, MPI_FLOAT_INT, ... (MAXLOC/MINLOC) */

typedef struct {
    MPI_Datatype datatype;
    int elem;           /* enum MPIR_Hip_elem */
    unsigned groups;
    const char *name;   /* MPI_Type_get_name spelling */
} MPIR_Type_desc;

/* descriptor of a predefined datatype, NULL if not a supported basic type */
const MPIR_Type_desc *MPIR_Type_lookup(MPI_Datatype datatype);

/* group masks an op index (1..14) handles in compute / accepts in check_dtype */
unsigned MPIR_Op_compute_groups(int opidx);
unsigned MPIR_Op_check_groups(int opidx);

/* Resolve (op index, datatype) to the device element class used by the
 * compute switch; returns 0 when the reference's compute switch would take
 * its `default:` branch (op_errno = MPI_ERR_OP). */
int MPIR_Op_resolve_elem(int opidx, MPI_Datatype datatype);

/* MPICH's per-thread state and critical sections, as the drop-in sees them.
 *   MPIR_Op_errno_ptr: the per-thread op error slot (mpir_thread.h:61-62,
 *     reduce_local.c:51-59,107-117);
 *   MPIR_Dropin_cs_enter / _exit: GLOBAL is the section MPI_Reduce_local and
 *     MPI_Op_create / _free / _commutative hold (reduce_local.c:162,205,
 *     op_create.c:151-164); HANDLE the one around the op store's avail list
 *     (mpir_handlemem.h:221-225,338-384).
 * Standalone build: this library's own TLS slot (op_kernels.c), a mutex for
 * HANDLE and nothing for GLOBAL (op_objects.c).  Compiled into libmpi with
 * -DMPIR_DROPIN_IN_LIBMPI (INTEGRATION.md Option 1): csrc/host/mpich_glue.c,
 * built against MPICH's mpiimpl.h, binds them to MPIR_Per_thread.op_errno --
 * the slot unchanged schedules reset and read themselves -- and to
 * MPID_THREAD_CS_ENTER / EXIT, so libmpi's inline op releases and this
 * library's creates serialise on the same lock. */
int *MPIR_Op_errno_ptr(void);
#define MPIR_DROPIN_CS_GLOBAL 0
#define MPIR_DROPIN_CS_HANDLE 1
void MPIR_Dropin_cs_enter(int which);
void MPIR_Dropin_cs_exit(int which);

/* record a HIP runtime failure inside an op kernel (sets op_errno) */
void MPIR_Op_report_hip_error(const char *opname, int hip_rc);

/* MPICH's error interface (src/mpi/errhan/errutil.c:238,848): weak
 * standalone definitions in errutil.c, libmpi's own when linked into MPICH */
#define MPIR_ERR_RECOVERABLE 0
#define MPIR_ERR_FATAL 1
int MPIR_Err_create_code(int lastcode, int fatal, const char fcname[], int line, int error_class,
                         const char generic_msg[], const char specific_msg[], ...);
int MPIR_Err_return_comm(void *comm_ptr, const char fcname[], int errcode);

/* the MPI-level error exit shared by the entry points: the thread's detail
 * text becomes the innermost error-stack level, then
 * MPIR_Err_return_comm(NULL, ...) applies COMM_WORLD's handler (fatal by
 * default) and returns the code (MPI_Error_class(code) is the class) */
int MPIR_Err_wrap_detail(const char *fcname, int line, int mpi_errno);

/* PMPI_Reduce_local's body (validation, MPIR_Reduce_local, error exit) */
int MPIR_Reduce_local_checked(const void *inbuf, void *inoutbuf, int count, MPI_Datatype datatype, MPI_Op op);
int MPIR_Err_return_at(const char *fcname, int line, int mpi_errno);
#define MPIR_Err_return(fc, e) MPIR_Err_return_at((fc), __LINE__, (e))

/* last error detail text for this thread (for MPI_Error_string) */
const char *MPIR_Err_last_detail(void);
void MPIR_Err_set_detail(const char *fmt, ...);

#endif /* MPIR_OP_TYPES_H_INCLUDED */

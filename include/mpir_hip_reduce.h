/*
 * mpir_hip_reduce.h -- the thin C-ABI shim between MPICH's host C op layer
 * and the gfx950 HIP kernels.  Plain pointers and sizes only.
 *
 * The host C layer (the C files under mpich-pip_amd/csrc/host) keeps the reference's
 * structure: MPIR_SUM(invec, inoutvec, len, type) switches over the MPI
 * datatype exactly like src/mpi/coll/op/opsum.c:21-76, and where the
 * reference runs its scalar loop (MPIR_OP_TYPE_REDUCE_CASE,
 * src/include/mpir_op_util.h:48-55) it calls MPIR_Hip_reduce() with the
 * resolved (op, element class) pair instead.
 */
#ifndef MPIR_HIP_REDUCE_H_INCLUDED
#define MPIR_HIP_REDUCE_H_INCLUDED

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* op codes == the reference's MPIR_Op_table index (allreduce.c:121-129) */
enum MPIR_Hip_op {
    MPIR_HIP_OP_MAX = 1,
    MPIR_HIP_OP_MIN = 2,
    MPIR_HIP_OP_SUM = 3,
    MPIR_HIP_OP_PROD = 4,
    MPIR_HIP_OP_LAND = 5,
    MPIR_HIP_OP_BAND = 6,
    MPIR_HIP_OP_LOR = 7,
    MPIR_HIP_OP_BOR = 8,
    MPIR_HIP_OP_LXOR = 9,
    MPIR_HIP_OP_BXOR = 10,
    MPIR_HIP_OP_MINLOC = 11,
    MPIR_HIP_OP_MAXLOC = 12,
    MPIR_HIP_OP_REPLACE = 13,
    MPIR_HIP_NOPS = 14
};

/* element classes: the device storage type an MPI basic type maps to */
enum MPIR_Hip_elem {
    MPIR_HIP_I8 = 1, MPIR_HIP_U8, MPIR_HIP_I16, MPIR_HIP_U16,
    MPIR_HIP_I32, MPIR_HIP_U32, MPIR_HIP_I64, MPIR_HIP_U64,
    MPIR_HIP_F16, MPIR_HIP_F32, MPIR_HIP_F64,
    MPIR_HIP_CF32, MPIR_HIP_CF64,                 /* C float/double _Complex */
    MPIR_HIP_P2INT, MPIR_HIP_PFLOATINT, MPIR_HIP_PLONGINT,
    MPIR_HIP_PSHORTINT, MPIR_HIP_PDOUBLEINT,      /* MAXLOC/MINLOC pairs */
    MPIR_HIP_F80, MPIR_HIP_CF80,                  /* x87 long double (16 B slot), its _Complex */
    MPIR_HIP_PLDOUBLEINT,                         /* MPI_LONG_DOUBLE_INT pair (32 B) */
    MPIR_HIP_NELEMS
};

/* return codes */
#define MPIR_HIP_OK        0
#define MPIR_HIP_EBUFFER   1   /* host-only pointer where device memory is required */
#define MPIR_HIP_ERUNTIME  2   /* HIP runtime failure; see MPIR_Hip_error_string() */
#define MPIR_HIP_ENOKERNEL 3   /* (op, elem) pair has no kernel */
#define MPIR_HIP_ENODEV    4   /* no usable GPU */

/* Combine inoutbuf[i] = op(inoutbuf[i], inbuf[i]) for i < count elements of
 * class `elem`.  Pointers may be device, pinned-host or pageable-host memory
 * in any mix (host operands are staged through device scratch).
 * hip_stream: a hipStream_t, or NULL for the calling thread's library stream
 * on the device that owns inoutbuf.  sync != 0: wait for completion (and for
 * the copy-back of a host inoutbuf) before returning.  sync == 0 requires
 * both buffers device-resident on one device (else MPIR_HIP_EBUFFER). */
int MPIR_Hip_reduce(const void *inbuf, void *inoutbuf, uint64_t count, int op, int elem,
                    void *hip_stream, int sync);

/* Multi-operand combine: outbuf = fold(inbufs[0..n-1]) in one pass, in the
 * association of a reduction schedule (the schedule's MPIR_Reduce_local steps
 * fused; left operand = the step's inoutbuf):
 *   MPIR_HIP_ORDER_TREE  (n a power of two <= 64; one fused pass for n <= 8):
 *       ((y0+y1)+(y2+y3))+((y4+y5)+(y6+y7)),
 *       the recursive-halving order of reduce_intra_reduce_scatter_gather.c;
 *   MPIR_HIP_ORDER_CHAIN (1 <= n <= 64): ((y0+y1)+y2)+..., the pairwise order
 *       of reduce_scatter_block_intra_pairwise.c.
 * All buffers device-resident on one device; outbuf may alias inbufs[0]. */
#define MPIR_HIP_ORDER_TREE  0
#define MPIR_HIP_ORDER_CHAIN 1
int MPIR_Hip_combine(const void *const *inbufs, int n, void *outbuf, uint64_t count, int op, int elem,
                     int order, void *hip_stream, int sync);

/* Flags for the calling thread's later MPIR_Hip_combine calls; returns the
 * previous flags.  MPIR_HIP_COMBINE_UNCAPPED: the fused folds run without the
 * LDS reservation that caps a CU at one (P >= 5) or three (P = 3, 4) of their
 * workgroups -- for a fold that overlaps other work on the device (the
 * collectives' pipelined folds beside RCCL's transfers). */
#define MPIR_HIP_COMBINE_UNCAPPED 1
int MPIR_Hip_combine_set_flags(int flags);

/* byte size of an element class (0 if unknown) */
size_t MPIR_Hip_elem_size(int elem);
/* 1 if a kernel exists for (op, elem) */
int MPIR_Hip_has_kernel(int op, int elem);
/* 1 if p is device-accessible memory (hipMalloc / managed), 0 otherwise */
int MPIR_Hip_is_device_ptr(const void *p);
/* how a reduction of `bytes` sees p: 0 pageable host memory, 1 device memory,
 * 2 pinned host memory (hipHostMalloc / hipHostRegister).  A call within the
 * mixed slot's and the host combine's limits (MPIR_Hip_mixed_max_bytes,
 * MPIR_Hip_host_max_bytes) may take this thread's kept verdict for p's page; a
 * larger one asks HIP again (pointer classification) */
int MPIR_Hip_pointer_kind(const void *p, uint64_t bytes);
/* synchronous copy between any two pointers (device/host in any mix) */
int MPIR_Hip_memcpy(void *dst, const void *src, size_t bytes);
/* last runtime error text for this thread ("" if none) */
const char *MPIR_Hip_error_string(void);
/* number of visible devices (0 if none / runtime unavailable) */
int MPIR_Hip_device_count(void);
/* per-thread contexts (streams, completion word, scratch) created so far; a
   context returns to a pool when its thread exits and is reused, so this stays
   at the peak number of threads calling at once (diagnostic) */
/* Largest operand (bytes) combined on the host when both operands are host
 * memory (MPIR_CVAR_REDUCE_LOCAL_HOST_MAX_KB; default no limit, 0 = always
 * stage through the GPU).  The setter changes it at run time (an MPI_T-style
 * cvar write; bench.py uses it to time the staging pipeline) and returns the
 * previous value. */
uint64_t MPIR_Hip_host_max_bytes(void);
uint64_t MPIR_Hip_set_host_max_bytes(uint64_t bytes);

/* Results of at most this many bytes are stored into the Infinity Cache (sc1)
 * for their next reader, larger ones bypass it (nt): MPIR_CVAR_REDUCE_LOCAL_KEEP_MB,
 * default 64 MiB.  The setter changes it at run time and returns the previous
 * value (bench.py reports config 2 both ways). */
uint64_t MPIR_Hip_set_keep_bytes(uint64_t bytes);
/* Results of at most `bytes` are stored nt whatever MPIR_Hip_set_keep_bytes says
 * (MPIR_CVAR_REDUCE_LOCAL_KEEP_MIN_MB, default 16 MiB: below it sc1 costs the
 * call more than its next reader gains); returns the previous value. */
uint64_t MPIR_Hip_set_keep_min_bytes(uint64_t bytes);

/* One operand host memory, the other on a device, at most this many bytes
 * (MPIR_CVAR_REDUCE_LOCAL_MIXED_MAX_KB, default 1 MiB): the host operand is
 * copied into the calling thread's pinned, device-mapped slot and the kernel
 * reads (writes) it there directly; larger calls use the staging pipeline. */
uint64_t MPIR_Hip_mixed_max_bytes(void);

/* Synchronous device-resident reductions completed through the direct AQL
 * dispatch (direct_dispatch.hip) so far in this process (0 with
 * MPIR_CVAR_REDUCE_LOCAL_DISPATCH=hip or where the path is unavailable). */
uint64_t MPIR_Hip_direct_dispatches(void);

/* Kernel timing of the direct dispatch: with profiling on, the CP's start /
 * end timestamps of each dispatch (as rocprofv3 reads them); the calling
 * thread's last direct dispatch in ns (0 if none or profiling off). */
void MPIR_Hip_direct_profile(int on);
uint64_t MPIR_Hip_direct_last_kernel_ns(void);

/* Direct-dispatch diagnostics: the device's state (0 not yet tried, 1 ready,
 * 2 ready with every kernarg write made visible by a flush read back before
 * the doorbell -- the queue's dispatch ids are not its packet indices, as
 * under a tool that intercepts queues such as rocprofv3 --kernel-trace;
 * -1..-12 the initialisation step that failed: properties, hsa_init, agents,
 * VRAM pool, HDP register, code-object file, code-object load, kernel
 * symbols, kernarg memory, queue, error word, and (-12) a code object built
 * from other sources than this library (MPIR_Hip_build_id); -20 disabled by
 * MPIR_CVAR_REDUCE_LOCAL_DISPATCH=hip), and the number of direct calls that
 * first synchronised with work reported pending on the legacy null stream. */
int MPIR_Hip_direct_state(int dev);
/* Initialise device `dev`'s direct path now -- its HSA queue, the device-only
 * code object, the kernarg slots, the dispatch-id probe (2-10 ms) -- rather
 * than inside the first synchronous call on that device; meant for MPI_Init
 * (Option 1).  Idempotent and thread-safe; returns
 * MPIR_Hip_direct_state(dev). */
int MPIR_Hip_direct_prepare(int dev);

/* The library's load-time default HSA_ALLOCATE_QUEUE_DEV_MEM=1 (AQL rings in
 * VRAM), applied on request: 1 set now, 0 the environment already holds a
 * value (kept), -1 the HSA runtime has started (too late, nothing done), -2 the
 * process runs other threads and threads_ok is 0.  The constructor applies it
 * with threads_ok 0; the Python package's load() with 1. */
int MPIR_Hip_default_rings_in_vram(int threads_ok);
/* With profiling on, the calling thread's last direct call on the system
 * clock, ns from entering the dispatch: doorbell rung, CP start, CP end,
 * completion seen by the host.  The CP's two stamps reach the system clock
 * through the runtime's translation, so they carry its offset (a few us at
 * most) and are two's-complement int64 values in the uint64 slots. */
void MPIR_Hip_direct_last_split(uint64_t out[4]);
uint64_t MPIR_Hip_direct_busy_skips(void);
/* Direct calls whose kernel arguments missed the kernarg cache (written into a
 * VRAM slot before the doorbell, with an HDP flush; read back under a queue-
 * intercepting tool). */
uint64_t MPIR_Hip_direct_kernarg_writes(void);
/* Test hook: with us > 0, a checked dispatch's kernarg write moves behind the
 * doorbell and is held back `us` microseconds, as if it had lost the race to
 * the CP; the dispatched workgroups wait for it
 * (tests/test_parity_gpu.py::test_direct_dispatch_preempted_writer,
 * tests/test_direct_timeout_gpu.py, tools/late_write_probe.py).  0, the
 * default: the write precedes the doorbell.  Returns the previous value. */
uint32_t MPIR_Hip_direct_test_write_delay_us(uint32_t us);
/* Test hook: the next probe of a newly created timestamped (profiled) queue
 * reports that dispatch ids are not packet indices, as under a tool that
 * intercepts the queue; the first profiled call then switches the device to
 * read-back flushes (MPIR_Hip_direct_state 2) and must still complete
 * (tests/test_direct_prepare_gpu.py). */
void MPIR_Hip_direct_test_fail_probe(void);
/* Where the synchronous call's host side runs relative to device `dev`
 * (diagnostic; bench.py records it per rank): out[0] the calling thread's CPU
 * (sched_getcpu), out[1] that CPU's NUMA node, out[2] the device's NUMA node
 * (its PCI function's sysfs numa_node), out[3] the node of the page holding
 * this thread's completion signal for dev, out[4] the node of the device's
 * error word; -1 where unknown or not yet created. */
void MPIR_Hip_direct_placement(int dev, int out[5]);
/* Where device dev's direct-path queue keeps its AQL ring (diagnostic): 1 device
 * memory (HSA_ALLOCATE_QUEUE_DEV_MEM=1, the library's default), 0 host memory,
 * -1 no queue yet / unknown. */
int MPIR_Hip_direct_ring_location(int dev);
int MPIR_Hip_thread_contexts(void);

/* The build id of this library: "src=<hash of csrc/ and include/> tiles=<hash
 * of the direct path's code object sources> git=<commit>[+dirty]" (Makefile),
 * so a run can show which sources its binaries came from. */
const char *MPIR_Hip_build_id(void);

/* Ranks of this job on this node, for sizing the host combine's threads: the
 * node's CPUs are shared by every local rank, and all of them reach the
 * combine of a host-buffer MPI_Allreduce together.  Inside libmpi the op layer
 * passes MPICH's node communicator size (mpich_glue.c) before its first
 * combine; otherwise MPI_LOCALNRANKS / MPIR_PIP_SIZE / LOCAL_WORLD_SIZE /
 * OMPI_COMM_WORLD_LOCAL_SIZE, else 1.  Takes effect if called before the first
 * host combine sizes the pool; returns the previous value (0 = unset). */
int MPIR_Hip_set_local_ranks(int n);
/* Threads one host combine uses, the caller included (1 = the caller alone):
 * this rank's share of the node's CPUs, at most 16, or
 * MPIR_CVAR_REDUCE_LOCAL_STAGE_THREADS.  Sizes the pool without starting it. */
int MPIR_Hip_host_threads(void);

#ifdef __cplusplus
}
#endif
#endif /* MPIR_HIP_REDUCE_H_INCLUDED */

/*
 * coll_trace.c -- TEST ONLY: one rank of the device collectives
 * (csrc/host/coll_hip.c, the product source, compiled unchanged) with the GPU
 * taken out: the HIP runtime calls coll_hip.c makes and the MPIR_Hip_* kernels
 * it launches are stand-ins defined here that move no data, and librccl is
 * tests/progs/rccl_stub.c (MPIR_TEST_RCCL_LIBRARY), which records every RCCL
 * call.  Device buffers are address ranges reserved with PROT_NONE: coll_hip.c
 * only passes them on, so configs 4 and 5 run at their full sizes in no memory.
 *
 *   coll_trace <rank> <size>   < plan
 * plan lines:  allreduce <count> <type> <op> <alg>
 *              reduce_scatter_block <recvcount> <type> <op> <alg>
 *              reduce <count> <type> <op> <alg> <root>
 *              scan <count> <type> <op> | exscan <count> <type> <op>
 *   type: f32 f16 f64 i32    op: sum max min    alg: auto ref rccl
 * tests/test_rccl_sequence_cpu.py runs N of these and matches their logs.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#include <hip/hip_runtime_api.h>

#include "mpi_reduce_local.h"
#include "mpir_hip_reduce.h"
#include "mpix_hip_coll.h"
#include "mpir_op_types.h"

static void note(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
static void note(const char *fmt, ...)
{
    static void (*fn)(const char *);
    char buf[256];
    va_list ap;
    if (!fn)
        *(void **) (&fn) = dlsym(RTLD_DEFAULT, "rccl_stub_note");
    if (!fn)
        return;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    fn(buf);
}

/* ---- a reserved, never-touched address range stands in for device memory */
static void *reserve(size_t bytes)
{
    void *p = mmap(NULL, bytes ? bytes : 1, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    return p == MAP_FAILED ? NULL : p;
}

/* ---- the HIP runtime calls of coll_hip.c */
hipError_t hipGetDevice(int *d) { *d = 0; return hipSuccess; }
hipError_t hipSetDevice(int d) { (void) d; return hipSuccess; }
hipError_t hipStreamCreate(hipStream_t *s) { *s = (hipStream_t) (uintptr_t) 0x5100; return hipSuccess; }
hipError_t hipStreamDestroy(hipStream_t s) { (void) s; return hipSuccess; }
hipError_t hipStreamSynchronize(hipStream_t s) { (void) s; return hipSuccess; }
hipError_t hipDeviceSynchronize(void) { return hipSuccess; }
hipError_t hipStreamWaitEvent(hipStream_t s, hipEvent_t e, unsigned int f) { (void) s; (void) e; (void) f; return hipSuccess; }
hipError_t hipEventCreateWithFlags(hipEvent_t *e, unsigned f) { (void) f; *e = (hipEvent_t) (uintptr_t) 0xe0; return hipSuccess; }
hipError_t hipEventRecord(hipEvent_t e, hipStream_t s) { (void) e; (void) s; return hipSuccess; }
hipError_t hipEventDestroy(hipEvent_t e) { (void) e; return hipSuccess; }
const char *hipGetErrorString(hipError_t e) { (void) e; return "stand-in"; }
hipError_t hipMalloc(void **p, size_t bytes)
{
    *p = reserve(bytes);
    note("malloc %zu", bytes);
    return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipFree(void *p) { (void) p; return hipSuccess; }    /* (the reservation is left: tiny, short-lived) */
hipError_t hipMemcpyAsync(void *dst, const void *src, size_t bytes, hipMemcpyKind k, hipStream_t s)
{
    (void) dst;
    (void) src;
    (void) k;
    (void) s;
    note("memcpy %zu", bytes);
    return hipSuccess;
}

/* ---- the shim's kernels (mpir_hip_reduce.h) */
static const size_t elem_size[MPIR_HIP_NELEMS] = {
    0, 1, 1, 2, 2, 4, 4, 8, 8, 2, 4, 8, 8, 16, 8, 8, 16, 8, 16, 16, 32, 32,
};
size_t MPIR_Hip_elem_size(int elem) { return elem > 0 && elem < MPIR_HIP_NELEMS ? elem_size[elem] : 0; }
int MPIR_Hip_has_kernel(int op, int elem) { (void) op; return elem > 0 && elem < MPIR_HIP_NELEMS; }
const char *MPIR_Hip_error_string(void) { return ""; }
int MPIR_Hip_is_device_ptr(const void *p) { (void) p; return 1; }
int MPIR_Hip_combine_set_flags(int flags)
{
    static int cur;
    const int prev = cur;
    cur = flags;
    return prev;
}
int MPIR_Hip_memcpy(void *d, const void *s, size_t n) { (void) d; (void) s; (void) n; return MPIR_HIP_OK; }
int MPIR_Hip_reduce(const void *in, void *io, uint64_t count, int op, int elem, void *s, int sync)
{
    (void) in; (void) io; (void) s; (void) sync;
    note("reduce_local %llu %d %d", (unsigned long long) count, op, elem);
    return MPIR_HIP_OK;
}
int MPIR_Hip_combine(const void *const *ins, int n, void *out, uint64_t count, int op, int elem, int order, void *s,
                     int sync)
{
    (void) ins; (void) out; (void) s; (void) sync;
    note("combine %d %llu %d %d %s", n, (unsigned long long) count, op, elem,
         order == MPIR_HIP_ORDER_TREE ? "tree" : "chain");
    return MPIR_HIP_OK;
}

static int type_of(const char *t)
{
    if (!strcmp(t, "f32")) return MPI_FLOAT;
    if (!strcmp(t, "f16")) return MPIX_C_FLOAT16;
    if (!strcmp(t, "f64")) return MPI_DOUBLE;
    if (!strcmp(t, "i32")) return MPI_INT;
    return MPI_DATATYPE_NULL;
}

static int op_of(const char *o)
{
    if (!strcmp(o, "sum")) return MPI_SUM;
    if (!strcmp(o, "max")) return MPI_MAX;
    if (!strcmp(o, "min")) return MPI_MIN;
    return MPI_OP_NULL;
}

static int alg_of(const char *a)
{
    if (!strcmp(a, "ref")) return MPIX_HIP_ALG_REFERENCE_ORDER;
    if (!strcmp(a, "rccl")) return MPIX_HIP_ALG_RCCL;
    return MPIX_HIP_ALG_AUTO;
}

int main(int argc, char **argv)
{
    char id[MPIX_HIP_UNIQUE_ID_BYTES], line[256];
    MPIX_Hip_comm comm = NULL;
    int rank, size, rc, n = 0;
    if (argc != 3)
        return 2;
    rank = atoi(argv[1]);
    size = atoi(argv[2]);
    MPIX_Reduce_local_set_errhandler(MPI_ERRORS_RETURN);
    if ((rc = MPIX_Hip_comm_get_unique_id(id)) || (rc = MPIX_Hip_comm_create(id, size, rank, &comm))) {
        fprintf(stderr, "comm: %d\n", rc);
        return 3;
    }
    while (fgets(line, sizeof line, stdin)) {
        char what[64], ty[16], op[16], alg[16];
        long long count;
        int root = 0, k = sscanf(line, "%63s %lld %15s %15s %15s %d", what, &count, ty, op, alg, &root);
        size_t esz, bytes, sbytes;
        void *sb, *rb = NULL;
        if (k < 4)
            continue;
        esz = (size_t) MPIR_Hip_elem_size(MPIR_Op_resolve_elem(op_of(op) & 0xf, type_of(ty)));
        bytes = (size_t) count * (esz ? esz : 8);
        sbytes = !strcmp(what, "reduce_scatter_block") ? bytes * (size_t) size : bytes;
        note("call %d %s", n++, what);
        if (!strcmp(what, "allreduce")) {
            sb = reserve(bytes);
            rb = reserve(bytes);
            rc = MPIX_Allreduce_hip(sb, rb, (int) count, type_of(ty), op_of(op), comm, alg_of(alg), NULL);
        } else if (!strcmp(what, "reduce_scatter_block")) {
            sb = reserve(sbytes);
            rb = reserve(bytes);
            rc = MPIX_Reduce_scatter_block_hip(sb, rb, (int) count, type_of(ty), op_of(op), comm, alg_of(alg), NULL);
        } else if (!strcmp(what, "reduce")) {
            sb = reserve(bytes);
            rb = rank == root ? reserve(bytes) : NULL;
            rc = MPIX_Reduce_hip(sb, rb, (int) count, type_of(ty), op_of(op), root, comm, alg_of(alg), NULL);
        } else if (!strcmp(what, "scan") || !strcmp(what, "exscan")) {
            sb = reserve(bytes);
            rb = reserve(bytes);
            rc = (what[0] == 's' ? MPIX_Scan_hip : MPIX_Exscan_hip)(sb, rb, (int) count, type_of(ty), op_of(op), comm,
                                                                   alg_of(k >= 5 ? alg : "auto"), NULL);
        } else {
            fprintf(stderr, "unknown plan line: %s", line);
            return 4;
        }
        munmap(sb, sbytes ? sbytes : 1);
        if (rb)
            munmap(rb, bytes ? bytes : 1);
        if (rc) {
            char msg[512];
            int len = 0;
            MPI_Error_string(rc, msg, &len);
            fprintf(stderr, "%s failed: %s\n", what, msg);
            return 5;
        }
    }
    MPIX_Hip_comm_free(&comm);
    return 0;
}

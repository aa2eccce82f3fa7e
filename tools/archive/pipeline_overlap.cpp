// pipeline_overlap.cpp -- one GPU's view of the collectives' pipelined
// schedule (coll_hip.c exchange_fold_pipelined): chunk k's
// fold running while chunk k+1's transfer runs, against the two one after the
// other, with the fold's LDS cap on and off.
//
//   hipcc -O2 -std=c++17 -Iinclude -o tools/archive/pipeline_overlap tools/archive/pipeline_overlap.cpp \
//         -Lmpich-pip_amd/lib -lmpir_hip -Wl,-rpath,$PWD/mpich-pip_amd/lib -lrccl
//   tools/archive/pipeline_overlap [reps = 15]
//
// The transfer stand-in is RCCL's own kernel: a one-rank ncclAllReduce, fp16
// SUM, over the (P - 1) chunks a rank receives in one group (7 x 32 MiB at
// config 5's 8 ranks: 224 MiB read and written); the fold is the product's
// (MPIR_Hip_combine, CHAIN8 fp16 over 8 chunks of 32 MiB in a staging slab).
// Per case, K = 4 chunks (config 5's 128 MiB blocks in 32 MiB chunks), HIP
// events around the whole sequence, median over reps:
//   transfers only / folds only       K of each back to back on one stream
//   serial                            transfer k, fold k, transfer k+1, ... on one stream
//   overlapped                        transfers on stream B; fold k on stream A after
//                                     transfer k (an event), as the pipeline runs them
// each with the fold capped (the library's default outside the pipeline) and
// uncapped (MPIR_HIP_COMBINE_UNCAPPED, what the pipeline uses).  On one GPU
// both streams draw on the same HBM, so this bounds what overlap gives when the
// transfer is a copy; over xGMI the transfer leaves the HBM mostly to the fold.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mpir_hip_reduce.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(2);} } while (0)
#define NK(x) do { ncclResult_t r_ = (x); if (r_ != ncclSuccess) { \
    fprintf(stderr, "RCCL %s at %s:%d\n", ncclGetErrorString(r_), __FILE__, __LINE__); exit(2);} } while (0)

constexpr int P = 8, K = 4;
constexpr size_t CHUNK = 32ull << 20;                 // bytes per operand per chunk
constexpr size_t STRIDE = 4 * CHUNK + 6400;           // staging slot of a 128 MiB block (coll_hip.c stage_stride)

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 15;
    CK(hipSetDevice(0));
    char *slab, *xin, *xout;
    CK(hipMalloc(&slab, (P + 1) * STRIDE));
    CK(hipMalloc(&xin, (P - 1) * CHUNK * K));
    CK(hipMalloc(&xout, (P - 1) * CHUNK * K));
    CK(hipMemset(slab, 0x11, (P + 1) * STRIDE));      // finite fp16 (0x1111)
    CK(hipMemset(xin, 0x22, (P - 1) * CHUNK * K));
    ncclUniqueId id;
    ncclComm_t comm;
    NK(ncclGetUniqueId(&id));
    NK(ncclCommInitRank(&comm, 1, id, 0));
    hipStream_t sa, sb;
    CK(hipStreamCreate(&sa));
    CK(hipStreamCreate(&sb));
    hipEvent_t e0, e1, xev[K];
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (auto &e : xev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    const size_t celems = CHUNK / 2;                  // fp16 elements per operand chunk
    auto transfer = [&](int k, hipStream_t s) {
        NK(ncclAllReduce(xin + (size_t)k * (P - 1) * CHUNK, xout + (size_t)k * (P - 1) * CHUNK,
                         (P - 1) * celems, ncclFloat16, ncclSum, comm, s));
    };
    auto fold = [&](int k, hipStream_t s) {
        const void *ys[P];
        for (int j = 0; j < P; ++j) ys[j] = slab + j * STRIDE + (size_t)k * CHUNK;
        if (MPIR_Hip_combine(ys, P, slab + P * STRIDE + (size_t)k * CHUNK, celems, MPIR_HIP_OP_SUM, MPIR_HIP_F16,
                             MPIR_HIP_ORDER_CHAIN, s, 0) != MPIR_HIP_OK) {
            fprintf(stderr, "combine failed\n");
            exit(3);
        }
    };
    enum { XFER, FOLD, SERIAL, OVERLAP };
    auto run = [&](int mode) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, sa));
        CK(hipStreamWaitEvent(sb, e0, 0));
        for (int k = 0; k < K; ++k) {
            switch (mode) {
            case XFER: transfer(k, sa); break;
            case FOLD: fold(k, sa); break;
            case SERIAL: transfer(k, sa); fold(k, sa); break;
            default:
                transfer(k, sb);
                CK(hipEventRecord(xev[k], sb));
                CK(hipStreamWaitEvent(sa, xev[k], 0));
                fold(k, sa);
            }
        }
        if (mode == OVERLAP) {
            CK(hipEventRecord(xev[0], sb));
            CK(hipStreamWaitEvent(sa, xev[0], 0));
        }
        CK(hipEventRecord(e1, sa));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return ms * 1e3;
    };
    const char *names[4] = {"transfers only", "folds only", "serial", "overlapped"};
    printf("K = %d chunks: transfer = one-rank ncclAllReduce fp16 over %d x 32 MiB, fold = CHAIN8 fp16 over 8 x 32 MiB\n",
           K, P - 1);
    for (int capped = 1; capped >= 0; --capped) {
        MPIR_Hip_combine_set_flags(capped ? 0 : MPIR_HIP_COMBINE_UNCAPPED);
        std::vector<double> us[4];
        for (int r = 0; r < reps + 1; ++r)
            for (int m = 0; m < 4; ++m) {
                const double t = run((m + r) % 4);
                if (r) us[(m + r) % 4].push_back(t);
            }
        printf("fold %s:\n", capped ? "capped (96 KiB LDS: one workgroup per CU)" : "uncapped (MPIR_HIP_COMBINE_UNCAPPED)");
        for (int m = 0; m < 4; ++m) {
            std::sort(us[m].begin(), us[m].end());
            printf("  %-16s median %8.1f us  (p10 %8.1f, p90 %8.1f)\n", names[m], us[m][us[m].size() / 2],
                   us[m][us[m].size() / 10], us[m][us[m].size() * 9 / 10]);
        }
    }
    NK(ncclCommDestroy(comm));
    return 0;
}

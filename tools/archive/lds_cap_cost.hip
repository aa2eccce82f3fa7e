// lds_cap_cost.hip -- what the fused folds' LDS reservation costs (or saves)
// other work on the GPU at the same time.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Impich-pip_amd/csrc/hip \
//         -o tools/archive/lds_cap_cost tools/archive/lds_cap_cost.hip -lrccl
//   tools/archive/lds_cap_cost
//
// The library launches the P = 8 fold (k_combine_multi<.., 8, .., 1, 1024>)
// with an unused 96 KiB dynamic LDS reservation: one 1024-thread workgroup per
// CU instead of two (reduce_kernels.hpp multi_cap_bytes).  While a run of such
// folds (config 5's CHAIN8 fp16 over 8 x 128 MiB, 40 launches on stream A)
// occupies the GPU, a "victim" runs 20 times on stream B, each bracketed by
// HIP events; its mean is compared with the victim alone, for the fold with
// and without the reservation:
//   tile      the two-operand tile, fp32 SUM over 64 MiB (no LDS)
//   lds64     a copy staged through 64 KiB of LDS per 256-thread workgroup
//             (an LDS-heavy kernel: a GEMM's tiles, an RCCL-sized buffer)
//   rccl      a one-rank RCCL all_reduce, fp32 SUM, 64 MiB (RCCL's own kernel)
// The fold run's own mean launch time under each victim is reported too.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "reduce_kernels.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(2);} } while (0)
#define NK(x) do { ncclResult_t r_ = (x); if (r_ != ncclSuccess) { \
    fprintf(stderr, "RCCL %s at %s:%d\n", ncclGetErrorString(r_), __FILE__, __LINE__); exit(2);} } while (0)

namespace mpir_hip {
uint64_t keep_bytes() { return kKeepBytes; }
uint64_t keep_for(uint64_t vbytes) { return vbytes <= keep_bytes() ? vbytes : 0; }
bool multi_uncapped() { return false; }
}
using namespace mpir_hip;

__global__ __launch_bounds__(kThreads) void k_tile(const char *in, char *io, uint64_t vbytes) {
    reduce_tile<OpSum, float>(in, io, blockIdx.x, vbytes, 0);
}

// 64 KiB of LDS per workgroup: 256 threads copy 64 KiB through it
__global__ __launch_bounds__(kThreads) void k_lds64(const u32x4 *src, u32x4 *dst, uint64_t n16) {
    extern __shared__ u32x4 lds[];
    const uint64_t base = (uint64_t)blockIdx.x * 4096;
    for (int i = threadIdx.x; i < 4096; i += kThreads)
        if (base + i < n16) lds[i] = src[base + i];
    __syncthreads();
    for (int i = threadIdx.x; i < 4096; i += kThreads)
        if (base + i < n16) dst[base + i] = lds[4095 - i];
}

__global__ void k_fill(uint16_t *p, uint64_t n, uint32_t seed) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        p[i] = (uint16_t)(x & 0xBFFF);
    }
}

int main() {
    CK(hipFuncSetAttribute((const void *)k_combine_multi<OpSum, f16, 8, false, 1, 1024>,
                           hipFuncAttributeMaxDynamicSharedMemorySize, 96 << 10));
    CK(hipFuncSetAttribute((const void *)k_lds64, hipFuncAttributeMaxDynamicSharedMemorySize, 64 << 10));
    const uint64_t block = 128ull << 20, stride = block + 4352, setbytes = 8 * stride + block;
    std::vector<char *> sets(2);
    for (auto &p : sets) {
        CK(hipMalloc(&p, setbytes));
        k_fill<<<4096, 256>>>((uint16_t *)p, setbytes / 2, (uint32_t)(uintptr_t)p);
    }
    const uint64_t vb = 64ull << 20;
    char *vin, *vio;
    CK(hipMalloc(&vin, vb));
    CK(hipMalloc(&vio, vb));
    k_fill<<<4096, 256>>>((uint16_t *)vin, vb / 2, 3);
    k_fill<<<4096, 256>>>((uint16_t *)vio, vb / 2, 4);
    CK(hipDeviceSynchronize());
    hipStream_t sa, sb;
    CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    ncclComm_t comm;
    ncclUniqueId id;
    NK(ncclGetUniqueId(&id));
    NK(ncclCommInitRank(&comm, 1, id, 0));

    auto fold = [&](int k, bool cap) {
        MultiArgs a{};
        char *b = sets[k & 1];
        for (int j = 0; j < 8; ++j) a.in[j] = b + j * stride;
        a.out = b + 8 * stride;
        a.vbytes = block;
        a.keep = keep_for(block);
        hipLaunchKernelGGL((k_combine_multi<OpSum, f16, 8, false, 1, 1024>), dim3((unsigned)(block / 16384)),
                           dim3(1024), cap ? (96 << 10) : 0, sa, a);
    };
    auto victim = [&](int v) {
        if (v == 0)
            hipLaunchKernelGGL(k_tile, dim3((unsigned)(vb / kTileBytes)), dim3(kThreads), 0, sb, vin, vio, vb);
        else if (v == 1)
            hipLaunchKernelGGL(k_lds64, dim3((unsigned)(vb / 65536)), dim3(kThreads), 64 << 10, sb,
                               (const u32x4 *)vin, (u32x4 *)vio, vb / 16);
        else
            NK(ncclAllReduce(vin, vio, vb / 4, ncclFloat, ncclSum, comm, sb));
    };
    const char *vname[3] = {"tile fp32 64 MiB", "lds64 copy 64 MiB", "rccl all_reduce 1 rank 64 MiB"};
    const int KV = 20, KA = 40, ROUNDS = 5;
    std::vector<hipEvent_t> ev(2 * std::max(KV, KA));
    for (auto &e : ev) CK(hipEventCreate(&e));
    auto victim_us = [&](int v) {
        for (int i = 0; i < KV; ++i) {
            CK(hipEventRecord(ev[2 * i], sb));
            victim(v);
            CK(hipEventRecord(ev[2 * i + 1], sb));
        }
    };
    auto mean_of = [&](int n) {
        double s = 0;
        for (int i = 0; i < n; ++i) {
            float ms = 0;
            CK(hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]));
            s += ms * 1e3;
        }
        return s / n;
    };
    for (int v = 0; v < 3; ++v) victim(v);
    CK(hipDeviceSynchronize());
    printf("fold: CHAIN8 fp16 SUM 8 x 128 MiB on stream A (%d launches back to back); victim on stream B "
           "(%d launches, HIP events); medians of %d rounds\n", KA, KV, ROUNDS);
    for (int v = 0; v < 3; ++v) {
        std::vector<double> alone, with_cap, no_cap, fold_cap, fold_nocap;
        for (int r = 0; r < ROUNDS; ++r) {
            victim_us(v);
            CK(hipStreamSynchronize(sb));
            alone.push_back(mean_of(KV));
            for (int cap = 1; cap >= 0; --cap) {
                hipEvent_t f0, f1;
                CK(hipEventCreate(&f0));
                CK(hipEventCreate(&f1));
                CK(hipEventRecord(f0, sa));
                for (int k = 0; k < KA; ++k) fold(k, cap);
                CK(hipEventRecord(f1, sa));
                victim_us(v);           // starts while the folds run (they take ~8 ms)
                CK(hipStreamSynchronize(sb));
                CK(hipStreamSynchronize(sa));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, f0, f1));
                (cap ? with_cap : no_cap).push_back(mean_of(KV));
                (cap ? fold_cap : fold_nocap).push_back(ms * 1e3 / KA);
                CK(hipEventDestroy(f0));
                CK(hipEventDestroy(f1));
            }
        }
        auto med = [](std::vector<double> x) { std::sort(x.begin(), x.end()); return x[x.size() / 2]; };
        printf("%-30s victim alone %8.2f us | beside capped fold %8.2f us (fold %7.2f us) | beside uncapped fold "
               "%8.2f us (fold %7.2f us)\n", vname[v], med(alone), med(with_cap), med(fold_cap), med(no_cap),
               med(fold_nocap));
    }
    NK(ncclCommDestroy(comm));
    return 0;
}

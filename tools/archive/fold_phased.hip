// fold_phased.hip -- does the 8-operand fold lose its ~6 points to the DRAM's
// read/write turnarounds?  (HISTORY.md, "Fused-fold experiments", round 5.)
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -Impich-pip_amd/csrc/hip -o tools/archive/fold_phased tools/archive/fold_phased.hip
//   tools/archive/fold_phased [rounds = 10]
//
// The product's fold mixes its eight read streams with its write stream all
// the time.  Here one workgroup per CU (1024 threads) folds K tiles per phase
// into registers -- reads only, chip-wide -- then every workgroup stores its K
// results -- writes only -- so the HBM sees long read phases and long write
// phases instead of a steady 8:1 mix.  The phases are aligned across the grid
// by a SOFT barrier: a workgroup counts in with one atomic and polls the count
// at most `spin` times before it goes on regardless.  The barrier orders no data
// (every workgroup writes only its own tiles, computed from its own reads), so a
// workgroup that gives up waiting -- say another kernel holds some CUs and part of
// the grid is not resident -- still produces the right bytes; it only loses the
// alignment.  Every output is compared bit for bit with the library's kernel.
// Cases: config 5's CHAIN8 fp16 SUM over 8 x 128 MiB and config 4's TREE8 fp32
// SUM over 8 x 32 MiB, operands at the collective's staging stride; HIP events
// around batches of back-to-back launches over rotating operand sets, variants
// alternated.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "reduce_kernels.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(2);} } while (0)

namespace mpir_hip {
uint64_t keep_bytes() { return kKeepBytes; }
uint64_t keep_for(uint64_t vbytes) { return vbytes <= keep_bytes() ? vbytes : 0; }
bool multi_uncapped() { return false; }
}
using namespace mpir_hip;

constexpr int TH = 1024;
constexpr uint32_t kTile = TH * 16;     // 16 KiB per operand per tile, as the product's P = 8 shape

// count in, then poll until `target` workgroups have, at most `spin` polls
__device__ __forceinline__ void soft_barrier(unsigned *ctr, unsigned target, unsigned spin, unsigned *timeouts) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned n = 0;
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target && ++n < spin)
            __builtin_amdgcn_s_sleep(1);
        if (n >= spin) __hip_atomic_fetch_add(timeouts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
}

// grid = G workgroups (one per CU); tiles of phase p: p*G*K + k*G + blockIdx.x
template <class T, bool TREE, int K>
__global__ __launch_bounds__(TH) void k_fold_phased(MultiArgs a, unsigned ntiles, unsigned *ctr, unsigned base,
                                                    unsigned spin, unsigned *timeouts) {
    const unsigned G = gridDim.x;
    const int t = (int)threadIdx.x;
    const int wb = (t >> 6) * 1024 + (t & 63) * 16;
    const unsigned phases = (ntiles + G * K - 1) / (G * K);
    unsigned target = base;
    for (unsigned p = 0; p < phases; ++p) {
        u32x4 res[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const unsigned tile = p * G * K + (unsigned)k * G + blockIdx.x;
            u32x4 x[8];
            if (tile < ntiles) {
                const uint64_t off = (uint64_t)tile * kTile;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(a.in[j] + off), 0, kTile, 0x00020000);
                    x[j] = __builtin_amdgcn_raw_buffer_load_b128(r, wb, 0, kCachePolicyNT);
                    if (j == 3) issue_gap();
                }
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) x[j] = u32x4{0, 0, 0, 0};
            }
            Pack16<T> pk[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) pk[j] = __builtin_bit_cast(Pack16<T>, x[j]);
            Pack16<T> r;
#pragma unroll
            for (int e = 0; e < (int)(16 / sizeof(T)); ++e) {
                T v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = pk[j].e[e];
                r.e[e] = fold_fast<OpSum, T, 8, TREE>(v);
            }
            res[k] = __builtin_bit_cast(u32x4, r);
        }
        target += G;
        soft_barrier(ctr, target, spin, timeouts);          // every workgroup's reads of the phase done
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const unsigned tile = p * G * K + (unsigned)k * G + blockIdx.x;
            if (tile < ntiles) {
                const uint64_t off = (uint64_t)tile * kTile;
                __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void *)(a.out + off), 0, kTile, 0x00020000);
                store16(res[k], ro, wb, keep_tile(off, a.vbytes, a.keep));
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        target += G;
        soft_barrier(ctr, target, spin, timeouts);          // and its writes
    }
}

__global__ void k_fill(uint16_t *p, uint64_t n, uint32_t seed, int f16) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        p[i] = f16 ? (uint16_t)(x & 0xBFFF) : (uint16_t)((i & 1) ? ((x & 0x803F) | 0x3E00) : x);
    }
}

struct Case {
    const char *name;
    uint64_t block;
    bool f16;
};

template <class T, bool TREE>
void set_attrs() {
    CK(hipFuncSetAttribute((const void *)k_combine_multi<OpSum, T, 8, TREE, 1, 1024>,
                           hipFuncAttributeMaxDynamicSharedMemorySize, 96 << 10));
    CK(hipFuncSetAttribute((const void *)k_fold_phased<T, TREE, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 << 10));
    CK(hipFuncSetAttribute((const void *)k_fold_phased<T, TREE, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 << 10));
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 10;
    set_attrs<f16, false>();
    set_attrs<float, true>();
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    unsigned *ctr, *timeouts;
    CK(hipMalloc(&ctr, 256));
    CK(hipMalloc(&timeouts, 256));
    CK(hipMemset(ctr, 0, 256));
    CK(hipMemset(timeouts, 0, 256));
    unsigned arrivals = 0;      // the counter's value after every launch so far (never reset)
    const unsigned spin = 1u << 14;
    const Case cases[] = {{"config5 CHAIN8 fp16 8 x 128 MiB", 128ull << 20, true},
                          {"config4 TREE8 fp32 8 x 32 MiB", 32ull << 20, false}};
    const char *vname[3] = {"library (1024 x 1, 1 / CU)", "phased K = 8", "phased K = 4"};
    for (const Case &c : cases) {
        const uint64_t stride = c.block + 4352, setbytes = 8 * stride + c.block;
        const int nsets = (int)std::max<uint64_t>(3, (3ull << 30) / setbytes + 1);
        std::vector<char *> sets(nsets);
        for (auto &p : sets) {
            CK(hipMalloc(&p, setbytes));
            k_fill<<<4096, 256>>>((uint16_t *)p, setbytes / 2, (uint32_t)(uintptr_t)p, c.f16);
        }
        CK(hipDeviceSynchronize());
        const unsigned ntiles = (unsigned)(c.block / kTile);
        auto args = [&](int k) {
            MultiArgs a{};
            for (int j = 0; j < 8; ++j) a.in[j] = sets[k % nsets] + j * stride;
            a.out = sets[k % nsets] + 8 * stride;
            a.vbytes = c.block;
            a.keep = keep_for(c.block);
            return a;
        };
        auto run = [&](int k, int v) {
            const MultiArgs a = args(k);
            if (v == 0) {
                if (c.f16) hipLaunchKernelGGL((k_combine_multi<OpSum, f16, 8, false, 1, 1024>), dim3(ntiles), dim3(TH), 96 << 10, s, a);
                else hipLaunchKernelGGL((k_combine_multi<OpSum, float, 8, true, 1, 1024>), dim3(ntiles), dim3(TH), 96 << 10, s, a);
                return;
            }
            const int K = v == 1 ? 8 : 4;
            const unsigned phases = (ntiles + ncu * K - 1) / (ncu * K);
            const unsigned base = arrivals;
            arrivals += 2u * phases * (unsigned)ncu;
            if (c.f16) {
                if (K == 8) hipLaunchKernelGGL((k_fold_phased<f16, false, 8>), dim3(ncu), dim3(TH), 96 << 10, s, a, ntiles, ctr, base, spin, timeouts);
                else hipLaunchKernelGGL((k_fold_phased<f16, false, 4>), dim3(ncu), dim3(TH), 96 << 10, s, a, ntiles, ctr, base, spin, timeouts);
            } else {
                if (K == 8) hipLaunchKernelGGL((k_fold_phased<float, true, 8>), dim3(ncu), dim3(TH), 96 << 10, s, a, ntiles, ctr, base, spin, timeouts);
                else hipLaunchKernelGGL((k_fold_phased<float, true, 4>), dim3(ncu), dim3(TH), 96 << 10, s, a, ntiles, ctr, base, spin, timeouts);
            }
        };
        std::vector<char> h0(c.block), h1(c.block);
        run(0, 0);
        CK(hipMemcpyAsync(h0.data(), args(0).out, c.block, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        bool same = true;
        for (int v = 1; v < 3; ++v) {
            CK(hipMemsetAsync(args(0).out, 0, c.block, s));
            run(0, v);
            CK(hipMemcpyAsync(h1.data(), args(0).out, c.block, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            const bool eq = memcmp(h0.data(), h1.data(), c.block) == 0;
            if (!eq) printf("  %s differs\n", vname[v]);
            same = same && eq;
        }
        std::vector<double> us[3];
        std::mt19937 rng(3);
        const int batch = 20;
        int k = 1;
        for (int r = 0; r < rounds + 1; ++r) {
            int order[3] = {0, 1, 2};
            std::shuffle(order, order + 3, rng);
            for (int v : order) {
                run(k++, v);
                CK(hipEventRecord(e0, s));
                for (int b = 0; b < batch; ++b) run(k++, v);
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r) us[v].push_back(ms * 1e3 / batch);
            }
        }
        unsigned to = 0;
        CK(hipMemcpy(&to, timeouts, 4, hipMemcpyDeviceToHost));
        const double bytes = 9.0 * c.block;
        printf("%s (%d sets, %d rounds x %d launches, grid %d for the phased kernels), outputs identical: %s, "
               "barrier timeouts so far %u\n", c.name, nsets, rounds, batch, ncu, same ? "yes" : "NO", to);
        for (int v = 0; v < 3; ++v) {
            std::sort(us[v].begin(), us[v].end());
            const double med = us[v][us[v].size() / 2];
            printf("  %-28s median %8.2f us  min %8.2f  frac of 8 TB/s %.4f\n", vname[v], med, us[v][0],
                   bytes / (med * 1e-6) / 8e12);
        }
        for (auto p : sets) CK(hipFree(p));
    }
    return 0;
}

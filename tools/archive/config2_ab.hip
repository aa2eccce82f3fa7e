// config2_ab.hip -- BASELINE config 2 (fp32 SUM, 64 MiB per operand) kernel
// variants, to find what costs the 64 MiB launch its last ~2 % against the
// 256 MiB one (ramp and drain: DESIGN.md §(d) "Config 2").  Every variant is
// the product's tile (csrc/hip/reduce_kernels.hpp reduce_tile: 16 KiB per
// operand per 256-thread workgroup, 8 x buffer_load_dwordx4 nt per lane, issue
// gap after each pair, grid on 16 KiB boundaries) except where named:
//   prod_sc1   the product as config 2 runs it (a result <= 64 MiB stored sc1)
//   prod_nt    the product with nt stores
//   prog_nt    progressive stores: pair u is combined and stored as soon as its
//              loads have returned (s_waitcnt vmcnt(6 - 2u)), nt
//   prog_sc1   the same with sc1 stores
//   first_nt   the first resident round (blockIdx < 2048) loads, combines and
//              stores one pair at a time; later workgroups as prod_nt
//   serial_nt  every workgroup one pair at a time, nt
// Launches rotate over 16 windows of a 2 GiB footprint (bench.py config2), so
// none finds its operands in the 256 MB Infinity Cache; variants interleave
// launch by launch.  HIP events per launch, medians; run under rocprofv3
// --kernel-trace for the CP's own durations (tools/config2_ab.sh).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Impich-pip_amd/csrc/hip \
//         -o tools/config2_ab tools/config2_ab.hip
//   tools/config2_ab [MiB per operand = 64] [launches per variant = 100] [set: nt | sc1 | all = nt]
// An sc1-stored result stays dirty in the Infinity Cache and is written back
// while LATER kernels run (store policy), which flatters
// sc1 variants interleaved with nt ones: the sets keep the policies apart.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "reduce_kernels.hpp"

using namespace mpir_hip;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ __launch_bounds__(kThreads) void prod_tile(const char *in, char *io, uint64_t vbytes, uint64_t keep) {
    reduce_tile<OpSum, float>(in, io, blockIdx.x, vbytes, keep);
}

__device__ __forceinline__ u32x4 add4(u32x4 a, u32x4 b) {
    float4 x = __builtin_bit_cast(float4, a), y = __builtin_bit_cast(float4, b);
    x.x += y.x; x.y += y.y; x.z += y.z; x.w += y.w;
    return __builtin_bit_cast(u32x4, x);
}

// MODE 0: progressive stores; 1: one pair at a time; 2: one pair at a time in
// the first resident round only
template <int MODE, int POLICY>
__global__ __launch_bounds__(kThreads) void var_tile(const char *in, char *io, uint64_t vbytes, uint32_t first) {
    const uint64_t tile = blockIdx.x;
    const int64_t start = (int64_t)(tile * kTileBytes) - (int64_t)tile_shift(io);
    const uint64_t lo = start > 0 ? (uint64_t)start : 0;
    if (lo >= vbytes) return;
    const uint64_t end = (uint64_t)(start + kTileBytes);
    const int nrec = (int)((end < vbytes ? end : vbytes) - lo);
    const int cut = (int)(lo - start);
    __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void *)(in + lo), 0, nrec, 0x00020000);
    __amdgpu_buffer_rsrc_t rio = __builtin_amdgcn_make_buffer_rsrc((void *)(io + lo), 0, nrec, 0x00020000);
    const int t = (int)threadIdx.x;
    const int wb = (t >> 6) * (kVecPerLane * 1024) + (t & 63) * 16 - cut;
    const bool serial = MODE == 1 || (MODE == 2 && blockIdx.x < first);
    if (serial) {
#pragma unroll
        for (int u = 0; u < kVecPerLane; ++u) {
            u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rio, wb + u * 1024, 0, kCachePolicyNT);
            u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(rin, wb + u * 1024, 0, kCachePolicyNT);
            __builtin_amdgcn_raw_buffer_store_b128(add4(a, b), rio, wb + u * 1024, 0, POLICY);
        }
        return;
    }
    u32x4 a[kVecPerLane], b[kVecPerLane];
#pragma unroll
    for (int u = 0; u < kVecPerLane; ++u) {
        a[u] = __builtin_amdgcn_raw_buffer_load_b128(rio, wb + u * 1024, 0, kCachePolicyNT);
        b[u] = __builtin_amdgcn_raw_buffer_load_b128(rin, wb + u * 1024, 0, kCachePolicyNT);
        if (u + 1 < kVecPerLane) issue_gap();
    }
    if (MODE == 0) {
        // (vmcnt counts the stores too; sched barriers keep each combine after its wait)
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_raw_buffer_store_b128(add4(a[0], b[0]), rio, wb, 0, POLICY);
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_raw_buffer_store_b128(add4(a[1], b[1]), rio, wb + 1024, 0, POLICY);
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_raw_buffer_store_b128(add4(a[2], b[2]), rio, wb + 2048, 0, POLICY);
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_raw_buffer_store_b128(add4(a[3], b[3]), rio, wb + 3072, 0, POLICY);
    } else {
#pragma unroll
        for (int u = 0; u < kVecPerLane; ++u)
            __builtin_amdgcn_raw_buffer_store_b128(add4(a[u], b[u]), rio, wb + u * 1024, 0, POLICY);
    }
}

int main(int argc, char **argv) {
    const size_t mib = argc > 1 ? strtoull(argv[1], 0, 10) : 64;
    const int per = argc > 2 ? atoi(argv[2]) : 100;
    const std::string set = argc > 3 ? argv[3] : "nt";
    const size_t bytes = mib << 20, big = 256ull << 20;
    const int nwin_per = (int)(big / bytes);
    std::vector<char *> A, B;
    for (int p = 0; p < 4; ++p) {
        char *a, *b;
        CK(hipMalloc(&a, big));
        CK(hipMalloc(&b, big));
        CK(hipMemset(a, 0x3c, big));
        CK(hipMemset(b, 0x3b, big));
        A.push_back(a);
        B.push_back(b);
    }
    struct Win { char *io; const char *in; };
    std::vector<Win> wins;
    for (int p = 0; p < 4; ++p)
        for (int j = 0; j < nwin_per; ++j) wins.push_back({A[p] + j * bytes, B[p] + j * bytes});
    const uint32_t groups = (uint32_t)tile_groups(wins[0].io, bytes);
    const uint32_t first = 256 * 8;
    const char *names[] = {"prod_sc1", "prod_nt", "prog_nt", "prog_sc1", "first_nt", "serial_nt"};
    const int NV = 6;
    std::vector<float> ms[NV];
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int w = 0;
    for (int it = 0; it < per + 5; ++it) {
        for (int v = 0; v < NV; ++v) {
            const bool sc1 = v == 0 || v == 3;
            if ((set == "nt" && sc1) || (set == "sc1" && !sc1)) continue;
            const Win &x = wins[w++ % wins.size()];
            CK(hipEventRecord(e0, 0));
            switch (v) {
            case 0: hipLaunchKernelGGL(prod_tile, dim3(groups), dim3(kThreads), 0, 0, x.in, x.io, bytes, bytes); break;
            case 1: hipLaunchKernelGGL(prod_tile, dim3(groups), dim3(kThreads), 0, 0, x.in, x.io, bytes, 0); break;
            case 2: hipLaunchKernelGGL((var_tile<0, kCachePolicyNT>), dim3(groups), dim3(kThreads), 0, 0, x.in, x.io, bytes, first); break;
            case 3: hipLaunchKernelGGL((var_tile<0, kCachePolicySC1>), dim3(groups), dim3(kThreads), 0, 0, x.in, x.io, bytes, first); break;
            case 4: hipLaunchKernelGGL((var_tile<2, kCachePolicyNT>), dim3(groups), dim3(kThreads), 0, 0, x.in, x.io, bytes, first); break;
            default: hipLaunchKernelGGL((var_tile<1, kCachePolicyNT>), dim3(groups), dim3(kThreads), 0, 0, x.in, x.io, bytes, first); break;
            }
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (it >= 5) ms[v].push_back(t);
        }
    }
    const double alg = 3.0 * bytes;
    for (int v = 0; v < NV; ++v) {
        if (ms[v].empty()) continue;
        std::sort(ms[v].begin(), ms[v].end());
        const double med = ms[v][ms[v].size() / 2] * 1e-3;
        printf("%-10s %4zu MiB  median %8.2f us  p10 %8.2f  p90 %8.2f  frac %.4f\n", names[v], mib, med * 1e6,
               ms[v][ms[v].size() / 10] * 1e3, ms[v][ms[v].size() * 9 / 10] * 1e3, alg / med / 8e12);
    }
    return 0;
}

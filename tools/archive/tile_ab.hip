// tile_ab.hip -- tile-size A/B for the MPI_Reduce_local kernel (fp32 SUM) at
// the BASELINE sizes: 16 / 64 MiB (config 2) / 256 MiB (configs 1-3) per operand.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -Impich-pip_amd/csrc/hip -o tools/tile_ab tools/tile_ab.hip
// Variant = (16-byte vectors per lane VPL, threads per WG); tile = VPL*TH*16 B
// per operand per workgroup.  Buffers rotate over windows totalling >= 1 GiB so
// no launch finds its operands in the Infinity Cache.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "reduce_kernels.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(2);} } while (0)

using namespace mpir_hip;

template <int VPL, int TH>
__global__ __launch_bounds__(TH) void k_tile_x(const char *in, char *io, uint64_t vbytes) {
    constexpr uint32_t tile = VPL * TH * 16;
    const uint64_t base = (uint64_t)blockIdx.x * tile;
    if (base >= vbytes) return;
    const uint64_t left = vbytes - base;
    const int nrec = (int)(left < tile ? left : tile);
    __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void *)(in + base), 0, nrec, 0x00020000);
    __amdgpu_buffer_rsrc_t rio = __builtin_amdgcn_make_buffer_rsrc((void *)(io + base), 0, nrec, 0x00020000);
    u32x4 a[VPL], b[VPL];
#pragma unroll
    for (int u = 0; u < VPL; ++u) {
        const int off = (u * TH + (int)threadIdx.x) * 16;
        a[u] = __builtin_amdgcn_raw_buffer_load_b128(rio, off, 0, kCachePolicyNT);
        b[u] = __builtin_amdgcn_raw_buffer_load_b128(rin, off, 0, kCachePolicyNT);
    }
#pragma unroll
    for (int u = 0; u < VPL; ++u) {
        const int off = (u * TH + (int)threadIdx.x) * 16;
        __builtin_amdgcn_raw_buffer_store_b128(combine16<OpSum, float>(a[u], b[u]), rio, off, 0, kCachePolicyNT);
    }
}

template <int VPL, int TH>
hipError_t launch_x(const void *in, void *io, uint64_t count, hipStream_t s) {
    const uint64_t vb = count * 4;
    constexpr uint32_t tile = VPL * TH * 16;
    hipLaunchKernelGGL((k_tile_x<VPL, TH>), dim3((unsigned)((vb + tile - 1) / tile)), dim3(TH), 0, s,
                       (const char *)in, (char *)io, vb);
    return hipGetLastError();
}

struct Var {
    std::string name;
    hipError_t (*fn)(const void *, void *, uint64_t, hipStream_t);
    std::vector<float> ms;
};

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 15;
    const size_t pool = 1536ull << 20;     // 1.5 GiB per side
    char *in, *io;
    CK(hipMalloc(&in, pool));
    CK(hipMalloc(&io, pool));
    CK(hipMemset(in, 0, pool));
    CK(hipMemset(io, 0, pool));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t sizes[] = {16u << 20, 64u << 20, 256u << 20};
    for (size_t bytes : sizes) {
        std::vector<Var> vs = {
            {"product (VPL4 T256)", &launch_reduce<OpSum, float>, {}},
            {"VPL1 T256 (4 KiB)", &launch_x<1, 256>, {}},
            {"VPL2 T256 (8 KiB)", &launch_x<2, 256>, {}},
            {"VPL4 T256 (16 KiB)", &launch_x<4, 256>, {}},
            {"VPL8 T256 (32 KiB)", &launch_x<8, 256>, {}},
            {"VPL2 T512 (16 KiB)", &launch_x<2, 512>, {}},
            {"VPL4 T512 (32 KiB)", &launch_x<4, 512>, {}},
            {"VPL1 T1024 (16 KiB)", &launch_x<1, 1024>, {}},
            {"VPL2 T1024 (32 KiB)", &launch_x<2, 1024>, {}},
        };
        const size_t nwin = pool / bytes;
        size_t w = 0;
        for (int r = -2; r < rounds; ++r)
            for (auto &v : vs) {
                const size_t off = (w++ % nwin) * bytes;
                CK(hipEventRecord(e0, st));
                CK(v.fn(in + off, io + off, bytes / 4, st));
                CK(hipEventRecord(e1, st));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r >= 0) v.ms.push_back(ms);
            }
        printf("fp32 SUM, %zu MiB per operand, %d interleaved rounds, %zu windows\n", bytes >> 20, rounds, nwin);
        for (auto &v : vs) {
            std::sort(v.ms.begin(), v.ms.end());
            const double med = v.ms[v.ms.size() / 2];
            const double gbs = 3.0 * bytes / (med * 1e-3) / 1e9;
            printf("  %-22s median %8.2f us  min %8.2f  %7.0f GB/s  frac %.3f\n", v.name.c_str(), med * 1e3,
                   v.ms[0] * 1e3, gbs, gbs / 8000.0);
        }
    }
    return 0;
}

// fused_channels.hip -- the launches behind DESIGN.md §(f) "Fused combine:
// channel counters": why the fused 8-operand combine (config 4's TREE8 fp32,
// 8 x 32 MiB -> 32 MiB) reaches ~0.75 of 8 TB/s while reading the same 8
// streams without the write reaches ~0.83.  Interleaved launches, operand sets
// rotated over a ~2.3 GiB footprint so nothing is found in the 256 MB Infinity
// Cache; run under rocprofv3 --pmc with the per-channel counters of
// tools/fused_channels.yaml (tools/fused_channels.sh), one pass per counter
// group, kernel durations from --kernel-trace in the same passes.
//   fused_nt   the product's k_combine_multi<SUM, float, 8, TREE> (launch_combine_p),
//              every store nt (the verdict's "all-nt" measurement)
//   fused_sc1  the same launch as the product issues it at 32 MiB (keep_for:
//              result stored sc1, written back from the Infinity Cache later)
//   ro8        the fused kernel's loads (same 1024-thread shape, same operand
//              buffers, nt), no stores: 8 read streams
//   tile2      the product's two-operand tile (reduce_tile, 2 reads + 1 write)
//              over the first operand pair, nt
//   pipe2/4    the fused kernel with NT tiles per workgroup at a grid stride
//              (tile b, b + G, ...: the tiles in flight stay one dense window),
//              the next tile's eight loads issued before this tile's store, so
//              a wave's store is acknowledged while its next loads are in
//              flight rather than at the end of its life; nt
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Impich-pip_amd/csrc/hip \
//         -o tools/fused_channels tools/fused_channels.hip
//   tools/fused_channels [rounds = 12]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "reduce_kernels.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(2);} } while (0)

namespace mpir_hip {
static uint64_t g_keep = 0;
uint64_t keep_for(uint64_t vbytes) { return vbytes <= g_keep ? vbytes : 0; }
bool multi_uncapped() { return false; }
}  // namespace mpir_hip

using namespace mpir_hip;

// k_combine_multi<.., U = 1, TH = 1024>'s load side exactly; the combine is an
// XOR whose result is written only if it matches a constant (practically never)
__global__ __launch_bounds__(1024) void k_ro8(MultiArgs a, uint32_t *sink) {
    constexpr uint32_t tile = 1024 * 16;
    const uint64_t base = (uint64_t)blockIdx.x * tile;
    if (base >= a.vbytes) return;
    const int t = (int)threadIdx.x;
    const int wb = (t >> 6) * 1024 + (t & 63) * 16;
    u32x4 x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(a.in[j] + base), 0, tile, 0x00020000);
        x[j] = __builtin_amdgcn_raw_buffer_load_b128(r, wb, 0, kCachePolicyNT);
        if ((j + 1) % 4 == 0 && j + 1 < 8) issue_gap();
    }
    u32x4 acc = x[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) acc ^= x[j];
    const uint32_t v = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (v == 0x9e3779b9u) sink[blockIdx.x & 1023] = v;
}

template <int NT>
__global__ __launch_bounds__(1024) void k_pipe_s(MultiArgs a) {
    constexpr uint32_t tile = 1024 * 16;
    const int t = (int)threadIdx.x;
    const int wb = (t >> 6) * 1024 + (t & 63) * 16;
    const uint64_t stride = (uint64_t)gridDim.x * tile;
    u32x4 x[2][8];
    auto load = [&](int buf, uint64_t base) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(a.in[j] + base), 0, tile, 0x00020000);
            x[buf][j] = __builtin_amdgcn_raw_buffer_load_b128(r, wb, 0, kCachePolicyNT);
            if ((j + 1) % 4 == 0 && j + 1 < 8) issue_gap();
        }
    };
    const uint64_t base0 = (uint64_t)blockIdx.x * tile;
    load(0, base0);
#pragma unroll
    for (int k = 0; k < NT; ++k) {
        const uint64_t base = base0 + (uint64_t)k * stride;
        if (k + 1 < NT) load((k + 1) & 1, base + stride);
        float v[8][4];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float4 f = __builtin_bit_cast(float4, x[k & 1][j]);
            v[j][0] = f.x; v[j][1] = f.y; v[j][2] = f.z; v[j][3] = f.w;
        }
        float4 res;
        float *rp = reinterpret_cast<float *>(&res);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float w[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) w[j] = v[j][e];
            rp[e] = fold_fast<OpSum, float, 8, true>(w);
        }
        __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void *)(a.out + base), 0, tile, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, res), ro, wb, 0, kCachePolicyNT);
    }
}

__global__ __launch_bounds__(kThreads) void k_tile2(const char *in, char *io, uint64_t vbytes) {
    reduce_tile<OpSum, float>(in, io, blockIdx.x, vbytes, 0);
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 12;
    const size_t bytes = 32u << 20;
    const int P = 8, NS = 8;   // 8 sets x 9 x 32 MiB = 2.25 GiB
    std::vector<char *> ins(P * NS), outs(NS);
    for (auto &p : ins) { CK(hipMalloc(&p, bytes)); CK(hipMemset(p, 0x3c, bytes)); }
    for (auto &p : outs) { CK(hipMalloc(&p, bytes)); CK(hipMemset(p, 0, bytes)); }
    uint32_t *sink;
    CK(hipMalloc(&sink, 4096 * 4));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    const uint32_t groups2 = (uint32_t)tile_groups(outs[0], bytes);
    int slot = 0;
    for (int r = -2; r < rounds; ++r) {
        for (int v = 0; v < 6; ++v) {
            const int s = slot++ % NS;
            const void *ptr[P];
            for (int j = 0; j < P; ++j) ptr[j] = ins[s * P + j];
            switch (v) {
            case 0: g_keep = 0; CK((launch_combine_p<OpSum, float, 8, true>(ptr, outs[s], bytes / 4, st))); break;
            case 1: g_keep = 64u << 20; CK((launch_combine_p<OpSum, float, 8, true>(ptr, outs[s], bytes / 4, st))); break;
            case 2: {
                MultiArgs a{};
                for (int j = 0; j < P; ++j) a.in[j] = static_cast<const char *>(ptr[j]);
                a.out = outs[s];
                a.vbytes = bytes;
                hipLaunchKernelGGL(k_ro8, dim3((unsigned)(bytes / (1024 * 16))), dim3(1024), 0, st, a, sink);
                CK(hipGetLastError());
                break;
            }
            case 4: case 5: {
                MultiArgs a{};
                for (int j = 0; j < P; ++j) a.in[j] = static_cast<const char *>(ptr[j]);
                a.out = outs[s];
                a.vbytes = bytes;
                const unsigned tiles = (unsigned)(bytes / (1024 * 16));   // 2048: divisible by 2 and 4
                if (v == 4) hipLaunchKernelGGL(k_pipe_s<2>, dim3(tiles / 2), dim3(1024), 0, st, a);
                else hipLaunchKernelGGL(k_pipe_s<4>, dim3(tiles / 4), dim3(1024), 0, st, a);
                CK(hipGetLastError());
                break;
            }
            default:
                hipLaunchKernelGGL(k_tile2, dim3(groups2), dim3(kThreads), 0, st, ins[s * P], outs[s], (uint64_t)bytes);
                CK(hipGetLastError());
            }
            CK(hipStreamSynchronize(st));
        }
    }
    printf("fused_channels: %d rounds x {fused_nt, fused_sc1, ro8, tile2, pipe2, pipe4}, 8 x 32 MiB, %d rotated sets\n", rounds, NS);
    return 0;
}

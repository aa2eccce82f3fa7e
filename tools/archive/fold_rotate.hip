// fold_rotate.hip -- the P = 8 fused fold with its operand reads rotated
// (DRAM row / bank conflicts between the eight operand
// streams at equal offsets?).  Three variants of one tile of 1024 threads x
// 1 vector (the library's P = 8 shape, one workgroup per CU), every output
// compared bit for bit with the library kernel's:
//   lib     k_combine_multi<OpSum, T, 8, TREE, 1, 1024> under the 96 KiB cap;
//   issue   each wave issues its eight operand loads starting at operand
//           (wave mod 8), so the waves of a tile open the operands in eight
//           different orders (96 KiB cap);
//   chunk   the verdict's form: wave w reads operand p's 1 KiB chunk
//           (w + p) mod 16 of the tile, so at equal issue slots the eight
//           reads of a tile are eight different column ranges; the chunks
//           meet in LDS (8 x 16 KiB, which also holds the CU to one
//           workgroup) and wave w folds and stores chunk w.
// Operands in one staging slab at coll_hip.c stage_stride (block + 4352 B, or
// + 6400 B for 96-192 MiB blocks), as the collectives lay them.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -Impich-pip_amd/csrc/hip -o tools/archive/fold_rotate tools/archive/fold_rotate.hip
//   tools/archive/fold_rotate [rounds = 9]
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

constexpr int P = 8, TH = 1024, WAVES = TH / 64;
constexpr uint32_t TILE = TH * 16;      // bytes per operand per tile

__global__ void k_fill(uint32_t *p, uint64_t n, uint32_t seed) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        p[i] = x & 0x3BFF3BFFu;      // finite in fp16 and fp32
    }
}

template <class T, bool TREE>
__device__ __forceinline__ u32x4 fold16(const u32x4 (&x)[P]) {
    Pack16<T> pk[P];
#pragma unroll
    for (int j = 0; j < P; ++j) pk[j] = __builtin_bit_cast(Pack16<T>, x[j]);
    Pack16<T> res;
#pragma unroll
    for (int k = 0; k < (int)(16 / sizeof(T)); ++k) {
        T v[P];
#pragma unroll
        for (int j = 0; j < P; ++j) v[j] = pk[j].e[k];
        res.e[k] = fold_fast<OpSum, T, P, TREE>(v);
    }
    return __builtin_bit_cast(u32x4, res);
}

// loads in the order R, R+1, ..., (mod P), an issue gap after every 4 (as the library)
template <int R>
__device__ __forceinline__ void loads_rot(const MultiArgs &a, uint64_t base, int nrec, int off, u32x4 (&x)[P]) {
#pragma unroll
    for (int i = 0; i < P; ++i) {
        const int j = (R + i) % P;
        __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(a.in[j] + base), 0, nrec, 0x00020000);
        x[j] = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kCachePolicyNT);
        if ((i + 1) % 4 == 0 && i + 1 < P) issue_gap();
    }
}

template <class T, bool TREE>
__global__ __launch_bounds__(TH) void k_issue_rot(MultiArgs a) {
    const uint64_t base = (uint64_t)blockIdx.x * TILE;
    if (base >= a.vbytes) return;
    const uint64_t left = a.vbytes - base;
    const int nrec = (int)(left < TILE ? left : TILE);
    const int t = (int)threadIdx.x, w = t >> 6;
    const int off = w * 1024 + (t & 63) * 16;
    u32x4 x[P];
    switch (w & 7) {       // wave-uniform
    case 0: loads_rot<0>(a, base, nrec, off, x); break;
    case 1: loads_rot<1>(a, base, nrec, off, x); break;
    case 2: loads_rot<2>(a, base, nrec, off, x); break;
    case 3: loads_rot<3>(a, base, nrec, off, x); break;
    case 4: loads_rot<4>(a, base, nrec, off, x); break;
    case 5: loads_rot<5>(a, base, nrec, off, x); break;
    case 6: loads_rot<6>(a, base, nrec, off, x); break;
    default: loads_rot<7>(a, base, nrec, off, x); break;
    }
    __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void *)(a.out + base), 0, nrec, 0x00020000);
    store16(fold16<T, TREE>(x), ro, off, keep_tile(base, a.vbytes, a.keep));
}

template <class T, bool TREE>
__global__ __launch_bounds__(TH) void k_chunk_rot(MultiArgs a) {
    extern __shared__ u32x4 lds[];        // [P][WAVES][64]
    const uint64_t base = (uint64_t)blockIdx.x * TILE;
    if (base >= a.vbytes) return;         // (uniform per workgroup)
    const uint64_t left = a.vbytes - base;
    const int nrec = (int)(left < TILE ? left : TILE);
    const int t = (int)threadIdx.x, w = t >> 6, l = t & 63;
    u32x4 x[P];
#pragma unroll
    for (int j = 0; j < P; ++j) {
        const int c = (w + j) & (WAVES - 1);
        __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(a.in[j] + base), 0, nrec, 0x00020000);
        x[j] = __builtin_amdgcn_raw_buffer_load_b128(r, c * 1024 + l * 16, 0, kCachePolicyNT);
        if ((j + 1) % 4 == 0 && j + 1 < P) issue_gap();
    }
#pragma unroll
    for (int j = 0; j < P; ++j) lds[(j * WAVES + ((w + j) & (WAVES - 1))) * 64 + l] = x[j];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < P; ++j) x[j] = lds[(j * WAVES + w) * 64 + l];
    __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void *)(a.out + base), 0, nrec, 0x00020000);
    store16(fold16<T, TREE>(x), ro, w * 1024 + l * 16, keep_tile(base, a.vbytes, a.keep));
}

size_t stage_stride(size_t bytes) {      // coll_hip.c
    size_t st = (bytes + 255) & ~(size_t)255;
    if (st >= ((size_t)96 << 20) && st < ((size_t)192 << 20)) return st + 6400;
    return st >= ((size_t)1 << 20) ? st + 4352 : st;
}

template <class T, bool TREE>
void run(int rounds, uint64_t block) {
    const size_t lds_chunk = (size_t)P * TILE;
    CK(hipFuncSetAttribute((const void *)k_combine_multi<OpSum, T, P, TREE, 1, TH>,
                           hipFuncAttributeMaxDynamicSharedMemorySize, 96 << 10));
    CK(hipFuncSetAttribute((const void *)k_issue_rot<T, TREE>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 << 10));
    CK(hipFuncSetAttribute((const void *)k_chunk_rot<T, TREE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)lds_chunk));
    const size_t stride = stage_stride(block);
    const int nsets = std::max<int>(2, (int)((3ull << 29) / ((P + 1) * block) + 1));
    std::vector<char *> slabs(nsets);
    for (auto &s : slabs) CK(hipMalloc(&s, (P + 1) * stride));
    for (int s = 0; s < nsets; ++s)
        for (int j = 0; j <= P; ++j) k_fill<<<2048, 256>>>((uint32_t *)(slabs[s] + j * stride), block / 4, 0x77u + 31u * (s * 9 + j));
    CK(hipDeviceSynchronize());
    auto args = [&](int s) {
        MultiArgs a{};
        for (int j = 0; j < P; ++j) a.in[j] = slabs[s] + j * stride;
        a.out = slabs[s] + P * stride;
        a.vbytes = block;
        a.keep = keep_for(block);
        return a;
    };
    const unsigned grid = (unsigned)((block + TILE - 1) / TILE);
    const char *names[3] = {"lib (96 KiB cap)", "issue order rotated by wave", "chunk rotated per operand (LDS)"};
    auto go = [&](int v, int s) {
        const MultiArgs a = args(s);
        if (v == 0) hipLaunchKernelGGL((k_combine_multi<OpSum, T, P, TREE, 1, TH>), dim3(grid), dim3(TH), 96 << 10, 0, a);
        else if (v == 1) hipLaunchKernelGGL((k_issue_rot<T, TREE>), dim3(grid), dim3(TH), 96 << 10, 0, a);
        else hipLaunchKernelGGL((k_chunk_rot<T, TREE>), dim3(grid), dim3(TH), lds_chunk, 0, a);
    };
    std::vector<char> want(block), got(block);
    int bad[3] = {};
    go(0, 0);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(want.data(), slabs[0] + P * stride, block, hipMemcpyDeviceToHost));
    for (int v = 1; v < 3; ++v) {
        CK(hipMemset(slabs[0] + P * stride, 0, block));
        go(v, 0);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got.data(), slabs[0] + P * stride, block, hipMemcpyDeviceToHost));
        bad[v] = memcmp(got.data(), want.data(), block) != 0;
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<double> us[3];
    std::mt19937 rng(7);
    const int batch = 10;
    int k = 0;
    for (int r = 0; r < rounds; ++r) {
        int order[3] = {0, 1, 2};
        std::shuffle(order, order + 3, rng);
        for (int v : order) {
            go(v, k++ % nsets);
            CK(hipEventRecord(e0, 0));
            for (int b = 0; b < batch; ++b) go(v, k++ % nsets);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r) us[v].push_back(ms * 1e3 / batch);
        }
    }
    printf("%s8 %s, 8 x %.0f MiB in a staging slab (stride +%zu B), %d sets\n", TREE ? "TREE" : "CHAIN",
           sizeof(T) == 2 ? "fp16" : "fp32", block / 1048576.0, stride - block, nsets);
    for (int v = 0; v < 3; ++v) {
        std::sort(us[v].begin(), us[v].end());
        const double med = us[v][us[v].size() / 2];
        printf("  %-34s median %8.2f us  frac of 8 TB/s %.4f  output %s\n", names[v], med,
               (P + 1.0) * block / (med * 1e-6) / 8e12, v == 0 ? "reference" : (bad[v] ? "DIFFERS" : "identical"));
    }
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    for (auto s : slabs) CK(hipFree(s));
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 9;
    run<f16, false>(rounds, 128ull << 20);     // config 5: CHAIN8 fp16, 8 x 128 MiB
    run<f16, false>(rounds, 32ull << 20);
    run<float, true>(rounds, 32ull << 20);     // config 4: TREE8 fp32, 8 x 32 MiB
    run<float, true>(rounds, 128ull << 20);
    return 0;
}

// kernel_ab.hip -- interleaved A/B timing of the product's reduce kernels
// (mpich-pip_amd/csrc/hip/reduce_kernels.hpp) on MI355X.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -Impich-pip_amd/csrc/hip -o tools/kernel_ab tools/kernel_ab.hip
//   ./tools/kernel_ab [MiB_per_operand=256] [rounds=20]
//
// Every variant runs once per round, rounds interleaved (guide §5.4 rule 24),
// buffers rotated over 3 pairs (> Infinity Cache).  Reports the median and
// min launch time and GB/s of algorithmic bytes (3 x operand bytes).  Also
// the op x dtype sweep of BASELINE config 3 (SUM/MAX/MIN/PROD x
// int32/int64/fp32/fp64 at 256 MiB).
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

// the pre-NaN-rule float add, for the A/B of the explicit x86 NaN rule
struct OpSumPlain {
    __device__ __forceinline__ float operator()(float a, float b) const { return a + b; }
};

// ---- experimental shapes (not the product) --------------------------------
__device__ __forceinline__ void ld_tile(const char *in, char *io, uint64_t vbytes, uint64_t t, u32x4 *a, u32x4 *b) {
    const uint64_t base = t * kTileBytes;
    const uint64_t left = vbytes - base;
    const int nrec = (int)(left < kTileBytes ? left : kTileBytes);
    __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void *)(in + base), 0, nrec, 0x00020000);
    __amdgpu_buffer_rsrc_t rio = __builtin_amdgcn_make_buffer_rsrc((void *)(io + base), 0, nrec, 0x00020000);
#pragma unroll
    for (int u = 0; u < kVecPerLane; ++u) {
        const int off = (u * kThreads + (int)threadIdx.x) * 16;
        a[u] = __builtin_amdgcn_raw_buffer_load_b128(rio, off, 0, kCachePolicyNT);
        b[u] = __builtin_amdgcn_raw_buffer_load_b128(rin, off, 0, kCachePolicyNT);
    }
}
__device__ __forceinline__ void st_tile(char *io, uint64_t vbytes, uint64_t t, const u32x4 *a, const u32x4 *b) {
    const uint64_t base = t * kTileBytes;
    const uint64_t left = vbytes - base;
    const int nrec = (int)(left < kTileBytes ? left : kTileBytes);
    __amdgpu_buffer_rsrc_t rio = __builtin_amdgcn_make_buffer_rsrc((void *)(io + base), 0, nrec, 0x00020000);
#pragma unroll
    for (int u = 0; u < kVecPerLane; ++u) {
        const int off = (u * kThreads + (int)threadIdx.x) * 16;
        __builtin_amdgcn_raw_buffer_store_b128(combine16<OpSum, float>(a[u], b[u]), rio, off, 0, kCachePolicyNT);
    }
}
// persistent + register double buffer: next tile's loads in flight while storing this one
__global__ __launch_bounds__(256) void k_pipe(const char *in, char *io, uint64_t vbytes, uint64_t ntiles) {
    uint64_t t = blockIdx.x;
    if (t >= ntiles) return;
    u32x4 a[kVecPerLane], b[kVecPerLane], a2[kVecPerLane], b2[kVecPerLane];
    ld_tile(in, io, vbytes, t, a, b);
    for (; t < ntiles; t += gridDim.x) {
        const uint64_t tn = t + gridDim.x;
        if (tn < ntiles) ld_tile(in, io, vbytes, tn, a2, b2);
        st_tile(io, vbytes, t, a, b);
#pragma unroll
        for (int u = 0; u < kVecPerLane; ++u) { a[u] = a2[u]; b[u] = b2[u]; }
    }
}
template <int GRID>
hipError_t launch_pipe(const void *in, void *io, uint64_t count, hipStream_t s) {
    uint64_t vbytes = count * 4, ntiles = (vbytes + kTileBytes - 1) / kTileBytes;
    hipLaunchKernelGGL(k_pipe, dim3(GRID), dim3(256), 0, s, (const char *)in, (char *)io, vbytes, ntiles);
    return hipGetLastError();
}
// two tiles per workgroup, second tile's loads issued before the first tile's stores
__global__ __launch_bounds__(256) void k_two(const char *in, char *io, uint64_t vbytes, uint64_t ntiles) {
    uint64_t t = 2 * (uint64_t)blockIdx.x;
    u32x4 a[kVecPerLane], b[kVecPerLane], a2[kVecPerLane], b2[kVecPerLane];
    ld_tile(in, io, vbytes, t, a, b);
    if (t + 1 < ntiles) ld_tile(in, io, vbytes, t + 1, a2, b2);
    st_tile(io, vbytes, t, a, b);
    if (t + 1 < ntiles) st_tile(io, vbytes, t + 1, a2, b2);
}
hipError_t launch_two(const void *in, void *io, uint64_t count, hipStream_t s) {
    uint64_t vbytes = count * 4, ntiles = (vbytes + kTileBytes - 1) / kTileBytes;
    hipLaunchKernelGGL(k_two, dim3((ntiles + 1) / 2), dim3(256), 0, s, (const char *)in, (char *)io, vbytes, ntiles);
    return hipGetLastError();
}

// plain adds with no NaN rule, for the A/B of the fused tree's fast path
struct OpSumPlainM {
    __device__ __forceinline__ float operator()(float a, float b) const { return a + b; }
};

struct Var {
    std::string name;
    size_t esz;
    hipError_t (*fn)(const void *, void *, uint64_t, hipStream_t);
    std::vector<float> ms;
};

int main(int argc, char **argv) {
    size_t mib = argc > 1 ? strtoull(argv[1], 0, 10) : 256;
    int rounds = argc > 2 ? atoi(argv[2]) : 20;
    size_t bytes = mib << 20;
    const int NS = 3;
    char *in[NS], *io[NS];
    for (int s = 0; s < NS; ++s) {
        CK(hipMalloc(&in[s], bytes));
        CK(hipMalloc(&io[s], bytes));
        // small positive values: finite under every op for many rounds
        std::vector<float> h(bytes / 4);
        for (size_t i = 0; i < h.size(); ++i) h[i] = 1.0f + (float)((i * 2654435761u) % 1024) * (1.0f / 1024);
        CK(hipMemcpy(in[s], h.data(), bytes, hipMemcpyHostToDevice));
        CK(hipMemcpy(io[s], h.data(), bytes, hipMemcpyHostToDevice));
    }
    std::vector<Var> vs = {
        {"SUM fp32", 4, &launch_reduce<OpSum, float>, {}},
        {"SUM fp32 plain add", 4, &launch_reduce<OpSumPlain, float>, {}},
        {"SUM fp16", 2, &launch_reduce<OpSum, f16>, {}},
        {"SUM fp64", 8, &launch_reduce<OpSum, double>, {}},
        {"PROD fp32", 4, &launch_reduce<OpProd, float>, {}},
        {"MAX fp32", 4, &launch_reduce<OpMax, float>, {}},
        {"SUM int32", 4, &launch_reduce<OpSum, int32_t>, {}},
        {"SUM cf32", 8, &launch_reduce<OpSum, cf32>, {}},
        {"PROD cf64", 16, &launch_reduce<OpProd, cf64>, {}},
        {"MAXLOC double_int", 16, &launch_reduce<OpMaxloc, pdoubleint>, {}},
        {"SUM fp32 (again)", 4, &launch_reduce<OpSum, float>, {}},
    };
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int slot = 0;
    for (int r = -2; r < rounds; ++r) {
        for (auto &v : vs) {
            int s = slot++ % NS;
            CK(hipEventRecord(e0, st));
            CK(v.fn(in[s], io[s], bytes / v.esz, st));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 0) v.ms.push_back(ms);
        }
    }
    // fused schedule combines: P = 8 operands of `bytes` each -> 1 output
    struct MVar { std::string name; size_t esz; hipError_t (*fn)(const void *const *, void *, uint64_t, hipStream_t); std::vector<float> ms; };
    std::vector<MVar> mvs = {
        {"TREE8 SUM fp32 U1 (product)", 4, &launch_combine_p<OpSum, float, 8, true>, {}},
        {"TREE8 SUM fp32 U2", 4, &launch_combine_pu<OpSum, float, 8, true, 2, 256>, {}},
        {"TREE8 SUM fp32 U4", 4, &launch_combine_pu<OpSum, float, 8, true, 4, 256>, {}},
        {"TREE8 SUM fp32 U1 plain", 4, &launch_combine_pu<OpSumPlainM, float, 8, true, 1, 256>, {}},
        {"CHAIN8 SUM fp16 U1 (product)", 2, &launch_combine_p<OpSum, f16, 8, false>, {}},
        {"CHAIN8 SUM fp16 U2", 2, &launch_combine_pu<OpSum, f16, 8, false, 2, 256>, {}},
        {"CHAIN8 SUM fp32 U1", 4, &launch_combine_p<OpSum, float, 8, false>, {}},
        {"TREE4 SUM fp32 U2 (product)", 4, &launch_combine_p<OpSum, float, 4, true>, {}},
        {"TREE2 SUM fp32 U4 (product)", 4, &launch_combine_p<OpSum, float, 2, true>, {}},
    };
    const int P = 8;
    char *mins[P];
    for (int j = 0; j < P; ++j) { CK(hipMalloc(&mins[j], bytes)); CK(hipMemcpy(mins[j], in[j % NS], bytes, hipMemcpyDeviceToDevice)); }
    const void *mptr[P];
    for (int j = 0; j < P; ++j) mptr[j] = mins[j];
    for (int r = -2; r < rounds; ++r) {
        for (auto &v : mvs) {
            int s = slot++ % NS;
            CK(hipEventRecord(e0, st));
            CK(v.fn(mptr, io[s], bytes / v.esz, st));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 0) v.ms.push_back(ms);
        }
    }
    // long double (software x87, x87.hpp): valid encodings in [1, 2) with random
    // 64-bit significands, so every element takes the full add / mul path
    std::vector<Var> lds = {
        {"SUM long double", 16, &launch_reduce<OpSum, x80>, {}},
        {"PROD long double", 16, &launch_reduce<OpProd, x80>, {}},
        {"MAX long double", 16, &launch_reduce<OpMax, x80>, {}},
        {"SUM long double _Complex (E2)", 32, &launch_reduce_wide<OpSum, cx80, 2>, {}},
        {"PROD long double _Complex (E1)", 32, &launch_reduce_wide<OpProd, cx80, 1>, {}},
        {"PROD long double _Complex E2", 32, &launch_reduce_wide<OpProd, cx80, 2>, {}},
        {"MAXLOC long double_int (E2)", 32, &launch_reduce_wide<OpMaxloc, pldint, 2>, {}},
    };

    {
        std::vector<uint64_t> h(bytes / 8);
        uint64_t x = 88172645463325252ull;
        for (size_t i = 0; i < h.size(); i += 2) {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            h[i] = x | (1ull << 63);
            h[i + 1] = 0x3fff;
        }
        for (int s = 0; s < NS; ++s) {
            CK(hipMemcpy(in[s], h.data(), bytes, hipMemcpyHostToDevice));
            CK(hipMemcpy(io[s], h.data(), bytes, hipMemcpyHostToDevice));
        }
        for (int r = -2; r < rounds; ++r)
            for (auto &v : lds) {
                int s = slot++ % NS;
                // fresh inout every time so PROD / SUM never leave [1, 2^k)
                CK(hipMemcpyAsync(io[s], in[(s + 1) % NS], bytes, hipMemcpyDeviceToDevice, st));
                CK(hipEventRecord(e0, st));
                CK(v.fn(in[s], io[s], bytes / v.esz, st));
                CK(hipEventRecord(e1, st));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r >= 0) v.ms.push_back(ms);
            }
    }
    printf("%zu MiB per operand, %d interleaved rounds\n", mib, rounds);
    for (auto &v : lds) {
        std::sort(v.ms.begin(), v.ms.end());
        double med = v.ms[v.ms.size() / 2];
        double gbs = 3.0 * bytes / (med * 1e-3) / 1e9;
        printf("%-28s median %8.2f us  -> %7.0f GB/s  frac %.3f  (%.2f G elem/s)\n", v.name.c_str(), med * 1e3, gbs,
               gbs / 8000.0, bytes / v.esz / (med * 1e-3) / 1e9);
    }
    for (auto &v : mvs) {
        std::sort(v.ms.begin(), v.ms.end());
        double med = v.ms[v.ms.size() / 2];
        int pp = v.name.find("TREE4") != std::string::npos ? 4 : (v.name.find("TREE2") != std::string::npos ? 2 : 8);
        double gbs = (pp + 1.0) * bytes / (med * 1e-3) / 1e9;
        printf("%-36s median %8.2f us -> %7.0f GB/s ((P+1) x operand bytes) frac %.3f\n", v.name.c_str(), med * 1e3, gbs, gbs / 8000.0);
    }
    for (auto &v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        double med = v.ms[v.ms.size() / 2], mn = v.ms[0];
        double gbs = 3.0 * bytes / (med * 1e-3) / 1e9;
        printf("%-28s median %8.2f us  min %8.2f us  -> %7.0f GB/s  %6.0f GiB/s  frac %.3f\n", v.name.c_str(),
               med * 1e3, mn * 1e3, gbs, 3.0 * bytes / (med * 1e-3) / (1 << 30), gbs / 8000.0);
    }
    return 0;
}

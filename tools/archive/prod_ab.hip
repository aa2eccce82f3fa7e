// prod_ab.hip -- why is int32 MPI_PROD ~4 % below the other config-3 kernels?
// Interleaved A/B of k_reduce_tile<OpProd, int32_t> against shape variants.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -Impich-pip_amd/csrc/hip -o tools/prod_ab tools/prod_ab.hip
//   ./tools/prod_ab [MiB_per_operand=256] [rounds=20]
//
// v_mul_lo_u32 is a quarter-rate VALU op: 16 per lane per 16 KiB tile.  The
// variants test whether that work delays the workgroup's exit (shorter tiles,
// priority after the loads land) or whether a full-rate 24-bit decomposition
// of the 32-bit product helps.
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

// a*b mod 2^32 from full-rate 24-bit multiplies: with a = ah*2^24 + al,
// a*b = al*bl + ((ah*bl + al*bh) << 24)  (mod 2^32); v_mul_u32_u24 reads the
// low 24 bits of each source.
struct OpProdMul24 {
    __device__ __forceinline__ int32_t operator()(int32_t a, int32_t b) const {
        const uint32_t ua = (uint32_t)a, ub = (uint32_t)b;
        const uint32_t lo = __umul24(ua, ub);
        uint32_t t = __umul24(ua >> 24, ub);
        t += __umul24(ua, ub >> 24);
        return (int32_t)(lo + (t << 24));
    }
};

template <class Op, int VPL, int NT, bool PRIO>
__global__ __launch_bounds__(NT) void k_var(const char *in, char *io, uint64_t vbytes) {
    constexpr uint32_t tile = NT * VPL * 16;
    const uint64_t base = (uint64_t)blockIdx.x * tile;
    if (base >= vbytes) return;
    const uint64_t left = vbytes - base;
    const int nrec = (int)(left < tile ? left : tile);
    __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void *)(in + base), 0, nrec, 0x00020000);
    __amdgpu_buffer_rsrc_t rio = __builtin_amdgcn_make_buffer_rsrc((void *)(io + base), 0, nrec, 0x00020000);
    u32x4 a[VPL], b[VPL];
#pragma unroll
    for (int u = 0; u < VPL; ++u) {
        const int off = (u * NT + (int)threadIdx.x) * 16;
        a[u] = __builtin_amdgcn_raw_buffer_load_b128(rio, off, 0, kCachePolicyNT);
        b[u] = __builtin_amdgcn_raw_buffer_load_b128(rin, off, 0, kCachePolicyNT);
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(2);
#pragma unroll
    for (int u = 0; u < VPL; ++u) {
        const int off = (u * NT + (int)threadIdx.x) * 16;
        __builtin_amdgcn_raw_buffer_store_b128(combine16<Op, int32_t>(a[u], b[u]), rio, off, 0, kCachePolicyNT);
    }
}

template <class Op, int VPL, int NT, bool PRIO>
hipError_t launch_var(const void *in, void *io, uint64_t count, hipStream_t s) {
    constexpr uint32_t tile = NT * VPL * 16;
    const uint64_t vbytes = count * 4;   // 256 MiB: a multiple of every tile
    hipLaunchKernelGGL((k_var<Op, VPL, NT, PRIO>), dim3((unsigned)((vbytes + tile - 1) / tile)), dim3(NT), 0, s,
                       (const char *)in, (char *)io, vbytes);
    return hipGetLastError();
}

struct Var {
    std::string name;
    hipError_t (*fn)(const void *, void *, uint64_t, hipStream_t);
    std::vector<float> ms;
};

int main(int argc, char **argv) {
    size_t mib = argc > 1 ? strtoull(argv[1], 0, 10) : 256;
    int rounds = argc > 2 ? atoi(argv[2]) : 20;
    size_t bytes = mib << 20;
    const int NS = 3;
    char *in[NS], *io[NS];
    std::vector<int32_t> h(bytes / 4);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (int32_t)(i * 2654435761u);
    std::vector<int32_t> ones(bytes / 4, 1);
    for (int s = 0; s < NS; ++s) {
        CK(hipMalloc(&in[s], bytes));
        CK(hipMalloc(&io[s], bytes));
        CK(hipMemcpy(in[s], ones.data(), bytes, hipMemcpyHostToDevice));
        CK(hipMemcpy(io[s], h.data(), bytes, hipMemcpyHostToDevice));
    }
    // correctness of the mul24 form on a random slice
    {
        std::vector<int32_t> x(1 << 20), y(1 << 20), z(1 << 20);
        uint64_t st = 88172645463325252ull;
        for (size_t i = 0; i < x.size(); ++i) {
            st ^= st << 13; st ^= st >> 7; st ^= st << 17;
            x[i] = (int32_t)st; y[i] = (int32_t)(st >> 32);
        }
        char *dx, *dy;
        CK(hipMalloc(&dx, 4 << 20)); CK(hipMalloc(&dy, 4 << 20));
        CK(hipMemcpy(dx, y.data(), 4 << 20, hipMemcpyHostToDevice));
        CK(hipMemcpy(dy, x.data(), 4 << 20, hipMemcpyHostToDevice));
        CK((launch_var<OpProdMul24, 4, 256, false>(dx, dy, 1 << 20, 0)));
        CK(hipMemcpy(z.data(), dy, 4 << 20, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < x.size(); ++i) bad += (uint32_t)z[i] != (uint32_t)x[i] * (uint32_t)y[i];
        printf("mul24 form: %zu wrong of %zu\n", bad, x.size());
        CK(hipFree(dx)); CK(hipFree(dy));
    }
    std::vector<Var> vs = {
        {"PROD int32 product", &launch_reduce<OpProd, int32_t>, {}},
        {"SUM  int32 product", &launch_reduce<OpSum, int32_t>, {}},
        {"PROD int32 VPL2 T256", &launch_var<OpProd, 2, 256, false>, {}},
        {"PROD int32 VPL4 T256 prio", &launch_var<OpProd, 4, 256, true>, {}},
        {"PROD int32 VPL4 T512", &launch_var<OpProd, 4, 512, false>, {}},
        {"PROD int32 VPL8 T256", &launch_var<OpProd, 8, 256, false>, {}},
        {"PROD int32 VPL1 T256", &launch_var<OpProd, 1, 256, false>, {}},
        {"PROD int32 mul24 VPL4", &launch_var<OpProdMul24, 4, 256, false>, {}},
        {"PROD int32 mul24 VPL2", &launch_var<OpProdMul24, 2, 256, false>, {}},
        {"PROD int32 product (again)", &launch_reduce<OpProd, int32_t>, {}},
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
            CK(v.fn(in[s], io[s], bytes / 4, st));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 0) v.ms.push_back(ms);
        }
    }
    printf("int32 MPI_PROD variants, %zu MiB per operand, %d interleaved rounds\n", mib, rounds);
    for (auto &v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        const double med = v.ms[v.ms.size() / 2] * 1e-3;
        const double gbs = 3.0 * bytes / med / 1e9;
        printf("  %-30s median %8.2f us  %7.0f GB/s  frac %.3f\n", v.name.c_str(), med * 1e6, gbs, gbs / 8000.0);
    }
    return 0;
}

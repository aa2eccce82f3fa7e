// ticket_ab.hip -- can a persistent grid (a fixed set of workgroups looping
// over the tiles) stream as fast as the product's one-shot tile grid (one
// 16 KiB tile per workgroup, the hardware dispatcher handing tiles out in
// order)?  A resident reducer would need one.  fp32 SUM, the product's
// reduce_tile body in every variant:
//   product      k_reduce_tile_lean, one tile per workgroup
//   stride G     G workgroups, tile t = w, w + G, ...  (static)
//   chunk G      G workgroups, a contiguous run of tiles each (static)
//   ticket G/T   G workgroups; tickets of T tiles handed out per XCD
//                (workgroup w runs on XCD w % 8) by one counter per XCD,
//                the first ticket static, the next fetched while the
//                current one streams
// Run under rocprofv3 --kernel-trace and read the durations with
// tools/trace_medians.py.  Pairs rotate over >= 1 GiB (no Infinity Cache hits).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -Impich-pip_amd/csrc/hip -o tools/ticket_ab tools/ticket_ab.hip
//   rocprofv3 --kernel-trace -d gpurun_out/tk -o tk -- tools/ticket_ab [MiB=256] [rounds=20]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "reduce_kernels.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(2);} } while (0)

namespace mpir_hip {
uint64_t keep_bytes() { return 0; }
uint64_t keep_for(uint64_t) { return 0; }
}
using namespace mpir_hip;

template <int G>
__global__ __launch_bounds__(256) void k_stride(const char *in, char *io, uint64_t vbytes, uint32_t ntiles) {
    for (uint32_t t = blockIdx.x; t < ntiles; t += G) reduce_tile<OpSum, float>(in, io, (uint64_t)t, vbytes, 0);
}

template <int G>
__global__ __launch_bounds__(256) void k_chunk(const char *in, char *io, uint64_t vbytes, uint32_t ntiles) {
    const uint32_t per = (ntiles + G - 1) / G;
    const uint32_t b = blockIdx.x * per, e = min(ntiles, b + per);
    for (uint32_t t = b; t < e; ++t) reduce_tile<OpSum, float>(in, io, (uint64_t)t, vbytes, 0);
}

// ctr: this launch's 8 counters (64 B apart); other: the next launch's, zeroed here
template <int G, int T>
__global__ __launch_bounds__(256) void k_ticket(const char *in, char *io, uint64_t vbytes, uint32_t ntiles, uint32_t *ctr,
                                                uint32_t *other) {
    __shared__ uint32_t next_s;
    if (blockIdx.x == 0 && threadIdx.x < 8) other[threadIdx.x * 16] = 0u;
    const uint32_t x = blockIdx.x & 7u;
    const uint32_t ntickets = (ntiles + T - 1) / T;
    uint32_t j = blockIdx.x >> 3;
    for (;;) {
        const uint32_t ticket = x + 8u * j;
        if (ticket >= ntickets) break;
        if (threadIdx.x == 0) next_s = (uint32_t)(G / 8) + __hip_atomic_fetch_add(ctr + x * 16, 1u, __ATOMIC_RELAXED,
                                                                                  __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll 1
        for (int k = 0; k < T; ++k) {
            const uint32_t t = ticket * T + k;
            if (t < ntiles) reduce_tile<OpSum, float>(in, io, (uint64_t)t, vbytes, 0);
        }
        __syncthreads();
        j = next_s;
        __syncthreads();
    }
}

struct Var {
    std::string name;
    int kind;   // 0 product, 1 stride, 2 chunk, 3 ticket
    void (*k)();
    int G;
};

typedef void (*kfn4)(const char *, char *, uint64_t, uint32_t);
typedef void (*kfn6)(const char *, char *, uint64_t, uint32_t, uint32_t *, uint32_t *);

int main(int argc, char **argv) {
    const size_t mib = argc > 1 ? strtoull(argv[1], 0, 10) : 256;
    const int rounds = argc > 2 ? atoi(argv[2]) : 20;
    const size_t bytes = mib << 20;
    const int NS = (int)std::max<size_t>(4, (2048 + 2 * mib - 1) / (2 * mib));   // >= 2 GiB of pairs
    std::vector<char *> in(NS), io(NS);
    std::vector<float> h(bytes / 4);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 1.0f + (float)((i * 2654435761u) % 1024) * (1.0f / 1024);
    for (int s = 0; s < NS; ++s) {
        CK(hipMalloc(&in[s], bytes));
        CK(hipMalloc(&io[s], bytes));
        CK(hipMemcpy(in[s], h.data(), bytes, hipMemcpyHostToDevice));
        CK(hipMemcpy(io[s], h.data(), bytes, hipMemcpyHostToDevice));
    }
    uint32_t *ctr = nullptr;
    CK(hipMalloc(&ctr, 2 * 8 * 64));
    CK(hipMemset(ctr, 0, 2 * 8 * 64));
    const uint32_t ntiles = (uint32_t)((bytes + kTileBytes - 1) / kTileBytes);
    std::vector<Var> vs = {
        {"product one-shot", 0, nullptr, 0},
        {"stride 2048", 1, (void (*)())k_stride<2048>, 2048},
        {"chunk 2048", 2, (void (*)())k_chunk<2048>, 2048},
        {"ticket 2048/1", 3, (void (*)())k_ticket<2048, 1>, 2048},
        {"ticket 2048/2", 3, (void (*)())k_ticket<2048, 2>, 2048},
        {"ticket 2048/4", 3, (void (*)())k_ticket<2048, 4>, 2048},
        {"ticket 1024/2", 3, (void (*)())k_ticket<1024, 2>, 1024},
        {"ticket 1024/4", 3, (void (*)())k_ticket<1024, 4>, 1024},
        {"ticket 4096/1", 3, (void (*)())k_ticket<4096, 1>, 4096},
    };
    hipStream_t st;
    CK(hipStreamCreate(&st));
    std::vector<int> order(vs.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = (int)i;
    uint32_t rs = 4242;
    int slot = 0, parity = 0;
    for (int r = -2; r < rounds; ++r) {
        for (size_t i = order.size() - 1; i > 0; --i) {
            rs = rs * 1664525u + 1013904223u;
            std::swap(order[i], order[(rs >> 8) % (i + 1)]);
        }
        for (int vi : order) {
            const int s = slot++ % NS;
            const Var &v = vs[vi];
            if (v.kind == 0) {
                CK((launch_reduce<OpSum, float>(in[s], io[s], bytes / 4, st)));
            } else if (v.kind <= 2) {
                hipLaunchKernelGGL((kfn4)v.k, dim3(v.G), dim3(256), 0, st, (const char *)in[s], io[s], (uint64_t)bytes, ntiles);
            } else {
                uint32_t *c = ctr + parity * 8 * 16, *o = ctr + (parity ^ 1) * 8 * 16;
                parity ^= 1;
                hipLaunchKernelGGL((kfn6)v.k, dim3(v.G), dim3(256), 0, st, (const char *)in[s], io[s], (uint64_t)bytes, ntiles,
                                   c, o);
            }
            CK(hipGetLastError());
            CK(hipStreamSynchronize(st));
        }
    }
    printf("%zu MiB per operand, %d rounds, %d pairs, %zu variants; kernel times in the rocprofv3 trace\n", mib, rounds, NS,
           vs.size());
    // one more check: a fresh pair, each variant once, result = a + b
    {
        std::vector<float> got(h.size());
        for (const Var &v : vs) {
            CK(hipMemcpy(io[0], h.data(), bytes, hipMemcpyHostToDevice));
            if (v.kind == 0) CK((launch_reduce<OpSum, float>(in[0], io[0], bytes / 4, st)));
            else if (v.kind <= 2)
                hipLaunchKernelGGL((kfn4)v.k, dim3(v.G), dim3(256), 0, st, (const char *)in[0], io[0], (uint64_t)bytes, ntiles);
            else {
                uint32_t *c = ctr + parity * 8 * 16, *o = ctr + (parity ^ 1) * 8 * 16;
                parity ^= 1;
                hipLaunchKernelGGL((kfn6)v.k, dim3(v.G), dim3(256), 0, st, (const char *)in[0], io[0], (uint64_t)bytes, ntiles,
                                   c, o);
            }
            CK(hipStreamSynchronize(st));
            CK(hipMemcpy(got.data(), io[0], bytes, hipMemcpyDeviceToHost));
            size_t bad = 0;
            for (size_t i = 0; i < h.size(); ++i) bad += got[i] != h[i] + h[i];
            printf("check %-18s %s (%zu wrong)\n", v.name.c_str(), bad ? "FAIL" : "ok", bad);
        }
    }
    for (size_t i = 0; i < vs.size(); ++i) printf("variant %zu = %s\n", i, vs[i].name.c_str());
    return 0;
}

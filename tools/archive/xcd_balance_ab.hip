// xcd_balance_ab.hip -- can cross-XCD balancing of the last round absorb the
// isolated slow launches?  tools/tail_xcd_trace.hip showed that a slow launch
// is one or two XCDs (pairs {3,5} or {1,7}) finishing 5-14 us after the others,
// which idle meanwhile: workgroups go to the XCDs round-robin, so each XCD owns
// a fixed 1/8 of the tiles.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I mpich-pip_amd/csrc/hip \
//         tools/xcd_balance_ab.hip -o tools/xcd_balance_ab
//   tools/xcd_balance_ab [launches per variant, default 300]
//
// Variants, interleaved launch by launch over 4 rotating 256 MiB fp32 pairs:
//   static     the product tile grid (16,384 workgroups, one tile each);
//   tail T/C   the first N - T tiles static, one per workgroup (N - T
//              workgroups); the last round of 2,048 workgroups then also takes
//              tail tiles from C counters (the workgroups of eight consecutive
//              block ids -- one per XCD -- share a counter and its T / C tiles),
//              so a workgroup on a fast XCD takes a slow XCD's share.  The first
//              ticket is fetched before the static tile, each next one before
//              the tile in hand, so the atomic's latency hides behind a tile.
// Every workgroup records start / end wall clock (100 MHz); per variant: median,
// mean and p90 of the span (first start to last end), and the share of slow
// launches (> the static median + 4 us).  Results are verified (inbuf 1.0,
// inoutbuf counts its launches).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#include "reduce_kernels.hpp"

using namespace mpir_hip;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); exit(1); } } while (0)

struct Rec { unsigned long long t0, t1; };

__device__ __forceinline__ unsigned long long wall() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ void record(Rec *rec, unsigned long long t0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) rec[blockIdx.x] = Rec{t0, wall()};
}

__global__ __launch_bounds__(kThreads) void k_static(const char *in, char *io, uint64_t vbytes, Rec *rec) {
    const unsigned long long t0 = wall();
    reduce_tile<OpSum, float>(in, io, blockIdx.x, vbytes, 0);
    record(rec, t0);
}

// counters: C of them, 64 words apart (each on its own 256-byte line)
__global__ __launch_bounds__(kThreads) void k_tail(const char *in, char *io, uint64_t vbytes, unsigned nstatic,
                                                   unsigned per_ctr, unsigned nctr, unsigned *ctr, Rec *rec) {
    const unsigned long long t0 = wall();
    const unsigned b = blockIdx.x;
    const bool last_round = b + 2048u >= nstatic;
    const unsigned c = (b >> 3) % nctr;
    unsigned *my = ctr + 64u * c;
    __shared__ unsigned s_tk;
    unsigned tk = ~0u;
    if (last_round && threadIdx.x == 0) tk = __hip_atomic_fetch_add(my, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    reduce_tile<OpSum, float>(in, io, b, vbytes, 0);
    if (last_round) {
        for (;;) {
            __syncthreads();
            if (threadIdx.x == 0) s_tk = tk;
            __syncthreads();
            const unsigned t = s_tk;
            if (t >= per_ctr) break;
            if (threadIdx.x == 0) tk = __hip_atomic_fetch_add(my, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            reduce_tile<OpSum, float>(in, io, (uint64_t)nstatic + (uint64_t)c * per_ctr + t, vbytes, 0);
        }
    }
    record(rec, t0);
}

__global__ void k_fill(float *p, uint64_t n, float v) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = v;
}

int main(int argc, char **argv) {
    const int per = argc > 1 ? atoi(argv[1]) : 300;
    const uint64_t bytes = 256ull << 20;
    const unsigned ntiles = (unsigned)(bytes / kTileBytes);
    const int npairs = 4;
    struct V { const char *name; unsigned T, C; };
    const V vars[] = {{"static", 0, 0}, {"tail 2048/256", 2048, 256}, {"tail 1024/128", 1024, 128},
                      {"tail 4096/256", 4096, 256}};
    const int nv = 4;
    char *buf[2 * npairs];
    for (int k = 0; k < 2 * npairs; ++k) {
        CK(hipMalloc(&buf[k], bytes));
        k_fill<<<4096, 256>>>((float *)buf[k], bytes / 4, (k & 1) ? 0.0f : 1.0f);   // even: in = 1, odd: inout = 0
    }
    const int launches = per * nv;
    Rec *rec;
    CK(hipMalloc(&rec, sizeof(Rec) * ntiles * (size_t)launches));
    unsigned *ctr;
    const size_t ctr_words = 64u * 256u;
    CK(hipMalloc(&ctr, sizeof(unsigned) * ctr_words * (launches + 16)));
    CK(hipMemset(ctr, 0, sizeof(unsigned) * ctr_words * (launches + 16)));
    CK(hipDeviceSynchronize());
    int pair_uses[npairs] = {};
    auto launch = [&](int i, int v, Rec *r, unsigned *cw) {
        const int p = i % npairs;
        ++pair_uses[p];
        const char *in = buf[2 * p];
        char *io = buf[2 * p + 1];
        if (vars[v].T == 0) {
            k_static<<<ntiles, kThreads>>>(in, io, bytes, r);
        } else {
            const unsigned ns = ntiles - vars[v].T;
            k_tail<<<ns, kThreads>>>(in, io, bytes, ns, vars[v].T / vars[v].C, vars[v].C, cw, r);
        }
    };
    // warm-up: 16 launches, counters of their own
    for (int i = 0; i < 16; ++i) launch(i, i % nv, rec, ctr + ctr_words * (size_t)(launches + (i % 16)));
    CK(hipDeviceSynchronize());
    for (int i = 0; i < launches; ++i) launch(16 + i, i % nv, rec + (size_t)i * ntiles, ctr + ctr_words * (size_t)i);
    CK(hipDeviceSynchronize());
    // verify: every inout element counts the launches of its pair
    int bad = 0;
    std::vector<float> h(1 << 20);
    for (int p = 0; p < npairs; ++p)
        for (uint64_t off = 0; off < bytes; off += 64ull << 20) {
            CK(hipMemcpy(h.data(), buf[2 * p + 1] + off, 4u << 20, hipMemcpyDeviceToHost));
            for (float x : h) bad += x != (float)pair_uses[p];
        }
    std::vector<Rec> hr((size_t)ntiles * launches);
    CK(hipMemcpy(hr.data(), rec, sizeof(Rec) * hr.size(), hipMemcpyDeviceToHost));
    std::vector<std::vector<double>> span(nv);
    for (int i = 0; i < launches; ++i) {
        const int v = i % nv;
        const unsigned ng = vars[v].T ? ntiles - vars[v].T : ntiles;
        unsigned long long s0 = ~0ull, e1 = 0;
        for (unsigned g = 0; g < ng; ++g) {
            s0 = std::min(s0, hr[(size_t)i * ntiles + g].t0);
            e1 = std::max(e1, hr[(size_t)i * ntiles + g].t1);
        }
        span[v].push_back((e1 - s0) * 0.01);
    }
    std::vector<double> s = span[0];
    std::sort(s.begin(), s.end());
    const double ref = s[s.size() / 2];
    printf("verify: %d wrong elements (checked 4 MiB of every 64 MiB)\n", bad);
    for (int v = 0; v < nv; ++v) {
        std::vector<double> x = span[v];
        std::sort(x.begin(), x.end());
        double mean = 0;
        int slow = 0;
        for (double d : x) {
            mean += d;
            slow += d > ref + 4.0;
        }
        mean /= x.size();
        printf("%-14s launches %d  median %.2f us  mean %.2f  p90 %.2f  max %.2f  slow (> static median + 4) %.1f %%\n",
               vars[v].name, (int)x.size(), x[x.size() / 2], mean, x[x.size() * 9 / 10], x.back(),
               100.0 * slow / x.size());
    }
    return bad != 0;
}

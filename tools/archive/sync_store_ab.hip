// sync_store_ab.hip -- does the store cache policy change the cost of a
// SYNCHRONOUS call?  In the rocprofv3 trace of bench.py the next dispatch on
// the stream starts ~5 us after the reduce kernel's end timestamp; that gap
// holds the end-of-kernel release, which writes back dirty L2 lines.  nt
// stores may leave up to the L2 capacity (4 MiB x 8 XCDs) dirty; sc1 stores
// (device scope) write through.  This A/B runs the product tile shape
// (mpir_hip::reduce_tile: 16 KiB per operand per 256-thread workgroup, issue
// gaps) with the store aux bits as a template parameter, and times per call
//   sync: launch + hipStreamWriteValue32 + host spin (the library's wait),
//   ev:   HIP events around each launch (kernel only),
// over 4 rotating 256 MiB fp32 pairs, policies interleaved per round.
//   hipcc --offload-arch=gfx950 -O3 -Impich-pip_amd/csrc/hip -o tools/sync_store_ab tools/sync_store_ab.hip
//   ./tools/sync_store_ab [MiB=256] [rounds=12] [pairs=4]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "reduce_kernels.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(2);} } while (0)

using namespace mpir_hip;

template <int LP, int SP>
__global__ __launch_bounds__(kThreads) void k_pol(const char *in, char *io, uint64_t vbytes) {
    const uint64_t base = (uint64_t)blockIdx.x * kTileBytes;
    if (base >= vbytes) return;
    const uint64_t left = vbytes - base;
    const int nrec = (int)(left < kTileBytes ? left : kTileBytes);
    __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void *)(in + base), 0, nrec, 0x00020000);
    __amdgpu_buffer_rsrc_t rio = __builtin_amdgcn_make_buffer_rsrc((void *)(io + base), 0, nrec, 0x00020000);
    const int t = (int)threadIdx.x;
    const int wb = (t >> 6) * (kVecPerLane * 1024) + (t & 63) * 16;
    u32x4 a[kVecPerLane], b[kVecPerLane];
#pragma unroll
    for (int u = 0; u < kVecPerLane; ++u) {
        a[u] = __builtin_amdgcn_raw_buffer_load_b128(rio, wb + u * 1024, 0, LP);
        b[u] = __builtin_amdgcn_raw_buffer_load_b128(rin, wb + u * 1024, 0, LP);
        if (u + 1 < kVecPerLane) issue_gap();
    }
#pragma unroll
    for (int u = 0; u < kVecPerLane; ++u)
        __builtin_amdgcn_raw_buffer_store_b128(combine16<OpSum, float>(a[u], b[u]), rio, wb + u * 1024, 0, SP);
}

typedef void (*kfn)(const char *, char *, uint64_t);
struct Var { const char *name; kfn k; };

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char **argv) {
    const size_t mib = argc > 1 ? strtoull(argv[1], 0, 10) : 256;
    const int rounds = argc > 2 ? atoi(argv[2]) : 12;
    const size_t bytes = mib << 20;
    const int NP = argc > 3 ? atoi(argv[3]) : 4, K = 40;
    std::vector<char *> in(NP), io(NP);
    for (int p = 0; p < NP; ++p) {
        CK(hipMalloc(&in[p], bytes));
        CK(hipMalloc(&io[p], bytes));
        CK(hipMemset(in[p], 0, bytes));
        CK(hipMemset(io[p], 0, bytes));
    }
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    volatile unsigned *flag;
    CK(hipHostMalloc((void **)&flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
    *flag = 0;
    unsigned seq = 0;
    std::vector<hipEvent_t> e0(K), e1(K);
    for (int i = 0; i < K; ++i) { CK(hipEventCreate(&e0[i])); CK(hipEventCreate(&e1[i])); }
    Var vs[] = {
        {"store nt (product)", (kfn)&k_pol<2, 2>},
        {"store sc1", (kfn)&k_pol<2, 16>},
        {"store nt sc1", (kfn)&k_pol<2, 18>},
        {"store sc0 sc1", (kfn)&k_pol<2, 17>},
        {"store default", (kfn)&k_pol<2, 0>},
        {"library lean kernel", (kfn)&k_reduce_tile_lean<OpSum, float>},
    };
    const int NV = sizeof(vs) / sizeof(vs[0]);
    const unsigned grid = (unsigned)(bytes / kTileBytes);
    std::vector<std::vector<double>> sync_us(NV), ev_us(NV);
    std::vector<int> order(NV);
    for (int i = 0; i < NV; ++i) order[i] = i;
    uint32_t rs = 12345;
    int slot = 0;
    for (int r = -1; r < rounds; ++r) {
        for (int i = NV - 1; i > 0; --i) { rs = rs * 1664525u + 1013904223u; std::swap(order[i], order[(rs >> 8) % (i + 1)]); }
        for (int vi : order) {
            kfn k = vs[vi].k;
            // synchronous calls
            const double t0 = now();
            for (int i = 0; i < K; ++i) {
                const int p = slot++ % NP;
                hipLaunchKernelGGL(k, dim3(grid), dim3(kThreads), 0, s, (const char *)in[p], io[p], (uint64_t)bytes);
                CK(hipStreamWriteValue32(s, (void *)flag, ++seq, 0));
                while (*flag != seq) __builtin_ia32_pause();
            }
            const double t1 = now();
            // event-timed launches, back to back
            for (int i = 0; i < K; ++i) {
                const int p = slot++ % NP;
                CK(hipEventRecord(e0[i], s));
                hipLaunchKernelGGL(k, dim3(grid), dim3(kThreads), 0, s, (const char *)in[p], io[p], (uint64_t)bytes);
                CK(hipEventRecord(e1[i], s));
            }
            CK(hipStreamSynchronize(s));
            if (r < 0) continue;
            sync_us[vi].push_back((t1 - t0) / K * 1e6);
            std::vector<float> ms(K);
            for (int i = 0; i < K; ++i) CK(hipEventElapsedTime(&ms[i], e0[i], e1[i]));
            std::sort(ms.begin(), ms.end());
            ev_us[vi].push_back(ms[K / 2] * 1e3);
        }
    }
    printf("fp32 SUM %zu MiB per operand, %d rotating pairs, %d rounds x %d calls, policies interleaved\n", mib, NP, rounds, K);
    for (int v = 0; v < NV; ++v) {
        std::sort(sync_us[v].begin(), sync_us[v].end());
        std::sort(ev_us[v].begin(), ev_us[v].end());
        const double sm = sync_us[v][rounds / 2], em = ev_us[v][rounds / 2];
        printf("  %-22s sync %8.2f us/call (%.3f of peak)  kernel(ev, median) %8.2f us (%.3f)  sync - kernel %5.2f us\n",
               vs[v].name, sm, 3.0 * bytes / (sm * 1e-6) / 8e12, em, 3.0 * bytes / (em * 1e-6) / 8e12, sm - em);
    }
    return 0;
}

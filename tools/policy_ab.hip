// policy_ab.hip -- cache-policy bits of the k_reduce_tile loads / stores at the
// BASELINE config-2 size (64 MiB per operand, 8 rotating windows as in bench.py)
// and at 256 MiB.  gfx950 buffer aux bits: sc0 = 1, nt = 2, sc1 = 16.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -Impich-pip_amd/csrc/hip -o tools/policy_ab tools/policy_ab.hip
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

template <int LP, int SP>
__global__ __launch_bounds__(kThreads) void k_pol(const char *in, char *io, uint64_t vbytes) {
    const uint64_t base = (uint64_t)blockIdx.x * kTileBytes;
    if (base >= vbytes) return;
    const uint64_t left = vbytes - base;
    const int nrec = (int)(left < kTileBytes ? left : kTileBytes);
    __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void *)(in + base), 0, nrec, 0x00020000);
    __amdgpu_buffer_rsrc_t rio = __builtin_amdgcn_make_buffer_rsrc((void *)(io + base), 0, nrec, 0x00020000);
    u32x4 a[kVecPerLane], b[kVecPerLane];
#pragma unroll
    for (int u = 0; u < kVecPerLane; ++u) {
        const int off = (u * kThreads + (int)threadIdx.x) * 16;
        a[u] = __builtin_amdgcn_raw_buffer_load_b128(rio, off, 0, LP);
        b[u] = __builtin_amdgcn_raw_buffer_load_b128(rin, off, 0, LP);
    }
#pragma unroll
    for (int u = 0; u < kVecPerLane; ++u) {
        const int off = (u * kThreads + (int)threadIdx.x) * 16;
        __builtin_amdgcn_raw_buffer_store_b128(combine16<OpSum, float>(a[u], b[u]), rio, off, 0, SP);
    }
}

template <int LP, int SP>
hipError_t launch_pol(const void *in, void *io, uint64_t count, hipStream_t s) {
    const uint64_t vbytes = count * 4;
    hipLaunchKernelGGL((k_pol<LP, SP>), dim3((unsigned)((vbytes + kTileBytes - 1) / kTileBytes)), dim3(kThreads), 0,
                       s, (const char *)in, (char *)io, vbytes);
    return hipGetLastError();
}

struct Var {
    std::string name;
    hipError_t (*fn)(const void *, void *, uint64_t, hipStream_t);
    std::vector<float> ms;
};

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 15;
    const size_t total = 1024ull << 20;         // per operand array; windows rotate through it
    char *in, *io;
    CK(hipMalloc(&in, total));
    CK(hipMalloc(&io, total));
    {
        std::vector<float> h(total / 4);
        uint32_t x = 12345;
        for (auto &v : h) { x = x * 1664525u + 1013904223u; v = (float)(x >> 8) * (1.0f / 16777216.0f) - 0.5f; }
        CK(hipMemcpy(in, h.data(), total, hipMemcpyHostToDevice));
        CK(hipMemcpy(io, h.data(), total, hipMemcpyHostToDevice));
    }
    const int set = argc > 2 ? atoi(argv[2]) : 0;
    std::vector<Var> vs;
    if (set == 0)
        vs = {
            {"load nt  / store nt (product)", &launch_pol<2, 2>, {}},
            {"load nt  / store default", &launch_pol<2, 0>, {}},
            {"load nt  / store sc1", &launch_pol<2, 16>, {}},
            {"load nt  / store nt sc1", &launch_pol<2, 18>, {}},
            {"load nt  / store sc0 sc1", &launch_pol<2, 17>, {}},
            {"load nt  / store sc0 nt", &launch_pol<2, 3>, {}},
            {"load default / store nt", &launch_pol<0, 2>, {}},
            {"load sc1 / store nt", &launch_pol<16, 2>, {}},
            {"load nt sc1 / store nt sc1", &launch_pol<18, 18>, {}},
            {"load nt  / store nt (again)", &launch_pol<2, 2>, {}},
        };
    else if (set == 2)
        vs = {
            {"load nt  / store nt (product)", &launch_pol<2, 2>, {}},
            {"load nt  / store sc0 sc1", &launch_pol<2, 17>, {}},
            {"load nt  / store sc1", &launch_pol<2, 16>, {}},
            {"load nt  / store default", &launch_pol<2, 0>, {}},
        };
    else
        vs = {
            {"load nt  / store nt (product)", &launch_pol<2, 2>, {}},
            {"load nt  / store sc0 sc1", &launch_pol<2, 17>, {}},
            {"load nt  / store sc0 sc1 nt", &launch_pol<2, 19>, {}},
            {"load nt sc0 / store sc0 sc1", &launch_pol<3, 17>, {}},
            {"load sc0 / store sc0 sc1", &launch_pol<1, 17>, {}},
            {"load default / store sc0 sc1", &launch_pol<0, 17>, {}},
            {"load nt  / store sc0", &launch_pol<2, 1>, {}},
            {"load nt  / store sc0 sc1 (again)", &launch_pol<2, 17>, {}},
            {"load nt  / store nt (again)", &launch_pol<2, 2>, {}},
        };
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<size_t> sizes = {64, 256};
    if (set == 2) sizes = {16, 32, 64, 128, 256};
    for (size_t mib : sizes) {
        const size_t bytes = mib << 20, nwin = total / bytes;
        for (auto &v : vs) v.ms.clear();
        size_t w = 0;
        for (int r = -2; r < rounds; ++r) {
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
        }
        printf("fp32 MPI_SUM %zu MiB per operand, %zu rotating windows, %d interleaved rounds\n", mib, nwin, rounds);
        for (auto &v : vs) {
            std::sort(v.ms.begin(), v.ms.end());
            const double med = v.ms[v.ms.size() / 2] * 1e-3;
            const double gbs = 3.0 * bytes / med / 1e9;
            printf("  %-32s median %8.2f us  %7.0f GB/s  frac %.3f\n", v.name.c_str(), med * 1e6, gbs, gbs / 8000.0);
        }
    }
    return 0;
}

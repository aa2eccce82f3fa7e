// misalign_ab.hip -- MPI_Reduce_local with inbuf and inoutbuf at different
// offsets mod 16 (a schedule step whose tmp_buf and recvbuf sub-ranges start
// differently): element-granular kernel (k_reduce_elems, the previous path)
// vs the aligned-load + shuffle + funnel tile kernel (k_reduce_shift), with
// the aligned tile kernel as the ceiling.  Interleaved rounds, 3 buffer sets.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -Impich-pip_amd/csrc/hip -o tools/misalign_ab tools/misalign_ab.hip
//   ./tools/misalign_ab [MiB=256] [rounds=15]
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

template <class Op, class T>
hipError_t launch_elems(const void *in, void *io, uint64_t count, hipStream_t s) {
    uint64_t grid = (count + kThreads - 1) / kThreads;
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL((k_reduce_elems<Op, T, true>), dim3((unsigned)grid), dim3(kThreads), 0, s,
                       (const char *)in, (char *)io, count, grid * kThreads);
    return hipGetLastError();
}

struct Var {
    std::string name;
    size_t esz;
    int off_in, off_io;
    hipError_t (*fn)(const void *, void *, uint64_t, hipStream_t);
    std::vector<float> ms;
};

int main(int argc, char **argv) {
    size_t mib = argc > 1 ? strtoull(argv[1], 0, 10) : 256;
    int rounds = argc > 2 ? atoi(argv[2]) : 15;
    const size_t bytes = mib << 20;
    const int NS = 3;
    char *in[NS], *io[NS];
    std::vector<float> h(bytes / 4 + 64);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 1.0f + (float)((i * 2654435761u) % 1024) * (1.0f / 1024);
    for (int s = 0; s < NS; ++s) {
        CK(hipMalloc(&in[s], bytes + 256));
        CK(hipMalloc(&io[s], bytes + 256));
        CK(hipMemcpy(in[s], h.data(), bytes + 256, hipMemcpyHostToDevice));
        CK(hipMemcpy(io[s], h.data(), bytes + 256, hipMemcpyHostToDevice));
    }
    std::vector<Var> vs = {
        {"fp32 aligned (k_reduce_tile)", 4, 0, 0, &launch_reduce<OpSum, float>, {}},
        {"fp32 in+4  elems (old)", 4, 4, 0, &launch_elems<OpSum, float>, {}},
        {"fp32 in+4  shift", 4, 4, 0, &launch_reduce<OpSum, float>, {}},
        {"fp32 in+12 shift", 4, 12, 0, &launch_reduce<OpSum, float>, {}},
        {"fp32 io+8  shift", 4, 0, 8, &launch_reduce<OpSum, float>, {}},
        {"fp64 in+8  elems (old)", 8, 8, 0, &launch_elems<OpSum, double>, {}},
        {"fp64 in+8  shift", 8, 8, 0, &launch_reduce<OpSum, double>, {}},
        {"fp16 in+2  elems (old)", 2, 2, 0, &launch_elems<OpSum, f16>, {}},
        {"fp16 in+6  shift", 2, 6, 0, &launch_reduce<OpSum, f16>, {}},
        {"u8 in+1 SUM elems (old)", 1, 1, 0, &launch_elems<OpSum, uint8_t>, {}},
        {"u8 in+1 SUM shift", 1, 1, 0, &launch_reduce<OpSum, uint8_t>, {}},
        {"u8 in+7 SUM shift", 1, 7, 0, &launch_reduce<OpSum, uint8_t>, {}},
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
            CK(v.fn(in[s] + v.off_in, io[s] + v.off_io, bytes / v.esz, st));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 0) v.ms.push_back(ms);
        }
    }
    printf("MPI_Reduce_local, %zu MiB per operand, relative misalignment, %d interleaved rounds\n", mib, rounds);
    for (auto &v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        const double med = v.ms[v.ms.size() / 2] * 1e-3;
        const double gbs = 3.0 * bytes / med / 1e9;
        printf("  %-30s median %8.2f us  %7.0f GB/s  frac %.3f\n", v.name.c_str(), med * 1e6, gbs, gbs / 8000.0);
    }

    // data content: the same aligned fp32 kernel with zero operands.  MPI_BAND
    // with an all-zero inbuf keeps inout at zero, so every round sees the same bytes.
    {
        char *zi, *zo, *ri, *ro;
        CK(hipMalloc(&zi, bytes)); CK(hipMalloc(&zo, bytes));
        CK(hipMalloc(&ri, bytes)); CK(hipMalloc(&ro, bytes));
        CK(hipMemset(zi, 0, bytes)); CK(hipMemset(zo, 0, bytes));
        std::vector<uint32_t> r(bytes / 4);
        uint64_t x = 88172645463325252ull;
        for (auto &w : r) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; w = (uint32_t)x; }
        CK(hipMemcpy(ri, r.data(), bytes, hipMemcpyHostToDevice));
        CK(hipMemcpy(ro, r.data(), bytes, hipMemcpyHostToDevice));
        // every variant leaves its inout unchanged: x & x = x, 0 & 0 = 0, x | 0 = x
        struct D { const char *name; char *i, *o; hipError_t (*fn)(const void *, void *, uint64_t, hipStream_t);
                   std::vector<float> ms; };
        std::vector<D> ds = {{"u32 BAND random / random", ri, ro, &launch_reduce<OpBand, uint32_t>, {}},
                             {"u32 BAND zero / zero", zi, zo, &launch_reduce<OpBand, uint32_t>, {}},
                             {"u32 BOR zero in / random inout", zi, ro, &launch_reduce<OpBor, uint32_t>, {}}};
        for (int rr = -2; rr < rounds; ++rr) {
            for (auto &d : ds) {
                CK(hipEventRecord(e0, st));
                CK(d.fn(d.i, d.o, bytes / 4, st));
                CK(hipEventRecord(e1, st));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (rr >= 0) d.ms.push_back(ms);
            }
        }
        printf("data content (aligned k_reduce_tile, u32):\n");
        for (auto &d : ds) {
            std::sort(d.ms.begin(), d.ms.end());
            const double med = d.ms[d.ms.size() / 2] * 1e-3;
            const double gbs = 3.0 * bytes / med / 1e9;
            printf("  %-30s median %8.2f us  %7.0f GB/s  frac %.3f\n", d.name, med * 1e6, gbs, gbs / 8000.0);
        }
    }
    return 0;
}

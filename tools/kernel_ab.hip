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
        {"SUM fp32 (x86 NaN rule)", 4, &launch_reduce<OpSum, float>, {}},
        {"SUM fp32 (plain add)", 4, &launch_reduce<OpSumPlain, float>, {}},
        {"SUM fp64", 8, &launch_reduce<OpSum, double>, {}},
        {"SUM int32", 4, &launch_reduce<OpSum, int32_t>, {}},
        {"SUM int64", 8, &launch_reduce<OpSum, int64_t>, {}},
        {"MAX fp32", 4, &launch_reduce<OpMax, float>, {}},
        {"MAX fp64", 8, &launch_reduce<OpMax, double>, {}},
        {"MAX int32", 4, &launch_reduce<OpMax, int32_t>, {}},
        {"MAX int64", 8, &launch_reduce<OpMax, int64_t>, {}},
        {"MIN fp32", 4, &launch_reduce<OpMin, float>, {}},
        {"MIN fp64", 8, &launch_reduce<OpMin, double>, {}},
        {"MIN int32", 4, &launch_reduce<OpMin, int32_t>, {}},
        {"MIN int64", 8, &launch_reduce<OpMin, int64_t>, {}},
        {"PROD fp32", 4, &launch_reduce<OpProd, float>, {}},
        {"PROD fp64", 8, &launch_reduce<OpProd, double>, {}},
        {"PROD int32", 4, &launch_reduce<OpProd, int32_t>, {}},
        {"PROD int64", 8, &launch_reduce<OpProd, int64_t>, {}},
        {"SUM fp16", 2, &launch_reduce<OpSum, f16>, {}},
        {"SUM cf32", 8, &launch_reduce<OpSum, cf32>, {}},
        {"PROD cf32", 8, &launch_reduce<OpProd, cf32>, {}},
        {"PROD cf64", 16, &launch_reduce<OpProd, cf64>, {}},
        {"BXOR uint8", 1, &launch_reduce<OpBxor, uint8_t>, {}},
        {"LXOR fp32", 4, &launch_reduce<OpLxor, float>, {}},
        {"MAXLOC 2int", 8, &launch_reduce<OpMaxloc, p2int>, {}},
        {"MAXLOC double_int", 16, &launch_reduce<OpMaxloc, pdoubleint>, {}},
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
    printf("%zu MiB per operand, %d interleaved rounds\n", mib, rounds);
    for (auto &v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        double med = v.ms[v.ms.size() / 2], mn = v.ms[0];
        double gbs = 3.0 * bytes / (med * 1e-3) / 1e9;
        printf("%-28s median %8.2f us  min %8.2f us  -> %7.0f GB/s  %6.0f GiB/s  frac %.3f\n", v.name.c_str(),
               med * 1e3, mn * 1e3, gbs, 3.0 * bytes / (med * 1e-3) / (1 << 30), gbs / 8000.0);
    }
    return 0;
}

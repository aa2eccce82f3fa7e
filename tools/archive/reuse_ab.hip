// reuse_ab.hip -- does a read-only operand re-read every R launches come back
// faster (Infinity Cache reuse), and does that differ between SUM and PROD or
// between an all-ones and a random inbuf?  fp32, 256 MiB per operand; R in
// {2, 3, 4, 8} distinct (inbuf, inoutbuf) pairs rotated, interleaved rounds.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -Impich-pip_amd/csrc/hip -o tools/reuse_ab tools/reuse_ab.hip
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

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 12;
    const size_t bytes = 256ull << 20, count = bytes / 4;
    const int NP = 8;
    char *ones[NP], *rnd[NP], *io[NP];
    std::vector<float> h1(count, 1.0f), hr(count), hio(count);
    uint32_t x = 7;
    for (size_t i = 0; i < count; ++i) {
        x = x * 1664525u + 1013904223u;
        hr[i] = 1.0f + (float)(x >> 8) * (1.0f / 16777216.0f) * 1e-6f;   // ~1: PROD stays finite
        hio[i] = (float)(x >> 9) * (1.0f / 8388608.0f) - 1.0f;
    }
    for (int k = 0; k < NP; ++k) {
        CK(hipMalloc(&ones[k], bytes)); CK(hipMalloc(&rnd[k], bytes)); CK(hipMalloc(&io[k], bytes));
        CK(hipMemcpy(ones[k], h1.data(), bytes, hipMemcpyHostToDevice));
        CK(hipMemcpy(rnd[k], hr.data(), bytes, hipMemcpyHostToDevice));
        CK(hipMemcpy(io[k], hio.data(), bytes, hipMemcpyHostToDevice));
    }
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("fp32 256 MiB per operand, median of %d launches per cell (R pairs rotated)\n", rounds * 8);
    printf("  %-22s %8s %8s %8s %8s\n", "op / inbuf", "R=2", "R=3", "R=4", "R=8");
    for (int op = 0; op < 2; ++op) {
        for (int kind = 0; kind < 2; ++kind) {
            printf("  %-22s", (std::string(op ? "PROD" : "SUM") + (kind ? " / random~1" : " / ones")).c_str());
            for (int R : {2, 3, 4, 8}) {
                std::vector<float> ms;
                for (int i = -4; i < rounds * 8; ++i) {
                    const int k = ((i % R) + R) % R;
                    const char *in = kind ? rnd[k] : ones[k];
                    CK(hipEventRecord(e0, st));
                    if (op) CK((launch_reduce<OpProd, float>(in, io[k], count, st)));
                    else CK((launch_reduce<OpSum, float>(in, io[k], count, st)));
                    CK(hipEventRecord(e1, st));
                    CK(hipEventSynchronize(e1));
                    float t;
                    CK(hipEventElapsedTime(&t, e0, e1));
                    if (i >= 0) ms.push_back(t);
                }
                std::sort(ms.begin(), ms.end());
                const double med = ms[ms.size() / 2] * 1e-3;
                printf(" %8.3f", 3.0 * bytes / med / 8e12);
            }
            printf("\n");
        }
    }
    return 0;
}

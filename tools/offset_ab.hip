// offset_ab.hip -- does the distance between inbuf and inoutbuf change the
// bandwidth of the aligned fp32 MPI_SUM kernel?  Both operands are carved out
// of one allocation with io = in + 256 MiB + D; interleaved rounds, two
// allocations alternated so no launch finds its operands in the Infinity Cache.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//         -Impich-pip_amd/csrc/hip -o tools/offset_ab tools/offset_ab.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "reduce_kernels.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(2);} } while (0)

using namespace mpir_hip;

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 15;
    const size_t mib = 256, bytes = mib << 20, slack = 64ull << 20;
    const size_t D[] = {0, 256, 4096, 65536, 1u << 20, (1u << 20) + 256, 2u << 20, (2u << 20) + 4096,
                        8u << 20, 32u << 20, (32u << 20) + 256};
    const int ND = sizeof(D) / sizeof(D[0]);
    char *buf[2];
    std::vector<float> h(bytes / 4);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 2048) * (1.0f / 1024) - 1.0f;
    for (int s = 0; s < 2; ++s) {
        CK(hipMalloc(&buf[s], 2 * bytes + slack));
        for (size_t o = 0; o + bytes <= 2 * bytes + slack; o += bytes / 4)
            CK(hipMemcpy(buf[s] + o, h.data(), std::min(bytes, 2 * bytes + slack - o), hipMemcpyHostToDevice));
    }
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> ms(ND);
    int k = 0;
    for (int r = -2; r < rounds; ++r) {
        for (int d = 0; d < ND; ++d) {
            char *b = buf[k++ & 1];
            CK(hipEventRecord(e0, st));
            CK((launch_reduce<OpSum, float>(b, b + bytes + D[d], bytes / 4, st)));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (r >= 0) ms[d].push_back(t);
        }
    }
    printf("fp32 MPI_SUM 256 MiB, io = in + 256 MiB + D, %d interleaved rounds\n", rounds);
    for (int d = 0; d < ND; ++d) {
        std::sort(ms[d].begin(), ms[d].end());
        const double med = ms[d][ms[d].size() / 2] * 1e-3;
        const double gbs = 3.0 * bytes / med / 1e9;
        printf("  D = %10zu B  median %8.2f us  %7.0f GB/s  frac %.3f\n", D[d], med * 1e6, gbs, gbs / 8000.0);
    }
    return 0;
}

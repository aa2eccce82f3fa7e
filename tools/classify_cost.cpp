// classify_cost.cpp -- what one pointer classification costs once HIP is up:
// hipPointerGetAttributes (the library's classify()) against the HSA runtime's
// hsa_amd_pointer_info, for device, pinned and pageable pointers.
//
//   hipcc -O2 -std=c++17 tools/classify_cost.cpp -o tools/classify_cost -lhsa-runtime64
//   tools/classify_cost
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

static double now_ns() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e9 + ts.tv_nsec;
}

int main() {
    void *dev = nullptr, *pin = nullptr;
    if (hipMalloc(&dev, 1 << 20) != hipSuccess || hipHostMalloc(&pin, 1 << 20, 0) != hipSuccess) return 1;
    void *page = malloc(1 << 20);
    const char *names[3] = {"device", "pinned", "pageable"};
    void *ptrs[3] = {dev, pin, page};
    const int N = 200000;
    for (int k = 0; k < 3; ++k) {
        hipPointerAttribute_t at;
        hsa_amd_pointer_info_t info;
        info.size = sizeof info;
        for (int i = 0; i < 1000; ++i) {
            (void)hipPointerGetAttributes(&at, ptrs[k]);
            (void)hipGetLastError();
        }
        double t0 = now_ns();
        for (int i = 0; i < N; ++i) {
            (void)hipPointerGetAttributes(&at, (char *)ptrs[k] + (i & 1023));
            (void)hipGetLastError();
        }
        double t1 = now_ns();
        for (int i = 0; i < N; ++i) (void)hsa_amd_pointer_info((char *)ptrs[k] + (i & 1023), &info, nullptr, nullptr, nullptr);
        double t2 = now_ns();
        printf("%-9s hipPointerGetAttributes %6.1f ns   hsa_amd_pointer_info %6.1f ns (type %d)\n", names[k],
               (t1 - t0) / N, (t2 - t1) / N, (int)info.type);
    }
    return 0;
}

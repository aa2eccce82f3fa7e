// sync_modes.hip -- latency of an empty launch + completion under HIP's
// device scheduling flags (spin / yield / blocking-sync / auto), for
// hipStreamSynchronize, hipEventSynchronize and the completion word
// (hipStreamWriteValue32 + host spin) the library uses.
//   hipcc --offload-arch=gfx950 -O2 -o tools/sync_modes tools/sync_modes.hip
//   ./tools/sync_modes <flag: auto|spin|yield|block>
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(2);} } while (0)
__global__ void empty() {}
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char **argv) {
    const char *m = argc > 1 ? argv[1] : "auto";
    unsigned f = hipDeviceScheduleAuto;
    if (!strcmp(m, "spin")) f = hipDeviceScheduleSpin;
    else if (!strcmp(m, "yield")) f = hipDeviceScheduleYield;
    else if (!strcmp(m, "block")) f = hipDeviceScheduleBlockingSync;
    CK(hipSetDeviceFlags(f));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    volatile unsigned *flag;
    CK(hipHostMalloc((void **)&flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
    *flag = 0;
    unsigned seq = 0;
    const int K = 3000;
    for (int r = 0; r < 3; ++r) {
        for (int i = 0; i < 200; ++i) { hipLaunchKernelGGL(empty, 1, 64, 0, s); CK(hipStreamSynchronize(s)); }
        double t0 = now();
        for (int i = 0; i < K; ++i) { hipLaunchKernelGGL(empty, 1, 64, 0, s); CK(hipStreamSynchronize(s)); }
        double t1 = now();
        for (int i = 0; i < K; ++i) { hipLaunchKernelGGL(empty, 1, 64, 0, s); CK(hipEventRecord(ev, s)); CK(hipEventSynchronize(ev)); }
        double t2 = now();
        for (int i = 0; i < K; ++i) {
            hipLaunchKernelGGL(empty, 1, 64, 0, s);
            CK(hipStreamWriteValue32(s, (void *)flag, ++seq, 0));
            while (*flag != seq) __builtin_ia32_pause();
        }
        double t3 = now();
        printf("%-5s StreamSynchronize %6.2f us | EventSynchronize %6.2f us | WriteValue32 spin %6.2f us\n", m,
               (t1 - t0) / K * 1e6, (t2 - t1) / K * 1e6, (t3 - t2) / K * 1e6);
    }
    return 0;
}

// sync_ext.hip -- completion of a synchronous call without the extra
// dispatch: hipStreamWriteValue32 (what the library's completion word uses)
// is itself a blit kernel (__amd_rocclr_streamOpsWrite in the rocprofv3
// trace), so every synchronous MPI_Reduce_local costs two dispatches.
// hipExtLaunchKernel can bind a stop event to the kernel's own dispatch; this
// A/B times, per call, launch + wait for
//   flag    launch, hipStreamWriteValue32, host spin on the word (product);
//   extq    hipExtLaunchKernel(stop event), spin on hipEventQuery;
//   extsync hipExtLaunchKernel(stop event), hipEventSynchronize;
//   recq    launch, hipEventRecord, spin on hipEventQuery;
// for an empty kernel and for a 256 MiB fp32 a += b streaming kernel
// (4 rotating pairs), under hipDeviceScheduleSpin and Auto.
//   hipcc --offload-arch=gfx950 -O2 -o tools/sync_ext tools/sync_ext.hip
//   ./tools/sync_ext <auto|spin>
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(2);} } while (0)

__global__ void empty(const float *, float *, unsigned) {}

typedef float f4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void add4(const float *in, float *io, unsigned nvec) {
    const unsigned base = blockIdx.x * 1024u;   // 4 vectors per lane, 16 KiB per operand per WG
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const unsigned i = base + u * 256 + threadIdx.x;
        if (i < nvec) {
            f4 a = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(io) + i);
            f4 b = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(in) + i);
            __builtin_nontemporal_store(a + b, reinterpret_cast<f4 *>(io) + i);
        }
    }
}

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char **argv) {
    const char *m = argc > 1 ? argv[1] : "auto";
    CK(hipSetDeviceFlags(!strcmp(m, "spin") ? hipDeviceScheduleSpin : hipDeviceScheduleAuto));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t ev, evt;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    CK(hipEventCreate(&evt));
    volatile unsigned *flag;
    CK(hipHostMalloc((void **)&flag, 64, hipHostMallocCoherent | hipHostMallocMapped));
    *flag = 0;
    unsigned seq = 0;
    const size_t n = 64ull << 20;   // floats per operand (256 MiB)
    const unsigned nvec = (unsigned)(n / 4);
    std::vector<float *> bufs(8);
    for (auto &b : bufs) { CK(hipMalloc(&b, n * 4)); CK(hipMemset(b, 0, n * 4)); }
    CK(hipDeviceSynchronize());

    for (int big = 0; big < 2; ++big) {
        const int K = big ? 200 : 3000;
        const unsigned grid = big ? (nvec + 1023) / 1024 : 1;
        void (*kern)(const float *, float *, unsigned) = big ? add4 : empty;
        auto in = [&](int i) { return (const float *)bufs[2 * (i & 3)]; };
        auto io = [&](int i) { return bufs[2 * (i & 3) + 1]; };
        for (int r = 0; r < 3; ++r) {
            double t[5];
            // flag
            for (int i = 0; i < 20; ++i) { hipLaunchKernelGGL(kern, grid, 256, 0, s, in(i), io(i), nvec); CK(hipStreamSynchronize(s)); }
            t[0] = now();
            for (int i = 0; i < K; ++i) {
                hipLaunchKernelGGL(kern, grid, 256, 0, s, in(i), io(i), nvec);
                CK(hipStreamWriteValue32(s, (void *)flag, ++seq, 0));
                while (*flag != seq) __builtin_ia32_pause();
            }
            t[1] = now();
            // extq (timing-disabled event)
            for (int i = 0; i < K; ++i) {
                hipExtLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, s, nullptr, ev, 0, in(i), io(i), nvec);
                while (hipEventQuery(ev) == hipErrorNotReady) __builtin_ia32_pause();
            }
            t[2] = now();
            // extsync (timing event)
            for (int i = 0; i < K; ++i) {
                hipExtLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, s, nullptr, evt, 0, in(i), io(i), nvec);
                CK(hipEventSynchronize(evt));
            }
            t[3] = now();
            // recq
            for (int i = 0; i < K; ++i) {
                hipLaunchKernelGGL(kern, grid, 256, 0, s, in(i), io(i), nvec);
                CK(hipEventRecord(ev, s));
                while (hipEventQuery(ev) == hipErrorNotReady) __builtin_ia32_pause();
            }
            t[4] = now();
            CK(hipGetLastError());
            printf("%-4s %-5s flag %8.2f us | extq %8.2f us | extsync %8.2f us | recq %8.2f us\n", m,
                   big ? "256M" : "empty", (t[1] - t[0]) / K * 1e6, (t[2] - t[1]) / K * 1e6,
                   (t[3] - t[2]) / K * 1e6, (t[4] - t[3]) / K * 1e6);
        }
    }
    return 0;
}

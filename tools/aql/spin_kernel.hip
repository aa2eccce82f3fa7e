// spin_kernel.hip -- a one-wave kernel that waits for a flag word (or a time
// limit) and exits: the "pre-posted" dispatch of tools/aql/cp_latency.cpp.
//   hipcc --offload-arch=gfx950 -O3 --cuda-device-only --no-gpu-bundle-output -c tools/aql/spin_kernel.hip -o tools/aql/spin_kernel.co
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" __global__ void spin_wait(const uint32_t *flag, uint64_t max_ticks) {
    if (threadIdx.x != 0) return;
    const uint64_t t0 = wall_clock64();
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u) {
        if (wall_clock64() - t0 > max_ticks) break;
        __builtin_amdgcn_s_sleep(1);
    }
}

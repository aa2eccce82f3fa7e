// concurrent_kernels.hip -- kernels for tools/aql/concurrent_probe.cpp.
//   keeper: one wave that sleeps-polls a stop word (or a time limit) and exits;
//           it keeps a dispatch in flight on the queue while the host posts the
//           next packet.
//   stamp:  one wave that writes its start time (100 MHz wall clock) and a
//           sequence number to host memory at system scope, so the host sees
//           when a kernel really ran, whatever the CP's in-order bookkeeping.
// Every wait is bounded by max_ticks: a missed stop word ends the keeper.
//   hipcc --offload-arch=gfx950 -O3 --cuda-device-only --no-gpu-bundle-output -c \
//         tools/aql/concurrent_kernels.hip -o tools/aql/concurrent_kernels.co
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" __global__ void keeper(const uint32_t *stop, uint64_t *t_out, uint64_t max_ticks) {
    if (threadIdx.x != 0) return;
    const uint64_t t0 = wall_clock64();
    __hip_atomic_store(&t_out[0], t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    while (__hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u) {
        if (wall_clock64() - t0 > max_ticks) break;
        __builtin_amdgcn_s_sleep(2);
    }
    __hip_atomic_store(&t_out[1], wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

extern "C" __global__ void stamp(uint32_t *flag, uint64_t *t_out, uint32_t seq) {
    if (threadIdx.x != 0) return;
    __hip_atomic_store(&t_out[0], wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

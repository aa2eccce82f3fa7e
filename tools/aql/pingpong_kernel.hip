// pingpong_kernel.hip -- a resident kernel for tools/aql/pingpong.cpp: every
// workgroup waits for command word k, (optionally) fences, counts itself in,
// and the last one in writes k to a response word in host memory.  Measures
// the host -> waves -> host round trip that a resident reducer would pay per
// call instead of the command processor's doorbell path.  Every wait is
// bounded (max_ticks of the 100 MHz wall clock): a missed command ends the
// kernel instead of leaving it resident.
//   hipcc --offload-arch=gfx950 -O3 --cuda-device-only --no-gpu-bundle-output -c tools/aql/pingpong_kernel.hip -o tools/aql/pingpong_kernel.co
#include <hip/hip_runtime.h>
#include <stdint.h>

// fence: 0 none, 1 agent-scope release per workgroup before counting in,
// 2 system-scope release by the last workgroup only.  nwg = the grid's workgroup
// count, passed explicitly: the code object is loaded without hidden arguments
extern "C" __global__ void __launch_bounds__(256) pingpong(const uint32_t *cmd, uint32_t *ctr, uint32_t *resp,
                                                           uint32_t iters, uint32_t fence, uint64_t max_ticks,
                                                           uint32_t nwg) {
    __shared__ uint32_t go;
    for (uint32_t k = 1; k <= iters; ++k) {
        if (threadIdx.x == 0) {
            const uint64_t t0 = wall_clock64();
            uint32_t ok = 1;
            while (__hip_atomic_load(cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < k) {
                if (wall_clock64() - t0 > max_ticks) { ok = 0; break; }
                __builtin_amdgcn_s_sleep(1);
            }
            go = ok;
        }
        __syncthreads();
        if (!go) return;
        if (threadIdx.x == 0) {
            if (fence == 1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            const uint32_t prev = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (prev == k * nwg - 1u) {
                if (fence == 2) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                __hip_atomic_store(resp, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        __syncthreads();
    }
}

// prepost_kernel.hip -- kernels for tools/aql/prepost.cpp: can a reduction
// kernel that is ALREADY queued (pre-posted behind the previous call's kernel,
// its first workgroups resident and waiting on a go word) start a synchronous
// call sooner than the doorbell path (4.3 us from doorbell to dispatch start)?
//
//   plain_tile   the product's lean tile body (mpir_tile_SUM_MPIR_HIP_F32)
//   gated_tile   the same body behind a gate: workgroup 0 (dispatched first)
//                waits for mail->seq >= k with a bounded wait and publishes ONE
//                decision (run / expired) to 8 replicated words, one per XCD
//                (blockIdx % 8) and to the host; every workgroup follows that
//                decision, so a gate that times out never runs part of a grid.
//                The call's arguments come from the mailbox, read after the
//                decision with system-scope loads.
// Every wait is bounded by the 100 MHz wall clock.
//   hipcc --offload-arch=gfx950 -O3 --cuda-device-only --no-gpu-bundle-output -c \
//         -I mpich-pip_amd/csrc/hip tools/aql/prepost_kernel.hip -o tools/aql/prepost_kernel.co
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "reduce_kernels.hpp"

using namespace mpir_hip;

struct Mail {
    uint64_t in, io, vbytes, keep;
    uint32_t seq;
};

extern "C" __global__ __launch_bounds__(kThreads) void plain_tile(const char *in, char *io, uint64_t vbytes,
                                                                  uint64_t keep) {
    const uint64_t base = (uint64_t)blockIdx.x * kTileBytes;
    if (base >= vbytes) return;
    reduce_tile<OpSum, float>(in, io, base, vbytes, keep);
}

__device__ __forceinline__ uint64_t ld64_sys(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

extern "C" __global__ __launch_bounds__(kThreads) void gated_tile(const Mail *mail, uint32_t *dec, uint32_t *outcome,
                                                                  uint32_t k, uint64_t lead_ticks,
                                                                  uint64_t follow_ticks, uint32_t poll_sleep) {
    __shared__ uint64_t s_in, s_io, s_vb, s_keep;
    __shared__ uint32_t s_run;
    if (threadIdx.x == 0) {
        if (blockIdx.x == 0) {
            const uint64_t t0 = wall_clock64();
            uint32_t run = 0;
            for (;;) {
                if (__hip_atomic_load(&mail->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= k) { run = 1; break; }
                if (wall_clock64() - t0 > lead_ticks) break;
                __builtin_amdgcn_s_sleep(1);
            }
            const uint32_t v = (k << 1) | run;
#pragma unroll
            for (int r = 0; r < 8; ++r) __hip_atomic_store(dec + r * 32, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(outcome, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        const uint32_t *my = dec + (blockIdx.x & 7) * 32;
        const uint64_t t0 = wall_clock64();
        uint32_t v;
        for (;;) {
            v = __hip_atomic_load(my, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if ((v >> 1) == k) break;
            if (wall_clock64() - t0 > follow_ticks) { v = k << 1; break; }   // cannot happen: leader decides first
            for (uint32_t i = 0; i < poll_sleep; ++i) __builtin_amdgcn_s_sleep(8);
        }
        s_run = v & 1;
        if (v & 1) {
            s_in = ld64_sys(&mail->in);
            s_io = ld64_sys(&mail->io);
            s_vb = ld64_sys(&mail->vbytes);
            s_keep = ld64_sys(&mail->keep);
        }
    }
    __syncthreads();
    if (!s_run) return;
    const uint64_t base = (uint64_t)blockIdx.x * kTileBytes;
    if (base >= s_vb) return;
    reduce_tile<OpSum, float>((const char *)s_in, (char *)s_io, base, s_vb, s_keep);
}

// Measurement only (no single decision): every workgroup polls the host-written
// sequence word of its XCD (8 replicas, 128 B apart) -- the gate's best case.
extern "C" __global__ __launch_bounds__(kThreads) void direct_gate_tile(const uint32_t *seqs, const Mail *mail,
                                                                        uint32_t k, uint64_t ticks, uint32_t poll_sleep) {
    __shared__ uint64_t s_in, s_io, s_vb, s_keep;
    __shared__ uint32_t s_run;
    if (threadIdx.x == 0) {
        const uint32_t *my = seqs + (blockIdx.x & 7) * 32;
        const uint64_t t0 = wall_clock64();
        uint32_t run = 0;
        for (;;) {
            if (__hip_atomic_load(my, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= k) { run = 1; break; }
            if (wall_clock64() - t0 > ticks) break;
            for (uint32_t i = 0; i < poll_sleep; ++i) __builtin_amdgcn_s_sleep(8);
        }
        s_run = run;
        if (run) {
            s_in = ld64_sys(&mail->in);
            s_io = ld64_sys(&mail->io);
            s_vb = ld64_sys(&mail->vbytes);
            s_keep = ld64_sys(&mail->keep);
        }
    }
    __syncthreads();
    if (!s_run) return;
    const uint64_t base = (uint64_t)blockIdx.x * kTileBytes;
    if (base >= s_vb) return;
    reduce_tile<OpSum, float>((const char *)s_in, (char *)s_io, base, s_vb, s_keep);
}

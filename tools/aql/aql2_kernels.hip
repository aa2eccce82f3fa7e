// aql2_kernels.hip -- kernels for tools/aql/aql2.cpp, built twice: into the
// host tool (HIP launches) and as a device-only code object (direct AQL
// dispatch).  The fp32 SUM tile body of the product (16 KiB per operand per
// 256-thread workgroup, nt loads, issue gap) with three store/completion forms:
//   a2_nt     nt stores (the product at 256 MiB)
//   a2_hyb    nt stores, sc1 (write-through) stores from workgroup `sc1_from` on
//   a2_self   sc1 stores + a sharded completion counter; the workgroup that
//             completes the last shard writes `seq` to a host word
// Each records wall_clock64() at entry and exit of thread 0 into ts[2*block],
// when ts is non-null, so the host can split a call into GPU body and gap.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t a2u32x4 __attribute__((ext_vector_type(4)));
typedef float a2f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void a2_gap() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 0");
    __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void a2_body(const char *in, char *io, uint64_t vbytes, bool sc1) {
    const uint64_t base = (uint64_t)blockIdx.x * 16384u;
    if (base >= vbytes) return;
    const uint64_t left = vbytes - base;
    const int nrec = (int)(left < 16384u ? left : 16384u);
    __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void *)(in + base), 0, nrec, 0x00020000);
    __amdgpu_buffer_rsrc_t rio = __builtin_amdgcn_make_buffer_rsrc((void *)(io + base), 0, nrec, 0x00020000);
    const int t = (int)threadIdx.x;
    const int wb = (t >> 6) * 4096 + (t & 63) * 16;
    a2u32x4 a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        a[u] = __builtin_amdgcn_raw_buffer_load_b128(rio, wb + u * 1024, 0, 2);
        b[u] = __builtin_amdgcn_raw_buffer_load_b128(rin, wb + u * 1024, 0, 2);
        if (u < 3) a2_gap();
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        a2f32x4 r = __builtin_bit_cast(a2f32x4, a[u]) + __builtin_bit_cast(a2f32x4, b[u]);
        if (sc1) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(a2u32x4, r), rio, wb + u * 1024, 0, 16);
        else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(a2u32x4, r), rio, wb + u * 1024, 0, 2);
    }
}

__device__ __forceinline__ void a2_ts(uint64_t *ts, int which) {
    if (ts && threadIdx.x == 0) ts[2 * blockIdx.x + which] = (uint64_t)wall_clock64();
}

// kernarg visibility probe: no pointer comes from the kernarg segment
__device__ uint64_t a2_probe_out[2];
extern "C" __global__ __launch_bounds__(256) void a2_probe(uint64_t a, uint64_t b) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        a2_probe_out[0] = a;
        a2_probe_out[1] = b;
    }
}

extern "C" __global__ __launch_bounds__(256) void a2_empty(const char *, char *, uint64_t, uint64_t *) {}

extern "C" __global__ __launch_bounds__(256) void a2_nt(const char *in, char *io, uint64_t vbytes, uint64_t *ts) {
    a2_ts(ts, 0);
    a2_body(in, io, vbytes, false);
    a2_ts(ts, 1);
}

extern "C" __global__ __launch_bounds__(256) void a2_hyb(const char *in, char *io, uint64_t vbytes, uint64_t *ts,
                                                           uint32_t sc1_from) {
    a2_ts(ts, 0);
    a2_body(in, io, vbytes, blockIdx.x >= sc1_from);
    a2_ts(ts, 1);
}

// sc1 stores in workgroups with (blockIdx % m) < k: a mix spread over the launch
extern "C" __global__ __launch_bounds__(256) void a2_mod(const char *in, char *io, uint64_t vbytes, uint64_t *ts,
                                                           uint32_t m, uint32_t k) {
    a2_ts(ts, 0);
    a2_body(in, io, vbytes, (blockIdx.x % m) < k);
    a2_ts(ts, 1);
}

// (the grid size is an explicit argument: gridDim would need the hidden
// kernel arguments, which a direct AQL dispatch does not fill)
extern "C" __global__ __launch_bounds__(256) void a2_self(const char *in, char *io, uint64_t vbytes, uint64_t *ts,
                                                            uint32_t *cnt, uint32_t nsh, uint32_t *hflag, uint32_t seq,
                                                            uint32_t ngroups) {
    a2_ts(ts, 0);
    a2_body(in, io, vbytes, true);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t sh = blockIdx.x % nsh;
        const uint32_t expect = ngroups / nsh + (sh < ngroups % nsh ? 1u : 0u);
        const uint32_t old = __hip_atomic_fetch_add(cnt + sh * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old + 1 == expect) {
            __hip_atomic_store(cnt + sh * 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t top = __hip_atomic_fetch_add(cnt + nsh * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (top + 1 == nsh) {
                __hip_atomic_store(cnt + nsh * 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(hflag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
    a2_ts(ts, 1);
}

// ---- a2_selfh: the last `nlate` workgroups store sc1 (write-through), the
// others nt; completion signalled from inside the kernel.  Control block
// (uint32 words, one 128-byte line each): DONE[64] late-completion shards, TOP,
// EARLY[64] early-completion shards, CLAIM/WBOK/SEEN[16] per XCC.
//  * early workgroup: stores acknowledged -> SEEN[xcc] = 1 -> EARLY[b % 64] += 1
//  * the first late workgroup on each XCC (CLAIM) waits until every early
//    workgroup is counted, then writes its XCC's L2 back (agent release:
//    buffer_wbl2) and sets WBOK[xcc]
//  * every late workgroup: stores acknowledged -> DONE shard; the workgroup
//    completing the last shard (FINAL) checks that every XCC that ran an early
//    workgroup has WBOK, resets the block and writes seq to the host word --
//    or seq | 0x80000000 (host falls back to a stream wait; block not reset)
#define A2_LINE 32u
#define A2_DONE(s) ((s) * A2_LINE)
#define A2_TOP (64u * A2_LINE)
#define A2_EARLY(s) ((65u + (s)) * A2_LINE)
#define A2_CLAIM(x) ((129u + (x)) * A2_LINE)
#define A2_WBOK(x) ((145u + (x)) * A2_LINE)
#define A2_SEEN(x) ((161u + (x)) * A2_LINE)
#define A2_CTL_WORDS (177u * A2_LINE)

__device__ __forceinline__ uint32_t a2_ld(uint32_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void a2_st(uint32_t *p, uint32_t v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ uint32_t a2_add(uint32_t *p, uint32_t v) { return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ uint32_t a2_wave_sum(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

extern "C" __global__ __launch_bounds__(256) void a2_selfh(const char *in, char *io, uint64_t vbytes, uint64_t *ts,
                                                             uint32_t *ctl, uint32_t *hflag, uint32_t seq,
                                                             uint32_t ngroups, uint32_t from) {
    a2_ts(ts, 0);
    const bool late = blockIdx.x >= from;
    a2_body(in, io, vbytes, late);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x < 64) {
        const uint32_t lane = threadIdx.x;
        const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u;   // HW_REG_XCC_ID[3:0]
        if (!late) {
            if (lane == 0) {
                if (a2_ld(ctl + A2_SEEN(xcc)) == 0) a2_st(ctl + A2_SEEN(xcc), 1u);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                a2_add(ctl + A2_EARLY(blockIdx.x % 64u), 1u);
            }
        } else {
            uint32_t wber = 0;
            if (lane == 0 && from > 0 && a2_ld(ctl + A2_CLAIM(xcc)) == 0)
                wber = __hip_atomic_exchange(ctl + A2_CLAIM(xcc), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
            wber = __shfl(wber, 0, 64);
            if (wber) {
                bool all = false;
                for (int it = 0; it < (1 << 18); ++it) {            // bounded: on timeout, no WBOK (host falls back)
                    if (a2_wave_sum(a2_ld(ctl + A2_EARLY(lane))) == from) { all = true; break; }
                    __builtin_amdgcn_s_sleep(1);
                }
                if (all) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    if (lane == 0) a2_st(ctl + A2_WBOK(xcc), 1u);
                }
            }
            uint32_t fin = 0;
            if (lane == 0) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const uint32_t nlate = ngroups - from;
                const uint32_t li = blockIdx.x - from, sh = li % 64u;
                const uint32_t expect = nlate / 64u + (sh < nlate % 64u ? 1u : 0u);
                if (a2_add(ctl + A2_DONE(sh), 1u) + 1 == expect) {
                    a2_st(ctl + A2_DONE(sh), 0u);
                    const uint32_t nsh = nlate < 64u ? nlate : 64u;
                    if (a2_add(ctl + A2_TOP, 1u) + 1 == nsh) {
                        a2_st(ctl + A2_TOP, 0u);
                        fin = 1;
                    }
                }
            }
            fin = __shfl(fin, 0, 64);
            if (fin) {
                const uint32_t esum = a2_wave_sum(a2_ld(ctl + A2_EARLY(lane)));
                const bool uncovered = lane < 16 && a2_ld(ctl + A2_SEEN(lane)) != 0 && a2_ld(ctl + A2_WBOK(lane)) == 0;
                const bool ok = esum == from && __ballot(uncovered) == 0;
                if (ok) {
                    a2_st(ctl + A2_EARLY(lane), 0u);
                    if (lane < 16) {
                        a2_st(ctl + A2_CLAIM(lane), 0u);
                        a2_st(ctl + A2_WBOK(lane), 0u);
                        a2_st(ctl + A2_SEEN(lane), 0u);
                    }
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (lane == 0) __hip_atomic_store(hflag, ok ? seq : (seq | 0x80000000u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
    a2_ts(ts, 1);
}

// ---- a2_loop: a grid of `gridDim` workgroups, each walking tiles
// b, b + G, b + 2G, ... (G = ngroups), the same tile body per iteration; sc1
// stores for tiles >= sc1_from.  Shape test for amortising a per-workgroup
// completion epilogue over several tiles.
__device__ __forceinline__ void a2_tile_at(const char *in, char *io, uint64_t vbytes, uint64_t tile, bool sc1) {
    const uint64_t base = tile * 16384u;
    const uint64_t left = vbytes - base;
    const int nrec = (int)(left < 16384u ? left : 16384u);
    __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void *)(in + base), 0, nrec, 0x00020000);
    __amdgpu_buffer_rsrc_t rio = __builtin_amdgcn_make_buffer_rsrc((void *)(io + base), 0, nrec, 0x00020000);
    const int t = (int)threadIdx.x;
    const int wb = (t >> 6) * 4096 + (t & 63) * 16;
    a2u32x4 a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        a[u] = __builtin_amdgcn_raw_buffer_load_b128(rio, wb + u * 1024, 0, 2);
        b[u] = __builtin_amdgcn_raw_buffer_load_b128(rin, wb + u * 1024, 0, 2);
        if (u < 3) a2_gap();
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        a2f32x4 r = __builtin_bit_cast(a2f32x4, a[u]) + __builtin_bit_cast(a2f32x4, b[u]);
        if (sc1) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(a2u32x4, r), rio, wb + u * 1024, 0, 16);
        else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(a2u32x4, r), rio, wb + u * 1024, 0, 2);
    }
}

extern "C" __global__ __launch_bounds__(256) void a2_loop(const char *in, char *io, uint64_t vbytes, uint64_t *ts,
                                                            uint32_t ngroups, uint32_t ntiles, uint32_t sc1_from) {
    a2_ts(ts, 0);
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += ngroups) a2_tile_at(in, io, vbytes, tile, tile >= sc1_from);
    a2_ts(ts, 1);
}

extern "C" __global__ void a2_ts_clear_ends(uint64_t *ts, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) ts[2 * i + 1] = 0;
}

// direct_tiles.hip -- device-only code object lib/libmpir_hip_tiles.hsaco for
// the direct AQL dispatch of synchronous calls (direct_dispatch.hip).
//
// Five extern "C" kernels per (op, element class) whose launcher is
// launch_reduce (reg<Op, T> in the reg_*.hip units: every op on the integer,
// real, complex, pair and x87 classes; not the 32-byte classes or REPLACE) --
// one per kind of plan_reduce's launch plan (reduce_kernels.hpp), under plain
// names the host looks up, each taking one 128-byte kernarg slot and each in
// an unchecked and a checked form (below):
//   mpir_tile_<op>_<elem>    k_reduce_tile_lean's body (LeanArgs):
//                            16 B-aligned operands of 16 B multiples;
//   mpir_tilex_<op>_<elem>   k_reduce_tile's body (TileArgs): equal
//                            alignment mod 16, head / tail elements by
//                            workgroup 0;
//   mpir_tiles_<op>_<elem>   k_reduce_shift's body (ShiftArgs): unequal
//                            alignment mod 16, two tiles or more;
//   mpir_elems_<op>_<elem>   k_reduce_elems<NATURAL = true / false> (ElemsArgs,
//   mpir_elemsu_<op>_<elem>  the grid stride an argument): the rest.
// None reads a hidden argument (no gridDim), so a bare AQL packet launches it.
#include "kernel_table.hpp"

using namespace mpir_hip;

// Every kernel takes one 128-byte kernarg slot (KargSlot, reduce_kernels.hpp):
// the plan's argument bytes in words 0-5 and 8-13, the device's error word in
// word 6, a nonce in words 7 and 15 (one copy per 64-byte half).  Each plan
// kind comes twice:
//   mpir_<kind>_*    reads its arguments as they stand.  The host dispatches
//                    it on a kernarg-cache hit whose slot an earlier, checked
//                    dispatch has already read back complete: nothing is
//                    written for the call.
//   mpir_c<kind>_*   checked.  The host wrote the slot for this call through
//                    the BAR -- the argument words, an sfence, the nonce (the
//                    packet's queue index + 1, which the CP hands every wave
//                    as its dispatch id), an HDP flush never read back -- and
//                    then rang the doorbell.  A workgroup accepts its slot when
//                    the halves holding its arguments carry a nonce >= its
//                    dispatch id + 1 (a later dispatch of the same arguments
//                    may have re-stamped the slot meanwhile); one that still
//                    finds an older line (the flush not yet through, a copy an
//                    earlier dispatch left in its XCD's L2) re-reads past the
//                    caches until the write shows.  If the nonce never
//                    arrives (2 s: only a test hook's held-back write, or a
//                    dead host) the workgroup touches nothing and sets the
//                    error word, and the call fails instead of combining stale
//                    arguments.
// Measured against round 2's single protocol (tools/aql/kslot_ab.cpp,
// interleaved call by call, profiles/archive/r03/kslot_ab.log): checking on every call
// cost hits ~1.2 us (the heavier prologue and the per-call stamp), so hits stay
// unchecked.

// the dispatch id (SGPRs the CP fills from the packet's queue index; clang
// exposes the LLVM intrinsic without a builtin)
extern "C" __device__ uint64_t mpir_dispatch_id(void) __asm("llvm.amdgcn.dispatch.id");

template <class A>
constexpr bool kTwoHalves = sizeof(A) > 48;     // words 0-5 hold 48 bytes

template <class A>
__device__ __forceinline__ void unpack_args(const KargSlot &s, A *a) {
    static_assert(sizeof(A) <= kSlotArgBytes, "plan arguments exceed the kernarg slot");
    uint64_t words[12];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        words[i] = s.w[i];
        words[6 + i] = s.w[8 + i];
    }
    __builtin_memcpy(a, words, sizeof(A));
}

template <class A>
__device__ __forceinline__ bool slot_fresh(const KargSlot &s, uint64_t want) {
    return s.w[7] >= want && (!kTwoHalves<A> || s.w[15] >= want);
}

// checked: the slot's arguments once they carry this dispatch's nonce, or false
// (error word set) when they never arrived
template <class A>
__device__ __forceinline__ bool checked_args(KargSlot s, A *a) {
    const uint64_t want = mpir_dispatch_id() + 1;
    // the words in registers before the check, in one statement: the loads
    // issue together and cost one scalar round trip, as a plain argument load
    if constexpr (kTwoHalves<A>)
        asm volatile("" : "+s"(s.w[0]), "+s"(s.w[1]), "+s"(s.w[2]), "+s"(s.w[3]), "+s"(s.w[4]), "+s"(s.w[5]),
                     "+s"(s.w[7]), "+s"(s.w[8]), "+s"(s.w[9]), "+s"(s.w[10]), "+s"(s.w[11]), "+s"(s.w[12]),
                     "+s"(s.w[13]), "+s"(s.w[15]));
    else
        asm volatile("" : "+s"(s.w[0]), "+s"(s.w[1]), "+s"(s.w[2]), "+s"(s.w[3]), "+s"(s.w[7]));
    if (__builtin_expect(!slot_fresh<A>(s, want), 0)) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();      // 100 MHz
        const uint64_t *g = (const uint64_t *)(uintptr_t)__builtin_amdgcn_kernarg_segment_ptr();
        bool ok = false;
        while (!ok) {
            // the writes normally land within a few us of the doorbell; a host
            // thread preempted between the doorbell and its writes (a CPU-quota
            // throttle lasts up to the 100 ms period) makes the wait long, and
            // the workgroups then poll every ~3 us instead of every ~60 ns
            if (__builtin_amdgcn_s_memrealtime() - t0 < 5000)        // 50 us
                __builtin_amdgcn_s_sleep(2);
            else
                __builtin_amdgcn_s_sleep(127);
            __builtin_amdgcn_s_dcache_inv();
            asm volatile("buffer_inv sc0 sc1" ::: "memory");
            for (int i = 0; i < 16; ++i) s.w[i] = __builtin_nontemporal_load(g + i);
            ok = slot_fresh<A>(s, want);
            // another workgroup of this dispatch already gave up: so does this
            // one at once (every later resident round would wait its own 2 s)
            if (!ok && __hip_atomic_load(reinterpret_cast<const uint32_t *>(s.w[6]), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_SYSTEM) != 0u)
                return false;
            // 2 s: never landed (the host process stopped or died after ringing)
            if (!ok && __builtin_amdgcn_s_memrealtime() - t0 > 200000000) {
                if (threadIdx.x == 0)
                    __hip_atomic_store(reinterpret_cast<uint32_t *>(s.w[6]), 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
                return false;
            }
        }
    }
    unpack_args(s, a);
    return true;
}

// The nonce protocol needs the CP's dispatch id to be the index the host wrote
// the packet at.  A tool that intercepts the queue (rocprofv3, other
// HSA_TOOLS_LIB users) re-submits the packets to a hardware queue of its own
// whose indices differ; the host dispatches this probe at queue creation
// (direct_dispatch.hip probe_ids) and, when the ids do not match, makes the
// arguments visible before the doorbell instead (flush read back, unchecked
// kernels).  Word 0: where lane 0 stores its dispatch id (vector store).
extern "C" __global__ __launch_bounds__(64) void mpir_probe_dispatch_id(KargSlot ks) {
    if (threadIdx.x == 0)
        __hip_atomic_store(reinterpret_cast<uint64_t *>(ks.w[0]), mpir_dispatch_id(), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

// The hash of this code object's sources (Makefile TILES_HASH), as bytes in
// the file: direct_dispatch.hip loads the code object only if it matches the
// hash libmpir_hip.so was built with, so a stale .hsaco beside a newer library
// leaves the direct path off instead of running other kernel bodies.
#ifndef MPIR_TILES_HASH
#define MPIR_TILES_HASH "unknown"
#endif
extern "C" __attribute__((used)) __device__ const char mpir_tiles_build_id[] = "mpir-tiles-build:" MPIR_TILES_HASH;

// unchecked: the plan's argument words as they stand, all loaded up front in
// one statement (left to itself the compiler sinks the words the tile reads
// after its early exit into a second, dependent scalar round trip)
template <class A>
__device__ __forceinline__ bool plain_args(KargSlot s, A *a) {
    if constexpr (kTwoHalves<A>)
        asm volatile("" : "+s"(s.w[0]), "+s"(s.w[1]), "+s"(s.w[2]), "+s"(s.w[3]), "+s"(s.w[4]), "+s"(s.w[5]),
                     "+s"(s.w[8]), "+s"(s.w[9]), "+s"(s.w[10]), "+s"(s.w[11]), "+s"(s.w[12]), "+s"(s.w[13]));
    else if constexpr (sizeof(A) <= 32)
        asm volatile("" : "+s"(s.w[0]), "+s"(s.w[1]), "+s"(s.w[2]), "+s"(s.w[3]));
    else
        asm volatile("" : "+s"(s.w[0]), "+s"(s.w[1]), "+s"(s.w[2]), "+s"(s.w[3]), "+s"(s.w[4]), "+s"(s.w[5]));
    unpack_args(s, a);
    return true;
}

// A checked dispatch of a grid smaller than the chip's 8 XCDs is padded to 8
// workgroups (direct_dispatch.hip kMinCheckedGroups), so that every XCD's L2
// has read the slot's fresh line before later cache hits run the unchecked
// kernel on any XCD.  The padding workgroups check the slot and exit: the tile
// and shift kernels skip tiles past the region already; the grid-stride
// element kernels would re-process elements, so they stop a workgroup past the
// grid the stride was sized for.
__device__ __forceinline__ bool in_grid(const ElemsArgs &a) {
    return (uint64_t)blockIdx.x * kThreads < a.stride;
}

#define MPIR_DIRECT_KIND(PFX, GET, OPN, OP, E, T)                                                       \
    extern "C" __global__ __launch_bounds__(kThreads) void mpir_##PFX##tile_##OPN##_##E(KargSlot ks) {   \
        LeanArgs a;                                                                                       \
        if (GET(ks, &a)) reduce_tile<OP, T>(a.in, a.io, blockIdx.x, a.vbytes, a.keep);                    \
    }                                                                                                     \
    extern "C" __global__ __launch_bounds__(kThreads) void mpir_##PFX##tilex_##OPN##_##E(KargSlot ks) {  \
        TileArgs<T> a;                                                                                    \
        if (GET(ks, &a)) reduce_tile_body<OP, T>(a);                                                      \
    }                                                                                                     \
    extern "C" __global__ __launch_bounds__(kThreads) void mpir_##PFX##tiles_##OPN##_##E(KargSlot ks) {  \
        ShiftArgs<T> a;                                                                                   \
        if (GET(ks, &a)) reduce_shift_body<OP, T>(a);                                                     \
    }                                                                                                     \
    extern "C" __global__ __launch_bounds__(kThreads) void mpir_##PFX##elems_##OPN##_##E(KargSlot ks) {  \
        ElemsArgs a;                                                                                      \
        if (GET(ks, &a) && in_grid(a)) reduce_elems<OP, T, true>(a.in, a.io, a.n, a.stride);              \
    }                                                                                                     \
    extern "C" __global__ __launch_bounds__(kThreads) void mpir_##PFX##elemsu_##OPN##_##E(KargSlot ks) { \
        ElemsArgs a;                                                                                      \
        if (GET(ks, &a) && in_grid(a)) reduce_elems<OP, T, false>(a.in, a.io, a.n, a.stride);             \
    }

#define MPIR_DIRECT_TILE(OPN, OP, E, T) MPIR_DIRECT_KIND(, plain_args, OPN, OP, E, T) \
                                        MPIR_DIRECT_KIND(c, checked_args, OPN, OP, E, T)

// the (op, class) matrix of reg_sum_prod / reg_max_min / reg_logic / reg_pairs_x87
#define X(E, T) MPIR_DIRECT_TILE(SUM, OpSum, E, T) MPIR_DIRECT_TILE(PROD, OpProd, E, T)
FOR_INTS(X) FOR_REALS(X) FOR_CPLX(X) X(MPIR_HIP_F80, x80)
#undef X
#define X(E, T) MPIR_DIRECT_TILE(MAX, OpMax, E, T) MPIR_DIRECT_TILE(MIN, OpMin, E, T)
FOR_INTS(X) FOR_REALS(X) X(MPIR_HIP_F80, x80)
#undef X
#define X(E, T) MPIR_DIRECT_TILE(LAND, OpLand, E, T) MPIR_DIRECT_TILE(LOR, OpLor, E, T) \
                MPIR_DIRECT_TILE(BAND, OpBand, E, T) MPIR_DIRECT_TILE(BOR, OpBor, E, T) \
                MPIR_DIRECT_TILE(BXOR, OpBxor, E, T)
FOR_INTS(X)
#undef X
#define X(E, T) MPIR_DIRECT_TILE(LXOR, OpLxor, E, T)
FOR_INTS(X) FOR_REALS(X) X(MPIR_HIP_F80, x80)
#undef X
#define X(E, T) MPIR_DIRECT_TILE(MAXLOC, OpMaxloc, E, T) MPIR_DIRECT_TILE(MINLOC, OpMinloc, E, T)
FOR_PAIRS(X)
#undef X

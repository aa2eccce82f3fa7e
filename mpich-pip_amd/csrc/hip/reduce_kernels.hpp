// reduce_kernels.hpp -- gfx950 streaming kernels for MPIR_Reduce_local.
//
// The combine is element-wise: 2 reads + 1 write per element, arithmetic
// intensity <= 1/12 op/B for fp32, so the roofline is HBM bandwidth and MFMA
// is irrelevant.  The shape below is the winner of tools/bw_sweep*.hip on
// MI355X (256 MiB/operand fp32 SUM, profiles/ and DESIGN.md §Kernels):
//
//   * one 16 KiB tile per operand per 256-thread workgroup (4 x 16 B per lane,
//     lane-contiguous 1 KiB wave-instructions, each wave a contiguous 4 KiB
//     of the tile), no grid-stride loop: the grid
//     is vbytes / 16 KiB workgroups (16384 at 256 MiB), which keeps every CU's
//     queue deep and the DRAM pages of a tile together;
//   * all 8 loads of a lane issued before the first combine (latency hiding
//     by ILP + 8 waves/CU of TLP), with a one-instruction issue gap after
//     each (inout, in) pair (issue_gap below: 0.810 -> 0.830-0.841 of peak);
//   * buffer_load/store_dwordx4 with the `nt` cache policy (aux = 2) on both
//     operands and on the store (a result of at most 64 MiB is stored sc1
//     instead, so it stays in the Infinity Cache for its next reader:
//     kKeepBytes below): streamed-once data should not displace L2 / Infinity
//     Cache lines; measured 0.81 of the 8 TB/s HBM peak vs 0.70 for
//     default-policy loads and 0.63 for a grid-stride loop (before the gap);
//   * the buffer descriptor covers exactly this tile's bytes, so the ragged
//     last tile needs no branch: out-of-range loads return 0 and out-of-range
//     stores are dropped by the hardware range check.
// The < 16 B head (to 16 B-align inout) and tail are handled element-wise by
// workgroup 0 (k_reduce_tile), so a call is always exactly one launch; without
// them the launch takes k_reduce_tile_lean.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "reduce_ops.hpp"

namespace mpir_hip {

constexpr int kThreads = 256;
constexpr int kVecPerLane = 4;
constexpr uint32_t kTileBytes = kThreads * kVecPerLane * 16;  // 16 KiB per operand
constexpr int kCachePolicyNT = 2;                             // aux bit: nt
constexpr int kCachePolicySC1 = 16;                           // aux bit: sc1 (device scope)
// Store policy (keep_for(), hip_reduce.hip): a result of at most `keep` bytes
// (MPIR_CVAR_REDUCE_LOCAL_KEEP_MB, default kKeepBytes = 64 MiB) is stored with
// sc1 instead of nt, a larger one nt.  An sc1 store allocates in the 256 MB
// Infinity Cache (MALL), an nt store bypasses it; so a result of at most 64 MiB
// stays there for its next reader (the next schedule step, the RCCL send of a
// block, the D2H copy of a staged chunk): 64 MiB re-read within ~256 MiB of
// traffic 27.0 vs 33.2 us (tools/archive/sync_store_ab.hip,
// profiles/archive/r01s4_sync_store_ab.log).  With nothing re-read the two policies
// are within noise at <= 64 MiB, and at 256 MiB sc1 on any part of the result
// costs ~1 us (profiles/archive/r02/pairs_ab.log: a "last 64 MiB sc1" variant only won
// where the bench's own rotation let the next call but three re-read that tail
// from the MALL; withdrawn).  The kernels take the per-call `keep` and store
// sc1 the tiles in the last `keep` bytes: keep = vbytes (all) or 0 (none).
// Nothing else changes: the bytes reach HBM either way (MALL is memory-side).
constexpr uint64_t kKeepBytes = 64ull << 20;
uint64_t keep_bytes();               // MPIR_CVAR_REDUCE_LOCAL_KEEP_MB (hip_reduce.hip)
uint64_t keep_for(uint64_t vbytes);  // the per-call `keep` argument of the kernels

// true for a tile that starts inside the last `keep` bytes of a `vbytes` region
__device__ __forceinline__ bool keep_tile(uint64_t base, uint64_t vbytes, uint64_t keep) {
    return vbytes - base <= keep;
}


typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// one 16-byte store; `keep` (uniform per workgroup: keep_tile) picks sc1
__device__ __forceinline__ void store16(u32x4 v, __amdgpu_buffer_rsrc_t r, int off, bool keep) {
    if (keep) __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kCachePolicySC1);
    else __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kCachePolicyNT);
}

template <class T>
struct Pack16 {
    static_assert(16 % sizeof(T) == 0, "element must divide 16 bytes");
    T e[16 / sizeof(T)];
};

template <class T>
struct TileArgs {
    const char *in;     // 16 B-aligned vector region of inbuf
    char *io;           // 16 B-aligned vector region of inoutbuf
    uint64_t vbytes;    // bytes in the vector region (multiple of 16)
    const T *head_in;   // elements before the vector region
    T *head_io;
    uint32_t nhead;
    const T *tail_in;   // elements after the vector region
    T *tail_io;
    uint32_t ntail;
    uint64_t keep;      // keep_for(vbytes): the last `keep` bytes are stored sc1
};

template <class Op, class T>
__device__ __forceinline__ u32x4 combine16(u32x4 a, u32x4 b) {
    Pack16<T> pa = __builtin_bit_cast(Pack16<T>, a);
    Pack16<T> pb = __builtin_bit_cast(Pack16<T>, b);
    Op op;
    if constexpr (nan_fast<Op, T>::value) {
        // plain IEEE arithmetic (packed where the ISA has it); the x86 NaN
        // rule runs only for lanes whose vector produced a NaN
        Pack16<T> pr;
        bool bad = false;
#pragma unroll
        for (int k = 0; k < (int)(16 / sizeof(T)); ++k) {
            pr.e[k] = Op::raw(pa.e[k], pb.e[k]);
            bad |= isnan_(pr.e[k]);
        }
        if (__builtin_expect(bad, 0)) {
#pragma unroll
            for (int k = 0; k < (int)(16 / sizeof(T)); ++k) pr.e[k] = op(pa.e[k], pb.e[k]);
        }
        return __builtin_bit_cast(u32x4, pr);
    } else {
#pragma unroll
        for (int k = 0; k < (int)(16 / sizeof(T)); ++k) pa.e[k] = op(pa.e[k], pb.e[k]);
        return __builtin_bit_cast(u32x4, pa);
    }
}

// A short issue gap (s_nop 0, pinned in place by scheduling barriers) after
// every (inout, in) pair of 16 B loads.  rocprofv3 kernel trace, 256 MiB fp32
// SUM, same tile otherwise: 119.7 us (0.841 of the HBM peak) vs 124.2 us
// (0.810) with the eight loads back to back (tools/shape_ab.hip,
// profiles/archive/r01s3_shape_ab.log); a gap after every load, or s_nop 3, measured
// the same, s_nop 7 less.
__device__ __forceinline__ void issue_gap() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 0");
    __builtin_amdgcn_sched_barrier(0);
}

// The tile grid sits on kTileBytes boundaries of inoutbuf's ADDRESS, not of
// its start: tile t covers [t * kTileBytes - s, (t + 1) * kTileBytes - s) of the
// vector region, s = io mod kTileBytes, clipped to [0, vbytes).  Operands that
// start off a 16 KiB boundary otherwise put every tile across two 16 KiB
// blocks, every wave's 4 KiB across two 4 KiB blocks (and at 64 B off, every
// 1 KiB access across nine 128 B lines instead of eight): measured at 256 MiB
// (tools/archive/align_sweep.py, profiles/archive/r03/align_sweep.log), both operands 64 B /
// 4 KiB / 8 KiB off a 2 MiB boundary took 125.0 / 124.0 / 128.5 us against
// 120.8 us aligned.  Tile 0 is then the partial block up to the first
// boundary: its lanes below the cut get offsets that wrap past the buffer
// descriptor's range (loads return 0, stores are dropped), like the lanes past
// the end of the last tile.  `in` shares io's offset mod 16 (tile_split), not
// necessarily mod 16 KiB.
__device__ __forceinline__ uint32_t tile_shift(const void *io) {
    return (uint32_t)(reinterpret_cast<uintptr_t>(io) & (kTileBytes - 1));
}

// workgroups of the tile grid over a vector region of vbytes at io
__host__ __device__ inline uint64_t tile_groups(const void *io, uint64_t vbytes) {
    const uint64_t s = reinterpret_cast<uintptr_t>(io) & (kTileBytes - 1);
    const uint64_t g = (vbytes + s + kTileBytes - 1) / kTileBytes;
    return g ? g : 1;
}

// Tile `tile` of the grid: each wave owns a contiguous 4 KiB of it (one 1 KiB
// lane-contiguous access per instruction).
template <class Op, class T>
__device__ __forceinline__ void reduce_tile(const char *in, char *io, uint64_t tile, uint64_t vbytes, uint64_t keepb) {
    const int64_t start = (int64_t)(tile * kTileBytes) - (int64_t)tile_shift(io);
    const uint64_t lo = start > 0 ? (uint64_t)start : 0;
    if (lo >= vbytes) return;
    const uint64_t end = (uint64_t)(start + kTileBytes);
    const int nrec = (int)((end < vbytes ? end : vbytes) - lo);
    const int cut = (int)(lo - start);       // 0, or s for tile 0: lanes below it wrap out of range
    __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void *)(in + lo), 0, nrec, 0x00020000);
    __amdgpu_buffer_rsrc_t rio = __builtin_amdgcn_make_buffer_rsrc((void *)(io + lo), 0, nrec, 0x00020000);
    const int t = (int)threadIdx.x;
    const int wb = (t >> 6) * (kVecPerLane * 1024) + (t & 63) * 16 - cut;
    u32x4 a[kVecPerLane], b[kVecPerLane];
#pragma unroll
    for (int u = 0; u < kVecPerLane; ++u) {
        a[u] = __builtin_amdgcn_raw_buffer_load_b128(rio, wb + u * 1024, 0, kCachePolicyNT);
        b[u] = __builtin_amdgcn_raw_buffer_load_b128(rin, wb + u * 1024, 0, kCachePolicyNT);
        if (u + 1 < kVecPerLane) issue_gap();
    }
    const bool keep = keep_tile(lo, vbytes, keepb);
#pragma unroll
    for (int u = 0; u < kVecPerLane; ++u) store16(combine16<Op, T>(a[u], b[u]), rio, wb + u * 1024, keep);
}

// With head / tail elements (nhead or ntail != 0), workgroup 0 combines them
// after its tile.
template <class Op, class T>
__device__ __forceinline__ void reduce_tile_body(const TileArgs<T> &args) {
    reduce_tile<Op, T>(args.in, args.io, blockIdx.x, args.vbytes, args.keep);
    if (blockIdx.x == 0) {
        Op op;
        const unsigned t = threadIdx.x;
        if (t < args.nhead) args.head_io[t] = op(args.head_io[t], args.head_in[t]);
        else if (t >= 64 && t - 64 < args.ntail) args.tail_io[t - 64] = op(args.tail_io[t - 64], args.tail_in[t - 64]);
    }
}

template <class Op, class T>
__global__ __launch_bounds__(kThreads) void k_reduce_tile(TileArgs<T> args) {
    reduce_tile_body<Op, T>(args);
}

// No head / tail (the common case: 16 B-aligned buffers, bytes a multiple of
// 16): four scalar arguments and nothing after the tile.
template <class Op, class T>
__global__ __launch_bounds__(kThreads) void k_reduce_tile_lean(const char *in, char *io, uint64_t vbytes, uint64_t keep) {
    reduce_tile<Op, T>(in, io, blockIdx.x, vbytes, keep);
}

// inbuf misaligned relative to inoutbuf: (in - io) mod 16 = delta != 0, the
// case of a schedule step whose tmp_buf and recvbuf sub-ranges start at
// different offsets mod 16.  inoutbuf is peeled to 16 B alignment as in
// k_reduce_tile and streamed the same way; inbuf is read as ALIGNED 16-byte
// vectors (lane k loads vector k of the tile, starting delta bytes before the
// operand) and each lane rebuilds its 16 operand bytes from its own vector and
// its neighbour's: a wavefront shuffle (ds_bpermute) hands lane k the vector
// of lane k+1, lane 63 of each wave loads that one itself, and
// v_alignbyte funnels the two at byte offset delta.  The in-buffer descriptor
// ends at the last 16 B vector holding operand bytes; loads past it read 0.
template <int D>
__device__ __forceinline__ u32x4 funnel_d(const uint32_t (&w)[8], uint32_t sh) {
    u32x4 r;
    r.x = __builtin_amdgcn_alignbyte(w[D + 1], w[D + 0], sh);
    r.y = __builtin_amdgcn_alignbyte(w[D + 2], w[D + 1], sh);
    r.z = __builtin_amdgcn_alignbyte(w[D + 3], w[D + 2], sh);
    r.w = __builtin_amdgcn_alignbyte(w[D + 4], w[D + 3], sh);
    return r;
}

// bytes [delta, delta + 16) of the 32-byte concatenation lo:hi (delta uniform)
__device__ __forceinline__ u32x4 funnel16(u32x4 lo, u32x4 hi, uint32_t delta) {
    const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    const uint32_t sh = delta & 3;
    switch (delta >> 2) {
    case 0: return funnel_d<0>(w, sh);
    case 1: return funnel_d<1>(w, sh);
    case 2: return funnel_d<2>(w, sh);
    default: return funnel_d<3>(w, sh);
    }
}

template <class T>
struct ShiftArgs {
    TileArgs<T> t;      // t.in is unused: the in region is in_al + delta
    const char *in_al;  // in region start rounded down to 16 B
    uint32_t delta;     // 1..15
};

template <class Op, class T>
__device__ __forceinline__ void reduce_shift_body(const ShiftArgs<T> &args) {
    const TileArgs<T> &ta = args.t;
    const uint64_t base = (uint64_t)blockIdx.x * kTileBytes;
    if (base < ta.vbytes) {
        const uint64_t left = ta.vbytes - base;
        const int nrec = (int)(left < kTileBytes ? left : kTileBytes);
        // operand bytes from in_al + base on, rounded up to whole 16 B vectors: the
        // range check of a dwordx4 load is per access, so the vector holding the
        // operand's last bytes must be fully in range (an aligned 16 B block never
        // crosses a page, so its bytes past the operand are mapped; they are unused)
        const uint64_t in_left = (args.delta + left + 15) & ~(uint64_t)15;
        const int nrec_in = (int)(in_left < kTileBytes + 16 ? in_left : kTileBytes + 16);
        __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void *)(args.in_al + base), 0, nrec_in, 0x00020000);
        __amdgpu_buffer_rsrc_t rio = __builtin_amdgcn_make_buffer_rsrc((void *)(ta.io + base), 0, nrec, 0x00020000);
        const bool last_lane = (threadIdx.x & 63) == 63;
        // wave-contiguous 4 KiB per wave, as in the aligned tile kernel
        const int wb = ((int)threadIdx.x >> 6) * (kVecPerLane * 1024) + ((int)threadIdx.x & 63) * 16;
        u32x4 a[kVecPerLane], b[kVecPerLane], n63[kVecPerLane];
#pragma unroll
        for (int u = 0; u < kVecPerLane; ++u) {
            const int off = wb + u * 1024;
            a[u] = __builtin_amdgcn_raw_buffer_load_b128(rio, off, 0, kCachePolicyNT);
            b[u] = __builtin_amdgcn_raw_buffer_load_b128(rin, off, 0, kCachePolicyNT);
            // lane 63's neighbour vector: every lane issues the load, the others
            // at an offset past the descriptor's range (returns 0, no memory
            // request) -- a branch here would make the compiler drain vmcnt
            n63[u] = __builtin_amdgcn_raw_buffer_load_b128(rin, last_lane ? off + 16 : 0x40000000, 0, kCachePolicyNT);
            if (u + 1 < kVecPerLane) issue_gap();
        }
#pragma unroll
        for (int u = 0; u < kVecPerLane; ++u) {
            const int off = wb + u * 1024;
            // neighbour from the shuffle, OR the lane-63 load (0 on every other
            // lane): branch-free, so the load cannot be sunk into a branch
            const uint32_t keep = last_lane ? 0u : ~0u;
            u32x4 nb;
            nb.x = (__shfl_down(b[u].x, 1, 64) & keep) | n63[u].x;
            nb.y = (__shfl_down(b[u].y, 1, 64) & keep) | n63[u].y;
            nb.z = (__shfl_down(b[u].z, 1, 64) & keep) | n63[u].z;
            nb.w = (__shfl_down(b[u].w, 1, 64) & keep) | n63[u].w;
            store16(combine16<Op, T>(a[u], funnel16(b[u], nb, args.delta)), rio, off, keep_tile(base, ta.vbytes, ta.keep));
        }
    }
    if (blockIdx.x == 0) {
        Op op;
        const unsigned t = threadIdx.x;
        if (t < ta.nhead) {
            T x = ta.head_io[t], y;
            __builtin_memcpy(&y, reinterpret_cast<const char *>(ta.head_in) + t * sizeof(T), sizeof(T));
            ta.head_io[t] = op(x, y);
        } else if (t >= 64 && t - 64 < ta.ntail) {
            T x = ta.tail_io[t - 64], y;
            __builtin_memcpy(&y, reinterpret_cast<const char *>(ta.tail_in) + (t - 64) * sizeof(T), sizeof(T));
            ta.tail_io[t - 64] = op(x, y);
        }
    }
}

template <class Op, class T>
__global__ __launch_bounds__(kThreads) void k_reduce_shift(ShiftArgs<T> args) {
    reduce_shift_body<Op, T>(args);
}

// General path: inbuf and inoutbuf differ in alignment mod 16 (sub-range
// displacements of arbitrary element counts), or elements are not even
// naturally aligned.  Element-granular, coalesced, grid-stride; the stride
// (grid x kThreads) is an argument, not gridDim, so the direct AQL dispatch
// can launch it without hidden arguments.
template <class Op, class T, bool NATURAL>
__device__ __forceinline__ void reduce_elems(const char *in, char *io, uint64_t n, uint64_t stride) {
    Op op;
    for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) {
        if constexpr (NATURAL) {
            const T *pi = reinterpret_cast<const T *>(in) + i;
            T *po = reinterpret_cast<T *>(io) + i;
            *po = op(*po, *pi);
        } else {
            T x, y;
            __builtin_memcpy(&x, io + i * sizeof(T), sizeof(T));
            __builtin_memcpy(&y, in + i * sizeof(T), sizeof(T));
            x = op(x, y);
            __builtin_memcpy(io + i * sizeof(T), &x, sizeof(T));
        }
    }
}

template <class Op, class T, bool NATURAL>
__global__ __launch_bounds__(kThreads) void k_reduce_elems(const char *in, char *io, uint64_t n, uint64_t stride) {
    reduce_elems<Op, T, NATURAL>(in, io, n, stride);
}

// The tile kernels' split of [in, io) x count into head elements (to 16 B-align
// inoutbuf) / a 16 B vector body / tail elements.  False when the two pointers
// do not share their alignment mod 16 (or are not naturally aligned).
template <class T>
bool tile_split(const void *in_, void *io_, uint64_t count, TileArgs<T> &a) {
    const char *in = static_cast<const char *>(in_);
    char *io = static_cast<char *>(io_);
    const uintptr_t ai = reinterpret_cast<uintptr_t>(in), ao = reinterpret_cast<uintptr_t>(io);
    const uint64_t nbytes = count * sizeof(T);
    const bool natural = (ai % alignof(T) == 0) && (ao % alignof(T) == 0);
    const uint64_t head0 = (16 - (ao & 15)) & 15;
    if (!(natural && ((ai ^ ao) & 15) == 0 && head0 % sizeof(T) == 0)) return false;
    const uint64_t head_bytes = head0 < nbytes ? head0 : nbytes;
    const uint64_t rest = nbytes - head_bytes;
    const uint64_t vbytes = rest & ~(uint64_t)15;
    a.in = in + head_bytes;
    a.io = io + head_bytes;
    a.vbytes = vbytes;
    a.head_in = reinterpret_cast<const T *>(in);
    a.head_io = reinterpret_cast<T *>(io);
    a.nhead = (uint32_t)(head_bytes / sizeof(T));
    a.tail_in = reinterpret_cast<const T *>(in + head_bytes + vbytes);
    a.tail_io = reinterpret_cast<T *>(io + head_bytes + vbytes);
    a.ntail = (uint32_t)((rest - vbytes) / sizeof(T));
    a.keep = keep_for(vbytes);
    return true;
}

// The launch plan of one single-operand reduction: which kernel, its grid and
// its argument bytes.  launch_reduce launches it through HIP; the direct AQL
// dispatch (direct_dispatch.hip) launches the same kernel body from its code
// object -- so both paths treat every call identically.
enum : int {
    kPlanLean = 0,      // k_reduce_tile_lean: 16 B-aligned, 16 B multiple (LeanArgs)
    kPlanFull = 1,      // k_reduce_tile: equal alignment mod 16, head / tail elements (TileArgs)
    kPlanShift = 2,     // k_reduce_shift: unequal alignment, >= 2 tiles (ShiftArgs)
    kPlanElems = 3,     // k_reduce_elems<NATURAL = true> (ElemsArgs)
    kPlanElemsU = 4,    // k_reduce_elems<NATURAL = false> (ElemsArgs)
    kPlanKinds = 5
};
struct LeanArgs { const char *in; char *io; uint64_t vbytes; uint64_t keep; };
struct ElemsArgs { const char *in; char *io; uint64_t n; uint64_t stride; };
struct ReducePlan {
    int kind;
    uint32_t arg_bytes;
    uint64_t groups;    // workgroups of kThreads
    alignas(16) unsigned char args[sizeof(ShiftArgs<char>)];
};

// The direct AQL dispatch's kernarg slot (direct_dispatch.hip writes it,
// direct_tiles.hip's kernels read it): one 128-byte L2 line, two 64-byte halves.
//   words 0-5, 8-13   the plan's argument bytes (at most kSlotArgBytes)
//   word 6            address of the device's error word (host memory)
//   words 7, 15       the nonce, one copy per half: the queue index + 1 of the
//                     last packet that stamped the slot (its dispatch id + 1)
struct KargSlot { uint64_t w[16]; };
constexpr uint32_t kSlotArgBytes = 96;
static_assert(sizeof(ShiftArgs<char>) <= kSlotArgBytes, "ShiftArgs must fit the kernarg slot");

// Fills `p` (padding bytes zero: the direct path's kernarg cache compares bytes).
template <class T>
void plan_reduce(const void *in_, void *io_, uint64_t count, ReducePlan &p) {
    __builtin_memset(&p, 0, sizeof p);
    const char *in = static_cast<const char *>(in_);
    char *io = static_cast<char *>(io_);
    const uintptr_t ai = reinterpret_cast<uintptr_t>(in), ao = reinterpret_cast<uintptr_t>(io);
    const uint64_t nbytes = count * sizeof(T);
    const bool natural = (ai % alignof(T) == 0) && (ao % alignof(T) == 0);
    const uint64_t head0 = (16 - (ao & 15)) & 15;
    TileArgs<T> ta;
    __builtin_memset(&ta, 0, sizeof ta);
    if (tile_split<T>(in_, io_, count, ta)) {
        p.groups = tile_groups(ta.io, ta.vbytes);
        if (ta.nhead || ta.ntail) {
            p.kind = kPlanFull;
            __builtin_memcpy(p.args, &ta, sizeof ta);
            p.arg_bytes = sizeof ta;
        } else {
            const LeanArgs la{ta.in, ta.io, ta.vbytes, ta.keep};
            p.kind = kPlanLean;
            __builtin_memcpy(p.args, &la, sizeof la);
            p.arg_bytes = sizeof la;
        }
    } else if ((ao % alignof(T) == 0) && head0 % sizeof(T) == 0 && nbytes >= 2 * kTileBytes) {
        // inoutbuf element-aligned, inbuf at any other offset mod 16: the
        // aligned-load + shuffle + funnel tile kernel (small counts stay
        // on the element kernel, where a launch's setup dominates anyway)
        const uint64_t head_bytes = head0;
        const uint64_t rest = nbytes - head_bytes;
        const uint64_t vbytes = rest & ~(uint64_t)15;
        ShiftArgs<T> a;
        __builtin_memset(&a, 0, sizeof a);
        a.t.in = nullptr;
        a.t.io = io + head_bytes;
        a.t.vbytes = vbytes;
        a.t.head_in = reinterpret_cast<const T *>(in);
        a.t.head_io = reinterpret_cast<T *>(io);
        a.t.nhead = (uint32_t)(head_bytes / sizeof(T));
        a.t.tail_in = reinterpret_cast<const T *>(in + head_bytes + vbytes);
        a.t.tail_io = reinterpret_cast<T *>(io + head_bytes + vbytes);
        a.t.ntail = (uint32_t)((rest - vbytes) / sizeof(T));
        a.t.keep = keep_for(vbytes);
        const uintptr_t vin = ai + head_bytes;
        a.delta = (uint32_t)(vin & 15);
        a.in_al = reinterpret_cast<const char *>(vin - a.delta);
        p.kind = kPlanShift;
        p.groups = (vbytes + kTileBytes - 1) / kTileBytes;
        __builtin_memcpy(p.args, &a, sizeof a);
        p.arg_bytes = sizeof a;
    } else {
        uint64_t grid = (count + kThreads - 1) / kThreads;
        if (grid > 4096) grid = 4096;
        if (grid == 0) grid = 1;
        const ElemsArgs ea{in, io, count, grid * kThreads};
        p.kind = natural ? kPlanElems : kPlanElemsU;
        p.groups = grid;
        __builtin_memcpy(p.args, &ea, sizeof ea);
        p.arg_bytes = sizeof ea;
    }
}

// the same, type-erased (Entry::plan, kernel_table.hpp)
template <class T>
void plan_reduce_any(const void *in, void *io, uint64_t count, ReducePlan *p) {
    plan_reduce<T>(in, io, count, *p);
}

// Host-side launcher: the plan's kernel through HIP.  Returns the launch error.
template <class Op, class T>
hipError_t launch_reduce(const void *in, void *io, uint64_t count, hipStream_t s) {
    ReducePlan p;
    plan_reduce<T>(in, io, count, p);
    const dim3 grid((unsigned)p.groups), block(kThreads);
    switch (p.kind) {
    case kPlanLean: {
        LeanArgs a;
        __builtin_memcpy(&a, p.args, sizeof a);
        hipLaunchKernelGGL((k_reduce_tile_lean<Op, T>), grid, block, 0, s, a.in, a.io, a.vbytes, a.keep);
        break;
    }
    case kPlanFull: {
        TileArgs<T> a;
        __builtin_memcpy(&a, p.args, sizeof a);
        hipLaunchKernelGGL((k_reduce_tile<Op, T>), grid, block, 0, s, a);
        break;
    }
    case kPlanShift: {
        ShiftArgs<T> a;
        __builtin_memcpy(&a, p.args, sizeof a);
        hipLaunchKernelGGL((k_reduce_shift<Op, T>), grid, block, 0, s, a);
        break;
    }
    default: {
        ElemsArgs a;
        __builtin_memcpy(&a, p.args, sizeof a);
        if (p.kind == kPlanElems)
            hipLaunchKernelGGL((k_reduce_elems<Op, T, true>), grid, block, 0, s, a.in, a.io, a.n, a.stride);
        else
            hipLaunchKernelGGL((k_reduce_elems<Op, T, false>), grid, block, 0, s, a.in, a.io, a.n, a.stride);
        break;
    }
    }
    return hipGetLastError();
}

// Elements wider than 16 bytes (long double _Complex, MPI_LONG_DOUBLE_INT:
// 32 B): the LDS transpose.  The tile is loaded and stored lane-contiguous
// (fully coalesced buffer_load/store_dwordx4 nt, like k_reduce_tile), staged
// through LDS, and each lane combines whole elements out of LDS -- the soft
// x87 combine needs an element's two 16-byte halves in one lane.  Measured at
// 256 MiB (profiles/archive/r01_kernel_ab_wide_lds.log): SUM 0.78, MAXLOC 0.81 of the
// HBM peak vs 0.65 when each lane loads its own halves (lanes 32 B apart, every
// 128-byte line fetched twice under `nt`).  The buffer range check handles
// the ragged last tile (zeros in, stores dropped).
template <class Op, class T, int EPL>
__global__ __launch_bounds__(kThreads) void k_reduce_tile_wide(const char *in, char *io, uint64_t nbytes, uint64_t keep) {
    static_assert(sizeof(T) == 32, "two 16-byte halves per element");
    constexpr int NV = 2 * EPL;                       // 16-byte vectors per lane per operand
    constexpr uint32_t tile = kThreads * NV * 16;
    __shared__ u32x4 sa[kThreads * NV], sb[kThreads * NV];
    const uint64_t base = (uint64_t)blockIdx.x * tile;
    if (base >= nbytes) return;
    const uint64_t left = nbytes - base;
    const int nrec = (int)(left < tile ? left : tile);
    __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void *)(in + base), 0, nrec, 0x00020000);
    __amdgpu_buffer_rsrc_t rio = __builtin_amdgcn_make_buffer_rsrc((void *)(io + base), 0, nrec, 0x00020000);
    const int t = (int)threadIdx.x;
    // each wave owns a contiguous NV KiB of the tile; LDS slot = byte offset / 16,
    // so element e still sits in slots 2e, 2e+1 whichever lane loaded it
    const int wv = (t >> 6) * NV * 64 + (t & 63);    // 16-byte vector index of v = 0
    u32x4 a[NV], b[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        a[v] = __builtin_amdgcn_raw_buffer_load_b128(rio, (wv + v * 64) * 16, 0, kCachePolicyNT);
        b[v] = __builtin_amdgcn_raw_buffer_load_b128(rin, (wv + v * 64) * 16, 0, kCachePolicyNT);
        if (v + 1 < NV) issue_gap();
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        sa[wv + v * 64] = a[v];
        sb[wv + v * 64] = b[v];
    }
    __syncthreads();
    Op op;
    struct V { u32x4 h[2]; };
#pragma unroll
    for (int u = 0; u < EPL; ++u) {
        const int e = u * kThreads + t;
        const T x = __builtin_bit_cast(T, V{{sa[2 * e], sa[2 * e + 1]}});
        const T y = __builtin_bit_cast(T, V{{sb[2 * e], sb[2 * e + 1]}});
        const V r = __builtin_bit_cast(V, op(x, y));
        sa[2 * e] = r.h[0];
        sa[2 * e + 1] = r.h[1];
    }
    __syncthreads();
#pragma unroll
    for (int v = 0; v < NV; ++v)
        store16(sa[wv + v * 64], rio, (wv + v * 64) * 16, keep_tile(base, nbytes, keep));
}

// EPL: elements per lane (2 for the memory-bound ops; the compute-bound soft
// x87 complex PROD does better with 1, more waves per element).
// Pointers not 16 B-aligned take the element-granular kernel.
template <class Op, class T, int EPL = 2>
hipError_t launch_reduce_wide(const void *in_, void *io_, uint64_t count, hipStream_t s) {
    static_assert(sizeof(T) > 16, "16-byte and smaller elements use launch_reduce");
    const char *in = static_cast<const char *>(in_);
    char *io = static_cast<char *>(io_);
    const uintptr_t ai = reinterpret_cast<uintptr_t>(in), ao = reinterpret_cast<uintptr_t>(io);
    if (ai % 16 == 0 && ao % 16 == 0) {
        constexpr uint32_t tile = kThreads * EPL * 32;
        const uint64_t nbytes = count * sizeof(T);
        uint64_t grid = (nbytes + tile - 1) / tile;
        if (grid == 0) grid = 1;
        hipLaunchKernelGGL((k_reduce_tile_wide<Op, T, EPL>), dim3((unsigned)grid), dim3(kThreads), 0, s, in, io, nbytes,
                           keep_for(nbytes));
        return hipGetLastError();
    }
    uint64_t grid = (count + kThreads - 1) / kThreads;
    if (grid > 4096) grid = 4096;
    if (grid == 0) grid = 1;
    hipLaunchKernelGGL((k_reduce_elems<Op, T, false>), dim3((unsigned)grid), dim3(kThreads), 0, s, in, io, count,
                       grid * kThreads);
    return hipGetLastError();
}

// ============================================================================
// Multi-operand combines: the log2(p) / (p-1) MPIR_Reduce_local steps of a
// reduction schedule fused into ONE pass over HBM, in the schedule's exact
// association and operand order (so results are bit-identical to running the
// reference schedule step by step).
//
//   TREE  (recursive halving: reduce_intra_reduce_scatter_gather.c:186-249,
//          allreduce_intra_reduce_scatter_allgather.c:150-215):
//          v_j = y_j; for l = 0..L-1: v_j = v_j (+) v_{j + 2^l}, j % 2^(l+1) == 0
//          i.e. ((y0+y1)+(y2+y3))+((y4+y5)+(y6+y7)), left operand = inout.
//          The caller orders y_j = contribution of newrank (owner ^ j).
//   CHAIN (pairwise: reduce_scatter_block_intra_pairwise.c:97-134):
//          acc = y0; acc = acc (+) y1; ...; acc = acc (+) y_{P-1}.
//
// One workgroup reads P x TILE bytes and writes TILE bytes; the lane keeps
// P 16-byte loads in flight (P x 1 KiB per wave-instruction group).
// ============================================================================
constexpr int kMaxOperands = 16;

struct MultiArgs {
    const char *in[kMaxOperands];   // 16 B-aligned vector regions, same alignment as out
    char *out;
    uint64_t vbytes;                // multiple of 16
    uint32_t nhead, ntail;          // scalar elements before / after the vector region
    int64_t head_off, tail_off;     // byte offsets of head / tail from the region starts
    uint64_t keep;                  // keep_for(vbytes)
};

template <class Op, class T, int P, bool TREE, bool RAW = false>
__device__ __forceinline__ void fold_elems(T (&v)[P]) {
    Op op;
    if constexpr (TREE) {
#pragma unroll
        for (int step = 1; step < P; step *= 2)
#pragma unroll
            for (int j = 0; j < P; j += 2 * step) {
                if constexpr (RAW) v[j] = Op::raw(v[j], v[j + step]);
                else v[j] = op(v[j], v[j + step]);
            }
    } else {
#pragma unroll
        for (int j = 1; j < P; ++j) {
            if constexpr (RAW) v[0] = Op::raw(v[0], v[j]);
            else v[0] = op(v[0], v[j]);
        }
    }
}

// fold with the fast path: plain arithmetic, then the exact x86-rule fold only
// if the result is NaN (a NaN anywhere in an add/mul tree reaches the root)
template <class Op, class T, int P, bool TREE>
__device__ __forceinline__ T fold_fast(const T (&v0)[P]) {
    T v[P];
#pragma unroll
    for (int j = 0; j < P; ++j) v[j] = v0[j];
    if constexpr (nan_fast<Op, T>::value) {
        fold_elems<Op, T, P, TREE, true>(v);
        if (__builtin_expect(!isnan_(v[0]), 1)) return v[0];
#pragma unroll
        for (int j = 0; j < P; ++j) v[j] = v0[j];
    }
    fold_elems<Op, T, P, TREE>(v);
    return v[0];
}

// tile `blk` of the fused fold (TH threads, U vectors per lane per operand)
template <class Op, class T, int P, bool TREE, int U, int TH>
__device__ __forceinline__ void combine_multi_tile(const MultiArgs &a, uint64_t blk) {
    constexpr uint32_t tile = TH * U * 16;
    const uint64_t base = blk * tile;
    if (base < a.vbytes) {
        const uint64_t left = a.vbytes - base;
        const int nrec = (int)(left < tile ? left : tile);
        // each wave owns a contiguous U KiB of every operand's tile (as in the
        // two-operand kernel); the loads go vector by vector across the P
        // operands with an issue gap after every (P == 2 ? 2 : 4) of them
        const int t = (int)threadIdx.x;
        const int wb = (t >> 6) * (U * 1024) + (t & 63) * 16;
        constexpr int GAP = P == 2 ? 2 : 4;
        u32x4 x[P][U];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < P; ++j) {
                __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(a.in[j] + base), 0, nrec, 0x00020000);
                x[j][u] = __builtin_amdgcn_raw_buffer_load_b128(r, wb + u * 1024, 0, kCachePolicyNT);
                if ((u * P + j + 1) % GAP == 0 && u * P + j + 1 < U * P) issue_gap();
            }
        __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void *)(a.out + base), 0, nrec, 0x00020000);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            Pack16<T> pk[P];
#pragma unroll
            for (int j = 0; j < P; ++j) pk[j] = __builtin_bit_cast(Pack16<T>, x[j][u]);
            Pack16<T> res;
#pragma unroll
            for (int k = 0; k < (int)(16 / sizeof(T)); ++k) {
                T v[P];
#pragma unroll
                for (int j = 0; j < P; ++j) v[j] = pk[j].e[k];
                res.e[k] = fold_fast<Op, T, P, TREE>(v);
            }
            store16(__builtin_bit_cast(u32x4, res), ro, wb + u * 1024, keep_tile(base, a.vbytes, a.keep));
        }
    }
}

template <class Op, class T, int P, bool TREE, int U, int TH>
__global__ __launch_bounds__(TH) void k_combine_multi(MultiArgs a) {
    combine_multi_tile<Op, T, P, TREE, U, TH>(a, blockIdx.x);
    if (blockIdx.x == 0) {
        const unsigned t = threadIdx.x;
        int64_t off = 0;
        bool act = false;
        if (t < a.nhead) { off = a.head_off + (int64_t)(t * sizeof(T)); act = true; }
        else if (t >= 64 && t - 64 < a.ntail) { off = a.tail_off + (int64_t)((t - 64) * sizeof(T)); act = true; }
        if (act) {
            T v[P];
#pragma unroll
            for (int j = 0; j < P; ++j) v[j] = *reinterpret_cast<const T *>(a.in[j] + off);
            fold_elems<Op, T, P, TREE>(v);
            *reinterpret_cast<T *>(a.out + off) = v[0];
        }
    }
}

// Misaligned operands: element-granular grid-stride fallback.
template <class Op, class T, int P, bool TREE>
__global__ __launch_bounds__(kThreads) void k_combine_multi_elems(MultiArgs a, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * kThreads;
    for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) {
        T v[P];
#pragma unroll
        for (int j = 0; j < P; ++j) __builtin_memcpy(&v[j], a.in[j] + i * sizeof(T), sizeof(T));
        fold_elems<Op, T, P, TREE>(v);
        __builtin_memcpy(a.out + i * sizeof(T), &v[0], sizeof(T));
    }
}

// Fewer loads in flight per CU for the many-operand folds: a dynamic LDS
// reservation the kernel never touches caps the workgroups a CU holds.
//   * P = 8 (1024-thread workgroups): 96 KiB, one per CU instead of two, 128 KiB
//     of loads in flight per CU instead of 256.  The eight reads alone do not
//     gain: the write stream among them does (tools/fused_write_ab.hip,
//     tools/multi_occ_ab.hip, profiles/r04/fused_*.log, multi_occ_ab*.log).
//   * P = 4 (256 threads x 4 vectors): 53 KiB, three per CU (192 KiB in flight;
//     shape sweep: tools/multi_p24_occ_ab.hip, profiles/r04/multi_p24_occ_ab.log).
//   * P = 2: no cap (TREE2 loses 2 points under one, CHAIN2 moves by 0.3).
// Two library builds alternated (tools/multi_cap_ab.sh, profiles/r04/
// multi_cap_ab.log, four pairs per case, outputs identical), without -> with:
// TREE8 fp32 over 8 x 32 MiB 0.744-0.749 -> 0.750-0.757, CHAIN8 fp16 over
// 8 x 128 MiB 0.745-0.749 -> 0.762-0.764, TREE4 fp32 over 4 x 64 MiB
// 0.726-0.735 -> 0.756-0.758, CHAIN4 fp16 over 4 x 256 MiB 0.760-0.763 -> 0.809-0.813.
// 0 (no reservation) if the runtime refuses the attribute.
#ifndef MPIR_MULTI_CAP_LDS
#define MPIR_MULTI_CAP_LDS 1    // 0: no reservation (a build-time override for tools/multi_cap_ab.sh only)
#endif
template <int P, int TH>
constexpr int multi_cap_bytes() {
    // P = 5-7 (CHAIN folds of non-power-of-two rank counts) take P = 8's shape
    // and cap, P = 3 P = 4's: with the operands in one staging slab at
    // stage_stride() apart, as the collectives lay them, 1024 x 1 at one per CU
    // runs CHAIN5-7 0.765-0.773 against 0.749-0.762 for 256 x 4 at three per CU,
    // and CHAIN3 0.779 against 0.816 (tools/archive/chain_shape.hip chainslab,
    // profiles/r05/chainslab_shape.log).  (With one allocation per operand the
    // order reverses, also for P = 8 below 128 MiB: chain_shape.log,
    // p8_shape*.log against slab_shape.log; the library follows its collectives.)
    return !MPIR_MULTI_CAP_LDS ? 0
           : (P >= 5 && TH == 1024) ? (96 << 10)
           : ((P == 4 || P == 3) && TH == kThreads) ? (53 << 10) : 0;
}
// Per call (MPIR_Hip_combine_set_flags, MPIR_HIP_COMBINE_UNCAPPED): a fold
// that runs beside other kernels -- the device collectives' pipelined fold,
// overlapping RCCL's transfer kernels -- goes without the reservation, which
// would hold every CU to one of its workgroups and slow the kernels beside it
// (tools/archive/lds_cap_cost.hip).
bool multi_uncapped();      // the calling thread's flag (hip_reduce.hip)
template <class Op, class T, int P, bool TREE, int U, int TH>
size_t multi_lds_cap() {
    constexpr int cap = multi_cap_bytes<P, TH>();
    if constexpr (cap == 0) {
        return 0;
    } else {
        static const size_t v = hipFuncSetAttribute((const void *)k_combine_multi<Op, T, P, TREE, U, TH>,
                                                    hipFuncAttributeMaxDynamicSharedMemorySize,
                                                    cap) == hipSuccess ? (size_t)cap : 0;
        return v;
    }
}

template <class Op, class T, int P, bool TREE, int U, int TH>
hipError_t launch_combine_pu(const void *const *ins, void *out_, uint64_t count, hipStream_t s) {
    constexpr uint32_t tile = TH * U * 16;
    char *out = static_cast<char *>(out_);
    const uintptr_t ao = reinterpret_cast<uintptr_t>(out);
    const uint64_t nbytes = count * sizeof(T);
    bool vec_ok = (ao % alignof(T) == 0) && (((16 - (ao & 15)) & 15) % sizeof(T) == 0);
    for (int j = 0; j < P; ++j) {
        const uintptr_t ai = reinterpret_cast<uintptr_t>(ins[j]);
        vec_ok = vec_ok && (ai % alignof(T) == 0) && (((ai ^ ao) & 15) == 0);
    }
    MultiArgs a;
    for (int j = 0; j < kMaxOperands; ++j) a.in[j] = j < P ? static_cast<const char *>(ins[j]) : nullptr;
    if (vec_ok) {
        uint64_t head = (16 - (ao & 15)) & 15;
        if (head > nbytes) head = nbytes;
        const uint64_t rest = nbytes - head, vbytes = rest & ~(uint64_t)15;
        for (int j = 0; j < P; ++j) a.in[j] += head;
        a.out = out + head;
        a.vbytes = vbytes;
        a.keep = keep_for(vbytes);
        a.nhead = (uint32_t)(head / sizeof(T));
        a.head_off = -(int64_t)head;                // head elements sit before the region start
        a.ntail = (uint32_t)((rest - vbytes) / sizeof(T));
        a.tail_off = (int64_t)vbytes;
        uint64_t grid = (vbytes + tile - 1) / tile;
        if (grid == 0) grid = 1;
        const size_t lds = multi_uncapped() ? 0 : multi_lds_cap<Op, T, P, TREE, U, TH>();
        hipLaunchKernelGGL((k_combine_multi<Op, T, P, TREE, U, TH>), dim3((unsigned)grid), dim3(TH), lds, s, a);
    } else {
        a.out = out;
        a.vbytes = 0;
        a.keep = 0;
        uint64_t grid = (count + kThreads - 1) / kThreads;
        if (grid > 4096) grid = 4096;
        if (grid == 0) grid = 1;
        hipLaunchKernelGGL((k_combine_multi_elems<Op, T, P, TREE>), dim3((unsigned)grid), dim3(kThreads), 0, s, a, count);
    }
    return hipGetLastError();
}

// Any (op, element class), any n <= 64, either order, in ONE pass with no
// device temporaries: the combine for the (op, type) pairs the fused
// k_combine_multi is not instantiated for (logical / bitwise ops, MAXLOC /
// MINLOC pairs, complex PROD, long double) and for n > 8.  Element-granular
// and grid-stride; the tree is evaluated left to right with a per-thread
// stack (a binary counter of partial results), which is the association
// ((y0+y1)+(y2+y3))+... with the earlier partial always the left operand.
// out may alias in[0]: every input of element i is read before out[i] is written.
constexpr int kMaxAnyOperands = 64;
struct AnyArgs {
    const char *in[kMaxAnyOperands];
    char *out;
    int n;
    int tree;
};

template <class Op, class T>
__global__ __launch_bounds__(kThreads) void k_combine_any(AnyArgs a, uint64_t count) {
    Op op;
    const uint64_t stride = (uint64_t)gridDim.x * kThreads;
    for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < count; i += stride) {
        const uint64_t off = i * sizeof(T);
        T acc;
        __builtin_memcpy(&acc, a.in[0] + off, sizeof(T));
        if (!a.tree) {
            for (int j = 1; j < a.n; ++j) {
                T v;
                __builtin_memcpy(&v, a.in[j] + off, sizeof(T));
                acc = op(acc, v);
            }
        } else {
            T st[7];
            int lv[7];
            int sp = 0;
            for (int j = 0; j < a.n; ++j) {
                T v = acc;
                if (j) __builtin_memcpy(&v, a.in[j] + off, sizeof(T));
                int l = 0;
                while (sp > 0 && lv[sp - 1] == l) {
                    v = op(st[sp - 1], v);
                    --sp;
                    ++l;
                }
                st[sp] = v;
                lv[sp] = l;
                ++sp;
            }
            acc = st[0];
        }
        __builtin_memcpy(a.out + off, &acc, sizeof(T));
    }
}

template <class Op, class T>
hipError_t launch_combine_any(const void *const *ins, int n, int tree, void *out, uint64_t count, hipStream_t s) {
    if (n < 1 || n > kMaxAnyOperands || (tree && (n & (n - 1)))) return hipErrorInvalidValue;
    AnyArgs a;
    for (int j = 0; j < kMaxAnyOperands; ++j) a.in[j] = j < n ? static_cast<const char *>(ins[j]) : nullptr;
    a.out = static_cast<char *>(out);
    a.n = n;
    a.tree = tree;
    uint64_t grid = (count + kThreads - 1) / kThreads;
    if (grid > 8192) grid = 8192;
    if (grid == 0) grid = 1;
    hipLaunchKernelGGL((k_combine_any<Op, T>), dim3((unsigned)grid), dim3(kThreads), 0, s, a, count);
    return hipGetLastError();
}

template <class Op, class T, int P, bool TREE>
hipError_t launch_combine_p(const void *const *ins, void *out_, uint64_t count, hipStream_t s) {
    // (2, 4, 8 for TREE; every P of 2-8 for CHAIN: 5-7 in P = 8's shape, 3 in
    // P = 4's).  rocprofv3 trace, 32 MiB blocks (profiles/archive/r01s3_multi_shape_p24.log):
    // P = 8 on 1024-thread WGs (0.76-0.80 of peak); P = 4 with 4 vectors per lane
    // 0.78-0.80 (2 vectors: 0.72-0.74); P = 2 with 4 vectors per lane 0.74-0.76
    // P = 2 over blocks of 256 MiB or more (config 5's 2 x 512 MiB at 2 ranks) on
    // 1024 x 1, uncapped: 0.798-0.808 against 0.784-0.788 for 256 x 4 in the
    // staging slab; over 128 MiB the two tie (tools/archive/chain_shape.hip p2slab,
    // profiles/r05/p2slab*.log)
    if constexpr (P == 2) {
        if (count * sizeof(T) >= (256ull << 20))
            return launch_combine_pu<Op, T, 2, TREE, 1, 1024>(ins, out_, count, s);
    }
    return launch_combine_pu<Op, T, P, TREE, (P >= 5 ? 1 : 4), (P >= 5 ? 1024 : kThreads)>(ins, out_, count, s);
}

}  // namespace mpir_hip

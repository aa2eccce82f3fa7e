// reduce_kernels.hpp -- gfx950 streaming kernels for MPIR_Reduce_local.
//
// The combine is element-wise: 2 reads + 1 write per element, arithmetic
// intensity <= 1/12 op/B for fp32, so the roofline is HBM bandwidth and MFMA
// is irrelevant.  The shape below is the winner of tools/bw_sweep*.hip on
// MI355X (256 MiB/operand fp32 SUM, profiles/ and DESIGN.md §Kernels):
//
//   * one 16 KiB tile per operand per 256-thread workgroup (4 x 16 B per lane,
//     lane-contiguous 1 KiB wave-instructions), no grid-stride loop: the grid
//     is vbytes / 16 KiB workgroups (16384 at 256 MiB), which keeps every CU's
//     queue deep and the DRAM pages of a tile together;
//   * all 8 loads of a lane issued before the first combine (latency hiding
//     by ILP + 8 waves/CU of TLP);
//   * buffer_load/store_dwordx4 with the `nt` cache policy (aux = 2) on both
//     operands and on the store: streamed-once data should not displace L2 /
//     Infinity Cache lines; measured 0.81 of the 8 TB/s HBM peak vs 0.70 for
//     default-policy loads and 0.63 for a grid-stride loop;
//   * the buffer descriptor covers exactly this tile's bytes, so the ragged
//     last tile needs no branch: out-of-range loads return 0 and out-of-range
//     stores are dropped by the hardware range check.
// The < 16 B head (to 16 B-align inout) and tail are handled element-wise by
// workgroup 0, so a call is always exactly one launch.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "reduce_ops.hpp"

namespace mpir_hip {

constexpr int kThreads = 256;
constexpr int kVecPerLane = 4;
constexpr uint32_t kTileBytes = kThreads * kVecPerLane * 16;  // 16 KiB per operand
constexpr int kCachePolicyNT = 2;                             // aux bit: nt

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

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
};

template <class Op, class T>
__device__ __forceinline__ u32x4 combine16(u32x4 a, u32x4 b) {
    Pack16<T> pa = __builtin_bit_cast(Pack16<T>, a);
    Pack16<T> pb = __builtin_bit_cast(Pack16<T>, b);
    Op op;
#pragma unroll
    for (int k = 0; k < (int)(16 / sizeof(T)); ++k) pa.e[k] = op(pa.e[k], pb.e[k]);
    return __builtin_bit_cast(u32x4, pa);
}

template <class Op, class T>
__global__ __launch_bounds__(kThreads) void k_reduce_tile(TileArgs<T> args) {
    const uint64_t base = (uint64_t)blockIdx.x * kTileBytes;
    if (base < args.vbytes) {
        const uint64_t left = args.vbytes - base;
        const int nrec = (int)(left < kTileBytes ? left : kTileBytes);
        __amdgpu_buffer_rsrc_t rin = __builtin_amdgcn_make_buffer_rsrc((void *)(args.in + base), 0, nrec, 0x00020000);
        __amdgpu_buffer_rsrc_t rio = __builtin_amdgcn_make_buffer_rsrc((void *)(args.io + base), 0, nrec, 0x00020000);
        u32x4 a[kVecPerLane], b[kVecPerLane];
#pragma unroll
        for (int u = 0; u < kVecPerLane; ++u) {
            const int off = (u * kThreads + (int)threadIdx.x) * 16;
            a[u] = __builtin_amdgcn_raw_buffer_load_b128(rio, off, 0, kCachePolicyNT);
            b[u] = __builtin_amdgcn_raw_buffer_load_b128(rin, off, 0, kCachePolicyNT);
        }
#pragma unroll
        for (int u = 0; u < kVecPerLane; ++u) {
            const int off = (u * kThreads + (int)threadIdx.x) * 16;
            __builtin_amdgcn_raw_buffer_store_b128(combine16<Op, T>(a[u], b[u]), rio, off, 0, kCachePolicyNT);
        }
    }
    if (blockIdx.x == 0) {
        Op op;
        const unsigned t = threadIdx.x;
        if (t < args.nhead) args.head_io[t] = op(args.head_io[t], args.head_in[t]);
        else if (t >= 64 && t - 64 < args.ntail) args.tail_io[t - 64] = op(args.tail_io[t - 64], args.tail_in[t - 64]);
    }
}

// General path: inbuf and inoutbuf differ in alignment mod 16 (sub-range
// displacements of arbitrary element counts), or elements are not even
// naturally aligned.  Element-granular, coalesced, grid-stride.
template <class Op, class T, bool NATURAL>
__global__ __launch_bounds__(kThreads) void k_reduce_elems(const char *in, char *io, uint64_t n) {
    Op op;
    const uint64_t stride = (uint64_t)gridDim.x * kThreads;
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

// Host-side launcher: splits [in, io) x count into head / 16 B vector body /
// tail when both pointers share their alignment mod 16, else uses the
// element-granular kernel.  Returns the launch error.
template <class Op, class T>
hipError_t launch_reduce(const void *in_, void *io_, uint64_t count, hipStream_t s) {
    const char *in = static_cast<const char *>(in_);
    char *io = static_cast<char *>(io_);
    const uintptr_t ai = reinterpret_cast<uintptr_t>(in), ao = reinterpret_cast<uintptr_t>(io);
    const uint64_t nbytes = count * sizeof(T);
    const bool natural = (ai % alignof(T) == 0) && (ao % alignof(T) == 0);
    const uint64_t head0 = (16 - (ao & 15)) & 15;
    if (natural && ((ai ^ ao) & 15) == 0 && head0 % sizeof(T) == 0) {
        const uint64_t head_bytes = head0 < nbytes ? head0 : nbytes;
        const uint64_t rest = nbytes - head_bytes;
        const uint64_t vbytes = rest & ~(uint64_t)15;
        TileArgs<T> a;
        a.in = in + head_bytes;
        a.io = io + head_bytes;
        a.vbytes = vbytes;
        a.head_in = reinterpret_cast<const T *>(in);
        a.head_io = reinterpret_cast<T *>(io);
        a.nhead = (uint32_t)(head_bytes / sizeof(T));
        a.tail_in = reinterpret_cast<const T *>(in + head_bytes + vbytes);
        a.tail_io = reinterpret_cast<T *>(io + head_bytes + vbytes);
        a.ntail = (uint32_t)((rest - vbytes) / sizeof(T));
        uint64_t grid = (vbytes + kTileBytes - 1) / kTileBytes;
        if (grid == 0) grid = 1;
        hipLaunchKernelGGL((k_reduce_tile<Op, T>), dim3((unsigned)grid), dim3(kThreads), 0, s, a);
    } else {
        uint64_t grid = (count + kThreads - 1) / kThreads;
        if (grid > 4096) grid = 4096;
        if (grid == 0) grid = 1;
        if (natural)
            hipLaunchKernelGGL((k_reduce_elems<Op, T, true>), dim3((unsigned)grid), dim3(kThreads), 0, s, in, io, count);
        else
            hipLaunchKernelGGL((k_reduce_elems<Op, T, false>), dim3((unsigned)grid), dim3(kThreads), 0, s, in, io, count);
    }
    return hipGetLastError();
}

}  // namespace mpir_hip

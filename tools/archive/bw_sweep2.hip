// Bandwidth sweep for the fp32 MPI_SUM combine on gfx950: which streaming
// shape reaches the HBM roofline?  Standalone tuning tool (not the product);
// the winning shape is what mpich-pip_amd/csrc/hip/reduce_kernels.hpp uses.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bw_sweep tools/bw_sweep.hip
//   ./tools/bw_sweep [MiB_per_operand=256] [iters=30]
//
// Every variant computes inout[i] = inout[i] + in[i] over `count` floats and
// is checked against a host recomputation once.  Timed launches rotate over
// NSETS buffer pairs (NSETS*2*256 MiB >> 256 MiB Infinity Cache) so the
// numbers are HBM, not MALL.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(2);} } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

template <bool NT_LD>
__device__ __forceinline__ f4 ld(const f4 *p) {
    if constexpr (NT_LD) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT_ST>
__device__ __forceinline__ void st(f4 *p, f4 v) {
    if constexpr (NT_ST) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// A: grid-stride, UNROLL vectors per lane per trip
template <int U, bool NL, bool NS>
__global__ void k_gridstride(const f4 *__restrict__ in, f4 *__restrict__ io, size_t nvec) {
    size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < nvec; i += U * stride) {
        f4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) { a[u] = ld<NL>(io + i + u * stride); b[u] = ld<NL>(in + i + u * stride); }
#pragma unroll
        for (int u = 0; u < U; ++u) st<NS>(io + i + u * stride, a[u] + b[u]);
    }
    for (; i < nvec; i += stride) st<NS>(io + i, ld<NL>(io + i) + ld<NL>(in + i));
}

// B: one tile per block, no loop: block b owns vectors [b*T, (b+1)*T), T = blockDim*U
template <int U, bool NL, bool NS>
__global__ void k_tile(const f4 *__restrict__ in, f4 *__restrict__ io, size_t nvec) {
    size_t base = (size_t)blockIdx.x * blockDim.x * U + threadIdx.x;
    if (base + (size_t)(U - 1) * blockDim.x < nvec) {
        f4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) { a[u] = ld<NL>(io + base + u * blockDim.x); b[u] = ld<NL>(in + base + u * blockDim.x); }
#pragma unroll
        for (int u = 0; u < U; ++u) st<NS>(io + base + u * blockDim.x, a[u] + b[u]);
    } else {
        for (int u = 0; u < U; ++u) {
            size_t i = base + (size_t)u * blockDim.x;
            if (i < nvec) st<NS>(io + i, ld<NL>(io + i) + ld<NL>(in + i));
        }
    }
}

// C: persistent, contiguous chunk per block, U vectors per lane per trip
template <int U, bool NL, bool NS>
__global__ void k_chunk(const f4 *__restrict__ in, f4 *__restrict__ io, size_t nvec) {
    size_t per = (nvec + gridDim.x - 1) / gridDim.x;
    size_t step = (size_t)blockDim.x * U;
    per = (per + step - 1) / step * step;
    size_t beg = (size_t)blockIdx.x * per, end = std::min(nvec, beg + per);
    for (size_t i = beg + threadIdx.x; i < end; i += step) {
        f4 a[U], b[U];
        bool full = i + (U - 1) * blockDim.x < end;
        if (full) {
#pragma unroll
            for (int u = 0; u < U; ++u) { a[u] = ld<NL>(io + i + u * blockDim.x); b[u] = ld<NL>(in + i + u * blockDim.x); }
#pragma unroll
            for (int u = 0; u < U; ++u) st<NS>(io + i + u * blockDim.x, a[u] + b[u]);
        } else {
            for (int u = 0; u < U; ++u) {
                size_t j = i + (size_t)u * blockDim.x;
                if (j < end) st<NS>(io + j, ld<NL>(io + j) + ld<NL>(in + j));
            }
        }
    }
}

// D: LDS-DMA staging of both operands (global_load_lds_dwordx4), then ds_read + combine + store.
template <int U>
__global__ void k_ldsdma(const f4 *__restrict__ in, f4 *__restrict__ io, size_t nvec) {
    extern __shared__ f4 lds[];  // 2 * U * blockDim f4
    size_t base = (size_t)blockIdx.x * blockDim.x * U;
    if (base + (size_t)blockDim.x * U > nvec) {  // ragged last tile: plain path
        for (int u = 0; u < U; ++u) {
            size_t i = base + threadIdx.x + (size_t)u * blockDim.x;
            if (i < nvec) io[i] = io[i] + in[i];
        }
        return;
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    f4 *la = lds, *lb = lds + (size_t)U * blockDim.x;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        size_t g = base + (size_t)u * blockDim.x + threadIdx.x;
        // LDS dest is wave-uniform base + lane*16: pass the wave's base.
        f4 *wa = la + u * blockDim.x + wave * 64;
        f4 *wb = lb + u * blockDim.x + wave * 64;
        __builtin_amdgcn_global_load_lds((const void *)(io + g), (__attribute__((address_space(3))) void *)wa, 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void *)(in + g), (__attribute__((address_space(3))) void *)wb, 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < U; ++u) {
        size_t g = base + (size_t)u * blockDim.x + threadIdx.x;
        f4 a = la[u * blockDim.x + threadIdx.x], b = lb[u * blockDim.x + threadIdx.x];
        io[g] = a + b;
    }
    (void)lane;
}

__global__ void k_readonly(const f4 *__restrict__ in, const f4 *__restrict__ in2, size_t nvec, float *sink) {
    size_t base = (size_t)blockIdx.x * blockDim.x * 4 + threadIdx.x;
    f4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        size_t i = base + (size_t)u * blockDim.x;
        if (i < nvec) acc += in[i] + in2[i];
    }
    if (acc.x == 12345.678f) *sink = acc.y;  // keep live
}


// E: buffer loads/stores with explicit cache-policy aux bits (1=sc0, 2=nt, 16=sc1)
typedef unsigned int u4 __attribute__((ext_vector_type(4)));
template <int U, int LA, int SA>
__global__ void k_buf(const f4 *__restrict__ in, f4 *__restrict__ io, size_t nvec) {
    size_t base = (size_t)blockIdx.x * blockDim.x * U;
    size_t nb = nvec - base < (size_t)blockDim.x * U ? nvec - base : (size_t)blockDim.x * U;
    __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc((void *)(in + base), 0, (int)(nb * 16), 0x00020000);
    __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void *)(io + base), 0, (int)(nb * 16), 0x00020000);
    u4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        int off = (u * blockDim.x + threadIdx.x) * 16;
        a[u] = __builtin_amdgcn_raw_buffer_load_b128(ro, off, 0, LA);
        b[u] = __builtin_amdgcn_raw_buffer_load_b128(ri, off, 0, LA);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        int off = (u * blockDim.x + threadIdx.x) * 16;
        f4 r = __builtin_bit_cast(f4, a[u]) + __builtin_bit_cast(f4, b[u]);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, r), ro, off, 0, SA);
    }
}
// F: nt tile with XCD-contiguous remap (blocks b, b+8, ... share an XCD -> give them neighbouring tiles)
template <int U>
__global__ void k_tile_xcd(const f4 *__restrict__ in, f4 *__restrict__ io, size_t nvec) {
    unsigned nb = gridDim.x, b = blockIdx.x;
    unsigned per = nb / 8;  // launched with nb % 8 == 0
    unsigned t = (b % 8) * per + b / 8;
    size_t base = (size_t)t * blockDim.x * U + threadIdx.x;
    f4 a[U], c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { a[u] = ld<true>(io + base + u * blockDim.x); c[u] = ld<true>(in + base + u * blockDim.x); }
#pragma unroll
    for (int u = 0; u < U; ++u) st<true>(io + base + u * blockDim.x, a[u] + c[u]);
}
__global__ void k_readonly_nt(const f4 *__restrict__ in, const f4 *__restrict__ in2, size_t nvec, float *sink) {
    size_t base = (size_t)blockIdx.x * blockDim.x * 4 + threadIdx.x;
    f4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        size_t i = base + (size_t)u * blockDim.x;
        if (i < nvec) acc += ld<true>(in + i) + ld<true>(in2 + i);
    }
    if (acc.x == 12345.678f) *sink = acc.y;
}
__global__ void k_copy_nt(const f4 *__restrict__ in, f4 *__restrict__ out, size_t nvec) {
    size_t base = (size_t)blockIdx.x * blockDim.x * 4 + threadIdx.x;
    f4 a[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] = ld<true>(in + base + u * blockDim.x);
#pragma unroll
    for (int u = 0; u < 4; ++u) st<true>(out + base + u * blockDim.x, a[u]);
}

struct Set { f4 *in, *io; };

typedef void (*Launch)(const Set &, size_t nvec, hipStream_t);

static size_t g_count;

static double time_variant(const char *name, Launch fn, std::vector<Set> &sets, size_t nvec, int iters,
                           double bytes, hipStream_t s) {
    for (int w = 0; w < 3; ++w) fn(sets[w % sets.size()], nvec, s);
    CK(hipStreamSynchronize(s));
    std::vector<float> ms(iters);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int it = 0; it < iters; ++it) {
        CK(hipEventRecord(e0, s));
        fn(sets[it % sets.size()], nvec, s);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms[it], e0, e1));
    }
    // back-to-back throughput over all iters (one event pair)
    CK(hipEventRecord(e0, s));
    for (int it = 0; it < iters; ++it) fn(sets[it % sets.size()], nvec, s);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float tot; CK(hipEventElapsedTime(&tot, e0, e1));
    std::sort(ms.begin(), ms.end());
    double med = ms[iters / 2];
    printf("%-34s median %8.1f us  p10 %8.1f  p90 %8.1f  -> %7.0f GB/s (%.3f of 8 TB/s) | b2b %8.1f us %7.0f GB/s\n", name,
           med * 1e3, ms[iters / 10] * 1e3, ms[iters * 9 / 10] * 1e3, bytes / (med * 1e-3) / 1e9,
           bytes / (med * 1e-3) / 8e12, tot * 1e3 / iters, bytes / (tot * 1e-3 / iters) / 1e9);
    fflush(stdout);
    CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
    return med;
}

#define L_GS(U, NL, NS, G, B) [](const Set &st, size_t n, hipStream_t s) { \
    hipLaunchKernelGGL((k_gridstride<U, NL, NS>), dim3(G), dim3(B), 0, s, st.in, st.io, n); }
#define L_TILE(U, NL, NS, B) [](const Set &st, size_t n, hipStream_t s) { \
    size_t t = (size_t)(B) * (U); hipLaunchKernelGGL((k_tile<U, NL, NS>), dim3((n + t - 1) / t), dim3(B), 0, s, st.in, st.io, n); }
#define L_CHUNK(U, NL, NS, G, B) [](const Set &st, size_t n, hipStream_t s) { \
    hipLaunchKernelGGL((k_chunk<U, NL, NS>), dim3(G), dim3(B), 0, s, st.in, st.io, n); }
#define L_BUF(U, LA, SA, B) [](const Set &st, size_t n, hipStream_t s) { \
    size_t t = (size_t)(B) * (U); hipLaunchKernelGGL((k_buf<U, LA, SA>), dim3(n / t), dim3(B), 0, s, st.in, st.io, n); }
#define L_XCD(U, B) [](const Set &st, size_t n, hipStream_t s) { \
    size_t t = (size_t)(B) * (U); hipLaunchKernelGGL((k_tile_xcd<U>), dim3(n / t), dim3(B), 0, s, st.in, st.io, n); }
#define L_LDS(U, B) [](const Set &st, size_t n, hipStream_t s) { \
    size_t t = (size_t)(B) * (U); hipLaunchKernelGGL((k_ldsdma<U>), dim3((n + t - 1) / t), dim3(B), 2 * t * 16, s, st.in, st.io, n); }

int main(int argc, char **argv) {
    size_t mib = argc > 1 ? strtoull(argv[1], 0, 10) : 256;
    int iters = argc > 2 ? atoi(argv[2]) : 30;
    size_t count = mib * (1ull << 20) / 4;
    size_t nvec = count / 4;
    g_count = count;
    hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
    printf("device %s  CUs %d  %zu MiB/operand  count %zu\n", prop.gcnArchName, prop.multiProcessorCount, mib, count);
    const int NSETS = 3;
    std::vector<Set> sets(NSETS);
    std::vector<float> h_in(count), h_io(count);
    for (size_t i = 0; i < count; ++i) { h_in[i] = (float)((i * 2654435761u) % 1000) * 0.001f; h_io[i] = (float)(i % 977) * 0.5f; }
    for (auto &st : sets) {
        CK(hipMalloc(&st.in, count * 4)); CK(hipMalloc(&st.io, count * 4));
        CK(hipMemcpy(st.in, h_in.data(), count * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(st.io, h_io.data(), count * 4, hipMemcpyHostToDevice));
    }
    hipStream_t s; CK(hipStreamCreate(&s));
    double bytes = 3.0 * count * 4;

    struct V { const char *name; Launch fn; };
    std::vector<V> vs = {
        {"tile U4 256 ntLS", L_TILE(4, true, true, 256)},
        {"tile U1 256 ntLS", L_TILE(1, true, true, 256)},
        {"tile U2 256 ntLS", L_TILE(2, true, true, 256)},
        {"tile U4 128 ntLS", L_TILE(4, true, true, 128)},
        {"tile U8 128 ntLS", L_TILE(8, true, true, 128)},
        {"tile U1 512 ntLS", L_TILE(1, true, true, 512)},
        {"tile U2 1024 ntLS", L_TILE(2, true, true, 1024)},
        {"tile U4 64 ntLS", L_TILE(4, true, true, 64)},
        {"buf U4 256 ld0 st0", L_BUF(4, 0, 0, 256)},
        {"buf U4 256 ld nt st nt", L_BUF(4, 2, 2, 256)},
        {"buf U4 256 ld nt|sc0 st nt", L_BUF(4, 3, 2, 256)},
        {"buf U4 256 ld nt|sc1 st nt", L_BUF(4, 18, 2, 256)},
        {"buf U4 256 ld nt|sc0|sc1 st nt", L_BUF(4, 19, 2, 256)},
        {"buf U4 256 ld nt st nt|sc1", L_BUF(4, 2, 18, 256)},
        {"buf U4 256 ld nt st nt|sc0|sc1", L_BUF(4, 2, 19, 256)},
        {"buf U4 256 ld sc1 st sc1", L_BUF(4, 16, 16, 256)},
        {"buf U4 256 ld nt st sc0|sc1", L_BUF(4, 2, 17, 256)},
        {"buf U2 256 ld nt st nt", L_BUF(2, 2, 2, 256)},
        {"xcd U4 256 ntLS", L_XCD(4, 256)},
        {"tile U4 256 ntLS (again)", L_TILE(4, true, true, 256)},
    };

    // correctness check of every variant once on set 0 (fresh copy)
    std::vector<float> out(count);
    for (auto &v : vs) {
        CK(hipMemcpy(sets[0].io, h_io.data(), count * 4, hipMemcpyHostToDevice));
        v.fn(sets[0], nvec, s);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(out.data(), sets[0].io, count * 4, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < count; ++i) { float r = h_io[i] + h_in[i]; if (memcmp(&r, &out[i], 4)) ++bad; }
        if (bad) printf("VARIANT %s WRONG: %zu mismatches\n", v.name, bad);
    }
    for (auto &v : vs) time_variant(v.name, v.fn, sets, nvec, iters, bytes, s);

    // references: D2D copy and read-only stream
    {
        std::vector<float> ms;
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        for (int it = 0; it < iters; ++it) {
            CK(hipEventRecord(e0, s));
            CK(hipMemcpyAsync(sets[it % NSETS].io, sets[(it + 1) % NSETS].in, count * 4, hipMemcpyDeviceToDevice, s));
            CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
            float m; CK(hipEventElapsedTime(&m, e0, e1)); ms.push_back(m);
        }
        std::sort(ms.begin(), ms.end());
        printf("%-34s median %8.1f us -> %7.0f GB/s (2x bytes)\n", "hipMemcpy D2D", ms[iters / 2] * 1e3,
               2.0 * count * 4 / (ms[iters / 2] * 1e-3) / 1e9);
        float *sink; CK(hipMalloc(&sink, 4));
        ms.clear();
        for (int it = 0; it < iters; ++it) {
            CK(hipEventRecord(e0, s));
            size_t t = 256 * 4;
            hipLaunchKernelGGL(k_readonly, dim3((nvec + t - 1) / t), dim3(256), 0, s, sets[it % NSETS].in, sets[it % NSETS].io, nvec, sink);
            CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
            float m; CK(hipEventElapsedTime(&m, e0, e1)); ms.push_back(m);
        }
        std::sort(ms.begin(), ms.end());
        printf("%-34s median %8.1f us -> %7.0f GB/s (2 operands read)\n", "read-only 2 streams", ms[iters / 2] * 1e3,
               2.0 * count * 4 / (ms[iters / 2] * 1e-3) / 1e9);
    }
    {
        float *sink; CK(hipMalloc(&sink, 4));
        Launch ro = [](const Set &st, size_t n, hipStream_t s) { hipLaunchKernelGGL(k_readonly_nt, dim3(n / 1024), dim3(256), 0, s, st.in, st.io, n, (float*)nullptr); };
        time_variant("read-only 2 streams nt (2x bytes)", ro, sets, nvec, iters, 2.0 * count * 4, s);
        Launch cp = [](const Set &st, size_t n, hipStream_t s) { hipLaunchKernelGGL(k_copy_nt, dim3(n / 1024), dim3(256), 0, s, st.in, st.io, n); };
        time_variant("copy nt (2x bytes)", cp, sets, nvec, iters, 2.0 * count * 4, s);
    }
    printf("done\n");
    return 0;
}

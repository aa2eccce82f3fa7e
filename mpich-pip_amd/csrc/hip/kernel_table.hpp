// kernel_table.hpp -- the (op, element class) kernel tables of the C-ABI shim.
//
// g_table[op][elem].fn : the single-operand MPIR_Reduce_local launcher
//                        (k_reduce_tile / k_reduce_shift / k_reduce_elems, or the
//                        32-byte LDS-transpose kernel);
// g_table[op][elem].any: the one-pass n-operand combine (k_combine_any), the
//                        general path of MPIR_Hip_combine; REPLACE has none;
// g_table[op][elem].host: the same combine as a host loop over the same
//                        functors (reduce_ops.hpp), for small operands that
//                        both live in host memory (MPIR_Hip_reduce);
// g_multi[op][elem][order][P - 2]: the fused schedule combines
//                        (k_combine_multi) for the ops the collectives use most:
//                        TREE folds of P = 2, 4, 8 operands, CHAIN folds of every
//                        P from 2 to 8 (a pairwise chain over p ranks is one pass
//                        for any p <= 8).
// Storage lives in hip_reduce.hip (zero-initialised); the reg_*.hip units fill
// it from static constructors, one unit per op family so they compile in
// parallel.  The ops a type admits follow src/include/mpir_op_util.h:263-364.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mpir_hip_reduce.h"
#include "reduce_kernels.hpp"

namespace mpir_hip {

typedef hipError_t (*launch_fn)(const void *, void *, uint64_t, hipStream_t);
typedef hipError_t (*any_fn)(const void *const *, int, int, void *, uint64_t, hipStream_t);
typedef hipError_t (*multi_fn)(const void *const *, void *, uint64_t, hipStream_t);
typedef void (*host_fn)(const void *, void *, uint64_t);
typedef void (*plan_fn)(const void *, void *, uint64_t, ReducePlan *);

// plan: plan_reduce<T> (reduce_kernels.hpp) for the classes whose launcher is
// launch_reduce -- the kernel, grid and argument bytes the direct AQL dispatch
// launches from its code object; null for the 32-byte classes (LDS transpose)
// and REPLACE (a byte copy), which take the HIP launch
struct Entry { launch_fn fn; any_fn any; host_fn host; plan_fn plan; };

// float / double SUM and PROD on the host: the SSE instruction itself.  The
// reference's loop `a[i] = a[i] + b[i]` (opsum.c:21-76, gcc -O2) is an
// addss/addsd (addps/addpd when vectorised) with a[i] -- inout -- as the first
// source, and x86 applies exactly the NaN rule that x86_result restates for
// the GPU: the first source if it is a NaN, else the second, quieted; the
// indefinite for an invalid operation; denormals kept (MXCSR default).  The
// operand order is pinned with inline asm because the compiler treats
// addpd/mulpd as commutative.  4 floats / 2 doubles per instruction instead
// of the functor's per-element NaN checks: 1024 doubles 1.0 -> 0.4 us
// (tools/host_small_latency.c).  Unaligned operands: movups/movupd.
template <bool Prod, class T>
inline bool host_sse(const char *pi, char *po, uint64_t n) {
#if defined(__x86_64__) && !defined(__HIP_DEVICE_COMPILE__)
    typedef float v4f __attribute__((vector_size(16), aligned(1)));
    uint64_t i = 0;
    constexpr uint64_t per = 16 / sizeof(T);
    for (; i + per <= n; i += per) {
        v4f a, b;
        __builtin_memcpy(&a, po + i * sizeof(T), 16);
        __builtin_memcpy(&b, pi + i * sizeof(T), 16);
        if constexpr (sizeof(T) == 4) {
            if constexpr (Prod) asm("mulps %1, %0" : "+x"(a) : "x"(b));
            else asm("addps %1, %0" : "+x"(a) : "x"(b));
        } else {
            if constexpr (Prod) asm("mulpd %1, %0" : "+x"(a) : "x"(b));
            else asm("addpd %1, %0" : "+x"(a) : "x"(b));
        }
        __builtin_memcpy(po + i * sizeof(T), &a, 16);
    }
    for (; i < n; ++i) {
        T a, b;
        __builtin_memcpy(&a, po + i * sizeof(T), sizeof(T));
        __builtin_memcpy(&b, pi + i * sizeof(T), sizeof(T));
        if constexpr (sizeof(T) == 4) {
            if constexpr (Prod) asm("mulss %1, %0" : "+x"(a) : "x"(b));
            else asm("addss %1, %0" : "+x"(a) : "x"(b));
        } else {
            if constexpr (Prod) asm("mulsd %1, %0" : "+x"(a) : "x"(b));
            else asm("addsd %1, %0" : "+x"(a) : "x"(b));
        }
        __builtin_memcpy(po + i * sizeof(T), &a, sizeof(T));
    }
    return true;
#else
    return false;
#endif
}

// inout[i] = Op(inout[i], in[i]) on the host, element by element, through the
// device functors compiled for x86 (unaligned operands: memcpy'd elements)
template <class Op, class T>
void host_loop(const void *in, void *io, uint64_t n) {
    Op op;
    const char *pi = static_cast<const char *>(in);
    char *po = static_cast<char *>(io);
    if constexpr ((__is_same(T, float) || __is_same(T, double)) && (__is_same(Op, OpSum) || __is_same(Op, OpProd)))
        if (host_sse<__is_same(Op, OpProd), T>(pi, po, n)) return;
    for (uint64_t i = 0; i < n; ++i) {
        T a, b;
        __builtin_memcpy(&a, po + i * sizeof(T), sizeof(T));
        __builtin_memcpy(&b, pi + i * sizeof(T), sizeof(T));
        a = op(a, b);
        __builtin_memcpy(po + i * sizeof(T), &a, sizeof(T));
    }
}
extern Entry g_table[MPIR_HIP_NOPS][MPIR_HIP_NELEMS];
constexpr int kMultiMaxP = 8;
extern multi_fn g_multi[MPIR_HIP_NOPS][MPIR_HIP_NELEMS][2][kMultiMaxP - 1];

template <class Op, class T>
void reg(int op, int elem) {
    g_table[op][elem].fn = &launch_reduce<Op, T>;
    g_table[op][elem].host = &host_loop<Op, T>;
    if constexpr (!__is_same(Op, OpReplace)) {
        g_table[op][elem].any = &launch_combine_any<Op, T>;
        g_table[op][elem].plan = &plan_reduce_any<T>;
    }
}
template <class Op, class T, int EPL = 2>
void reg_wide(int op, int elem) {
    g_table[op][elem].fn = &launch_reduce_wide<Op, T, EPL>;
    g_table[op][elem].host = &host_loop<Op, T>;
    g_table[op][elem].any = &launch_combine_any<Op, T>;
}
template <class Op, class T>
void reg_multi(int op, int elem) {
    g_multi[op][elem][0][2 - 2] = &launch_combine_p<Op, T, 2, true>;
    g_multi[op][elem][0][4 - 2] = &launch_combine_p<Op, T, 4, true>;
    g_multi[op][elem][0][8 - 2] = &launch_combine_p<Op, T, 8, true>;
    g_multi[op][elem][1][2 - 2] = &launch_combine_p<Op, T, 2, false>;
    g_multi[op][elem][1][3 - 2] = &launch_combine_p<Op, T, 3, false>;
    g_multi[op][elem][1][4 - 2] = &launch_combine_p<Op, T, 4, false>;
    g_multi[op][elem][1][5 - 2] = &launch_combine_p<Op, T, 5, false>;
    g_multi[op][elem][1][6 - 2] = &launch_combine_p<Op, T, 6, false>;
    g_multi[op][elem][1][7 - 2] = &launch_combine_p<Op, T, 7, false>;
    g_multi[op][elem][1][8 - 2] = &launch_combine_p<Op, T, 8, false>;
}

}  // namespace mpir_hip

// Integer element classes and their device types.
#define FOR_INTS(X) \
    X(MPIR_HIP_I8, int8_t) X(MPIR_HIP_U8, uint8_t) X(MPIR_HIP_I16, int16_t) X(MPIR_HIP_U16, uint16_t) \
    X(MPIR_HIP_I32, int32_t) X(MPIR_HIP_U32, uint32_t) X(MPIR_HIP_I64, int64_t) X(MPIR_HIP_U64, uint64_t)
#define FOR_REALS(X) X(MPIR_HIP_F16, f16) X(MPIR_HIP_F32, float) X(MPIR_HIP_F64, double)
#define FOR_CPLX(X) X(MPIR_HIP_CF32, cf32) X(MPIR_HIP_CF64, cf64)
#define FOR_PAIRS(X) \
    X(MPIR_HIP_P2INT, p2int) X(MPIR_HIP_PFLOATINT, pfloatint) X(MPIR_HIP_PLONGINT, plongint) \
    X(MPIR_HIP_PSHORTINT, pshortint) X(MPIR_HIP_PDOUBLEINT, pdoubleint)

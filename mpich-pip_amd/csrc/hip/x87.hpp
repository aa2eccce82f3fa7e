// x87.hpp -- x86 80-bit extended precision (`long double` on x86-64) in
// software on gfx950, bit-exact with the x87 unit the reference's loops run on.
//
// The reference compiles `a[i] = a[i] + b[i]` on long double to
//   fldt a; fldt b; faddp; fstpt a
// (gcc -O2, probed), so each element is one x87 operation at the default
// 64-bit precision control, round-to-nearest-even, gradual underflow, and the
// 10-byte store leaves the 6 padding bytes of the 16-byte slot untouched.
// gfx950 has no 80-bit type, so the significand arithmetic is done in 64/128
// bit integers here.  x87 semantics restated (Intel SDM vol. 1 §4.8.3, §8.2,
// Table 4-7; each rule was checked against the host x87 by
// tests/test_oracle_x87.py):
//   * encodings: exponent 0 -> zero / denormal; exponent 0 with the explicit
//     integer bit set (pseudo-denormal) is accepted and read as exponent 1;
//     exponent 1..32766 with the integer bit clear (unnormal), and exponent
//     32767 with it clear (pseudo-infinity / pseudo-NaN) are invalid operands:
//     add / mul return the real indefinite (0xFFFF C000000000000000) even if the
//     other operand is a NaN, compares are unordered;
//   * NaNs: an SNaN is returned quieted; of two NaNs of the same kind (both
//     signalling or both quiet) the one with the larger significand wins, on a
//     tie the positive one; an SNaN paired with a QNaN yields the QNaN;
//   * inf - inf and 0 * inf give the real indefinite.
//
// The functions are host+device so that tests/progs/x87_check.cpp can compare
// them with the host's x87 on the CPU, millions of operations per second.
#pragma once
#include <stdint.h>
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define X87_FN __host__ __device__ __forceinline__
#else
#define X87_FN static inline
#endif

namespace mpir_hip {

struct alignas(16) x80 {
    uint64_t m;         // significand, explicit integer bit 63
    uint16_t se;        // sign bit 15, biased exponent 14..0
    uint16_t pad_[3];   // not part of the value; stores never touch it
};
static_assert(sizeof(x80) == 16, "x80 is the 16-byte long double slot");

typedef unsigned __int128 u128;

enum X80Class { X80_ZERO, X80_DENORM, X80_NORMAL, X80_INF, X80_QNAN, X80_SNAN, X80_INVALID };

X87_FN int x80_class(const x80 &v) {
    const uint32_t e = v.se & 0x7fffu;
    const bool j = (v.m >> 63) != 0;
    if (e == 0) return v.m == 0 ? X80_ZERO : X80_DENORM;        // incl. pseudo-denormal
    if (e == 0x7fffu) {
        if (!j) return X80_INVALID;                               // pseudo-inf / pseudo-NaN
        if ((v.m << 1) == 0) return X80_INF;
        return ((v.m >> 62) & 1) ? X80_QNAN : X80_SNAN;
    }
    return j ? X80_NORMAL : X80_INVALID;                          // unnormal
}

X87_FN x80 x80_make(uint32_t sign, uint32_t e, uint64_t m, const x80 &pad_from) {
    x80 r = pad_from;
    r.m = m;
    r.se = (uint16_t)((sign << 15) | e);
    return r;
}
X87_FN x80 x80_indefinite(const x80 &pad_from) {
    return x80_make(1, 0x7fff, 0xC000000000000000ull, pad_from);
}
X87_FN bool x80_is_nan_class(int c) { return c == X80_QNAN || c == X80_SNAN; }

// NaN propagation when at least one operand is a NaN and none is invalid
X87_FN x80 x80_nan_result(const x80 &a, const x80 &b, int ca, int cb, const x80 &pad) {
    const bool an = x80_is_nan_class(ca), bn = x80_is_nan_class(cb);
    bool take_a;
    if (an && bn) {
        if ((ca == X80_SNAN) != (cb == X80_SNAN)) take_a = ca == X80_QNAN;
        else if (a.m != b.m) take_a = a.m > b.m;
        else take_a = (a.se & 0x8000u) == 0;
    } else {
        take_a = an;
    }
    const uint64_t m = take_a ? a.m : b.m;
    const uint32_t sign = (uint32_t)(take_a ? a.se : b.se) >> 15;
    return x80_make(sign, 0x7fff, m | (1ull << 62), pad);
}

// leading-one position of a nonzero 128-bit value
X87_FN int x80_msb(u128 v) {
    const uint64_t hi = (uint64_t)(v >> 64), lo = (uint64_t)v;
    return hi ? 127 - __builtin_clzll(hi) : 63 - __builtin_clzll(lo);
}

// Round S * 2^(Eunb - 126 + ...) to the x87 extended format.  `s` is an exact
// (or sticky-augmented) 128-bit magnitude whose value is S * 2^(scale) with
// scale chosen by the caller so that a leading one at bit p gives the
// unbiased exponent Er = ebase + p.  Round-to-nearest-even, gradual
// underflow, overflow to infinity.
X87_FN x80 x80_round_pack(uint32_t sign, int ebase, u128 s, const x80 &pad) {
    if (s == 0) return x80_make(sign, 0, 0, pad);
    const int p = x80_msb(s);
    int er = ebase + p + 16383;          // biased exponent of the leading one
    int rs = p - 63;                     // right shift that leaves 64 significant bits
    if (er < 1) {                        // tiny: denormalise to exponent field 0
        rs += 1 - er;
        er = 0;
    }
    uint64_t sig;
    bool up;
    if (rs <= 0) {
        sig = (uint64_t)(s << (-rs));
        up = false;
    } else if (rs >= 128) {
        sig = 0;
        up = rs == 128 && s > ((u128)1 << 127);
    } else {
        const u128 rem = s & (((u128)1 << rs) - 1), half = (u128)1 << (rs - 1);
        sig = (uint64_t)(s >> rs);
        up = rem > half || (rem == half && (sig & 1));
    }
    if (up) {
        ++sig;
        if (sig == 0) {                  // carried out of 64 bits
            sig = 1ull << 63;
            ++er;
        } else if (er == 0 && (sig >> 63)) {
            er = 1;                      // rounded up into the normal range
        }
    }
    if (er >= 0x7fff) return x80_make(sign, 0x7fff, 1ull << 63, pad);
    return x80_make(sign, (uint32_t)er, sig, pad);
}

// unpack a finite (zero / denormal / pseudo-denormal / normal) value:
// value = m * 2^(E - 63)
X87_FN int x80_uexp(const x80 &v) {
    const int e = v.se & 0x7fff;
    return (e == 0 ? 1 : e) - 16383;
}

// finite, not both zero: sign, unbiased exponent (-100000 for a zero) and
// significand of each operand (the sign of b already flipped for a subtraction)
X87_FN x80 x80_addsub_core(uint32_t sa, uint32_t sb, int ea, int eb, uint64_t ma, uint64_t mb, const x80 &pad) {
    // order by magnitude: |a| >= |b|
    if (eb > ea || (eb == ea && mb > ma)) {
        int te = ea; ea = eb; eb = te;
        uint64_t tm = ma; ma = mb; mb = tm;
        uint32_t ts = sa; sa = sb; sb = ts;
    }
    if (mb == 0) return x80_round_pack(sa, ea - 126, (u128)ma << 63, pad);
    const int d = ea - eb;
    const u128 x = (u128)ma << 63;
    u128 y = (u128)mb << 63;
    if (d >= 127) {
        y = 1;                                      // pure sticky
    } else if (d > 0) {
        const bool sticky = (y & (((u128)1 << d) - 1)) != 0;
        y = (y >> d) | (sticky ? 1 : 0);
    }
    // Fast path: the larger significand has its integer bit (x in [2^126,
    // 2^127)), and either the signs agree or the exponents differ by >= 2, so
    // the result's leading one is at bit 127, 126 or 125 and the rounding
    // position is one of three fixed shifts (no 128-bit shifter, no clz).
    // Same rounding as x80_round_pack: the sticky bit sits in bit 0, far below.
    if ((ma >> 63) && (sa == sb || d >= 2)) {
        const u128 s = sa == sb ? x + y : x - y;
        const uint64_t hi = (uint64_t)(s >> 64), lo = (uint64_t)s;
        int p;
        uint64_t sig, rem, half;
        if (hi >> 63) { p = 127; sig = hi; rem = lo; half = 1ull << 63; }
        else if (hi >> 62) { p = 126; sig = (hi << 1) | (lo >> 63); rem = lo & ~(1ull << 63); half = 1ull << 62; }
        else { p = 125; sig = (hi << 2) | (lo >> 62); rem = lo & ((1ull << 62) - 1); half = 1ull << 61; }
        int er = ea - 126 + p + 16383;
        if (er >= 1 && er <= 0x7ffe) {
            if (rem > half || (rem == half && (sig & 1))) {
                if (++sig == 0) {
                    sig = 1ull << 63;
                    if (++er >= 0x7fff) return x80_make(sa, 0x7fff, 1ull << 63, pad);
                }
            }
            return x80_make(sa, (uint32_t)er, sig, pad);
        }
    }
    if (sa == sb) return x80_round_pack(sa, ea - 126, x + y, pad);
    const u128 s = x - y;
    if (s == 0) return x80_make(0, 0, 0, pad);      // exact cancellation: +0 (round to nearest)
    return x80_round_pack(sa, ea - 126, s, pad);
}


// result = a + b (sub: a - b); the pad bytes of the result are `pad`'s
X87_FN x80 x80_addsub(x80 a, x80 b, bool sub, const x80 &pad) {
    const int ca = x80_class(a), cb = x80_class(b);
    if (ca == X80_INVALID || cb == X80_INVALID) return x80_indefinite(pad);
    if (x80_is_nan_class(ca) || x80_is_nan_class(cb)) return x80_nan_result(a, b, ca, cb, pad);
    uint32_t sa = a.se >> 15, sb = (b.se >> 15) ^ (sub ? 1u : 0u);
    if (ca == X80_INF || cb == X80_INF) {
        if (ca == X80_INF && cb == X80_INF && sa != sb) return x80_indefinite(pad);
        return x80_make(ca == X80_INF ? sa : sb, 0x7fff, 1ull << 63, pad);
    }
    if (ca == X80_ZERO && cb == X80_ZERO) return x80_make(sa & sb, 0, 0, pad);
    const int ea = ca == X80_ZERO ? -100000 : x80_uexp(a), eb = cb == X80_ZERO ? -100000 : x80_uexp(b);
    return x80_addsub_core(sa, sb, ea, eb, a.m, b.m, pad);
}

// a + b (sub: a - b) of two NORMAL values (integer bit set, exponent field
// 1..32766): x80_addsub without the class checks, which cannot fire
X87_FN x80 x80_addsub_normal(const x80 &a, const x80 &b, bool sub, const x80 &pad) {
    return x80_addsub_core(a.se >> 15, (b.se >> 15) ^ (sub ? 1u : 0u), (int)(a.se & 0x7fff) - 16383,
                           (int)(b.se & 0x7fff) - 16383, a.m, b.m, pad);
}
X87_FN x80 x80_add(x80 a, x80 b, const x80 &pad) { return x80_addsub(a, b, false, pad); }
X87_FN x80 x80_sub(x80 a, x80 b, const x80 &pad) { return x80_addsub(a, b, true, pad); }

X87_FN x80 x80_mul(x80 a, x80 b, const x80 &pad) {
    const int ca = x80_class(a), cb = x80_class(b);
    if (ca == X80_INVALID || cb == X80_INVALID) return x80_indefinite(pad);
    if (x80_is_nan_class(ca) || x80_is_nan_class(cb)) return x80_nan_result(a, b, ca, cb, pad);
    const uint32_t s = (a.se >> 15) ^ (b.se >> 15);
    if (ca == X80_INF || cb == X80_INF) {
        if (ca == X80_ZERO || cb == X80_ZERO) return x80_indefinite(pad);
        return x80_make(s, 0x7fff, 1ull << 63, pad);
    }
    if (ca == X80_ZERO || cb == X80_ZERO) return x80_make(s, 0, 0, pad);
    const u128 prod = (u128)a.m * (u128)b.m;       // value = prod * 2^(Ea + Eb - 126)
    if (ca == X80_NORMAL && cb == X80_NORMAL) {
        // both significands in [2^63, 2^64): the product's leading one is at
        // bit 126 or 127, so the rounding position is fixed (no 128-bit shifter)
        const bool top = (uint64_t)(prod >> 127) != 0;
        const int er = (int)(a.se & 0x7fff) + (int)(b.se & 0x7fff) - 16383 + (top ? 1 : 0);
        if (er >= 1 && er <= 0x7ffe) {
            const uint64_t hi = (uint64_t)(prod >> 64), lo = (uint64_t)prod;
            uint64_t sig, rem, half;
            if (top) { sig = hi; rem = lo; half = 1ull << 63; }
            else { sig = (hi << 1) | (lo >> 63); rem = lo & ~(1ull << 63); half = 1ull << 62; }
            if (rem > half || (rem == half && (sig & 1))) {
                if (++sig == 0) {
                    if (er + 1 >= 0x7fff) return x80_make(s, 0x7fff, 1ull << 63, pad);
                    return x80_make(s, (uint32_t)(er + 1), 1ull << 63, pad);
                }
            }
            return x80_make(s, (uint32_t)er, sig, pad);
        }
    }
    return x80_round_pack(s, x80_uexp(a) + x80_uexp(b) - 126, prod, pad);
}

// ordered comparison of two non-NaN, valid values: -1, 0, +1
X87_FN int x80_cmp_ordered(const x80 &a, const x80 &b, int ca, int cb) {
    const bool za = ca == X80_ZERO, zb = cb == X80_ZERO;
    if (za && zb) return 0;
    const uint32_t sa = za ? 0 : a.se >> 15, sb = zb ? 0 : b.se >> 15;
    const int ea = za ? 0 : ((a.se & 0x7fff) == 0 ? 1 : (a.se & 0x7fff));
    const int eb = zb ? 0 : ((b.se & 0x7fff) == 0 ? 1 : (b.se & 0x7fff));
    const uint64_t ma = za ? 0 : a.m, mb = zb ? 0 : b.m;
    int mag = ea != eb ? (ea < eb ? -1 : 1) : (ma == mb ? 0 : (ma < mb ? -1 : 1));
    if (za) return sb ? 1 : -1;
    if (zb) return sa ? -1 : 1;
    if (sa != sb) return sa ? -1 : 1;
    return sa ? -mag : mag;
}

// fcomi / fucomi: unordered when either operand is a NaN or an invalid encoding
X87_FN bool x80_unordered(int ca, int cb) {
    return x80_is_nan_class(ca) || x80_is_nan_class(cb) || ca == X80_INVALID || cb == X80_INVALID;
}
X87_FN bool x80_gt(const x80 &a, const x80 &b) {
    const int ca = x80_class(a), cb = x80_class(b);
    return !x80_unordered(ca, cb) && x80_cmp_ordered(a, b, ca, cb) > 0;
}
X87_FN bool x80_lt(const x80 &a, const x80 &b) { return x80_gt(b, a); }
X87_FN bool x80_ge(const x80 &a, const x80 &b) {
    const int ca = x80_class(a), cb = x80_class(b);
    return !x80_unordered(ca, cb) && x80_cmp_ordered(a, b, ca, cb) >= 0;
}
X87_FN bool x80_le(const x80 &a, const x80 &b) { return x80_ge(b, a); }

// `v != 0` as compiled (fucomi against 0: unordered counts as true)
X87_FN bool x80_truth(const x80 &v) { return x80_class(v) != X80_ZERO; }
// __builtin_isnan (x != x via fucomi) and __builtin_isinf (|x| > LDBL_MAX)
X87_FN bool x80_isnan(const x80 &v) {
    const int c = x80_class(v);
    return x80_is_nan_class(c) || c == X80_INVALID;
}
X87_FN bool x80_isinf(const x80 &v) { return x80_class(v) == X80_INF; }
// copysign(k, v) for k in {0, 1}
X87_FN x80 x80_signed_const(int one, const x80 &v, const x80 &pad) {
    return x80_make(v.se >> 15, one ? 0x3fff : 0, one ? (1ull << 63) : 0, pad);
}
X87_FN x80 x80_one(const x80 &pad) { return x80_make(0, 0x3fff, 1ull << 63, pad); }
X87_FN x80 x80_zero(const x80 &pad) { return x80_make(0, 0, 0, pad); }

// Product of two normal values whose biased exponents both lie in
// [kX80SafeLo, kX80SafeHi]: the result is normal and finite (its biased
// exponent stays within [17, 32739] even after a rounding carry), so no class
// checks and no general rounder; same rounding as x80_mul's normal path.
constexpr int kX80SafeLo = 8200, kX80SafeHi = 24560;
X87_FN x80 x80_mul_safe(const x80 &a, const x80 &b, const x80 &pad) {
    const uint32_t s = (a.se >> 15) ^ (b.se >> 15);
    const u128 prod = (u128)a.m * (u128)b.m;
    const uint64_t hi = (uint64_t)(prod >> 64), lo = (uint64_t)prod;
    const bool top = (hi >> 63) != 0;
    int er = (int)(a.se & 0x7fff) + (int)(b.se & 0x7fff) - 16383 + (top ? 1 : 0);
    uint64_t sig, rem, half;
    if (top) { sig = hi; rem = lo; half = 1ull << 63; }
    else { sig = (hi << 1) | (lo >> 63); rem = lo & ~(1ull << 63); half = 1ull << 62; }
    if (rem > half || (rem == half && (sig & 1))) {
        if (++sig == 0) { sig = 1ull << 63; ++er; }
    }
    return x80_make(s, (uint32_t)er, sig, pad);
}
X87_FN bool x80_in_safe_range(const x80 &v) {
    const int e = v.se & 0x7fff;
    return (v.m >> 63) && e >= kX80SafeLo && e <= kX80SafeHi;
}

// C99 Annex G multiply for long double _Complex, as gcc emits it: the inline
// ac - bd / ad + bc, and __mulxc3's recovery when both parts are NaN.
X87_FN void x80_cmul(x80 a, x80 b, x80 c, x80 d, x80 &x, x80 &y) {
    const x80 pa = a, pb = b;   // result pads come from the inout element
    // Fast path: four normal parts of moderate exponent.  The four products
    // are normal and finite, so x and y can be neither NaN (no recovery) nor
    // invalid, and x80_addsub's class checks pass straight through.
    if (__builtin_expect(x80_in_safe_range(a) && x80_in_safe_range(b) && x80_in_safe_range(c) &&
                         x80_in_safe_range(d), 1)) {
        x = x80_addsub_normal(x80_mul_safe(a, c, pa), x80_mul_safe(b, d, pa), true, pa);
        y = x80_addsub_normal(x80_mul_safe(a, d, pb), x80_mul_safe(b, c, pb), false, pb);
        return;
    }
    x80 ac = x80_mul(a, c, pa), bd = x80_mul(b, d, pa), ad = x80_mul(a, d, pb), bc = x80_mul(b, c, pb);
    x = x80_sub(ac, bd, pa);
    y = x80_add(ad, bc, pb);
    if (__builtin_expect(x80_isnan(x) && x80_isnan(y), 0)) {
        bool recalc = false;
        if (x80_isinf(a) || x80_isinf(b)) {
            a = x80_signed_const(x80_isinf(a), a, pa);
            b = x80_signed_const(x80_isinf(b), b, pb);
            if (x80_isnan(c)) c = x80_signed_const(0, c, c);
            if (x80_isnan(d)) d = x80_signed_const(0, d, d);
            recalc = true;
        }
        if (x80_isinf(c) || x80_isinf(d)) {
            c = x80_signed_const(x80_isinf(c), c, c);
            d = x80_signed_const(x80_isinf(d), d, d);
            if (x80_isnan(a)) a = x80_signed_const(0, a, pa);
            if (x80_isnan(b)) b = x80_signed_const(0, b, pb);
            recalc = true;
        }
        if (!recalc && (x80_isinf(ac) || x80_isinf(bd) || x80_isinf(ad) || x80_isinf(bc))) {
            if (x80_isnan(a)) a = x80_signed_const(0, a, pa);
            if (x80_isnan(b)) b = x80_signed_const(0, b, pb);
            if (x80_isnan(c)) c = x80_signed_const(0, c, c);
            if (x80_isnan(d)) d = x80_signed_const(0, d, d);
            recalc = true;
        }
        if (recalc) {
            const x80 inf = x80_make(0, 0x7fff, 1ull << 63, pa);
            x = x80_mul(inf, x80_sub(x80_mul(a, c, pa), x80_mul(b, d, pa), pa), pa);
            y = x80_mul(inf, x80_add(x80_mul(a, d, pb), x80_mul(b, c, pb), pb), pb);
        }
    }
}

}  // namespace mpir_hip

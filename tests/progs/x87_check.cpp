// x87_check.cpp -- the soft x87 arithmetic of mpich-pip_amd/csrc/hip/x87.hpp
// (what the gfx950 long double kernels run) against the host's x87 unit,
// which is what the reference's `long double` loops run on.
//
//   g++ -O2 -I mpich-pip_amd/csrc/hip tests/progs/x87_check.cpp -o x87_check
//   ./x87_check [pairs=2000000] [seed=1]
//
// Operands mix every encoding class: normals across the whole exponent range
// (and clustered so that additions cancel and round), denormals,
// pseudo-denormals, zeros, infinities, quiet / signalling NaNs with random
// payloads and signs, unnormals, pseudo-infinities and pseudo-NaNs.
// Checked bit for bit (10 value bytes): +, -, *, the four ordered compares,
// `!= 0`, and C99 Annex G complex * (NaN results compared as NaN-class).
// Prints one summary line per op; exit status 1 on any mismatch.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <initializer_list>

#include "x87.hpp"

using namespace mpir_hip;

static uint64_t rs;
static uint64_t rnd() {   // xorshift64*
    rs ^= rs >> 12; rs ^= rs << 25; rs ^= rs >> 27;
    return rs * 2685821657736338717ull;
}

static x80 gen() {
    x80 v;
    memset(&v, 0, sizeof v);
    const uint32_t sign = (uint32_t)(rnd() & 1) << 15;
    const int k = (int)(rnd() % 100);
    uint64_t m = rnd();
    uint32_t e;
    if (k < 40) {            // normal, exponent near 1.0
        e = 0x3fff - 40 + (uint32_t)(rnd() % 80);
        m |= 1ull << 63;
        if (rnd() & 1) m &= ~0ull << (rnd() % 64);   // short significands -> exact / tie cases
    } else if (k < 52) {     // normal, anywhere; half of them at the edges of x80_cmul's fast-path range
        e = (rnd() & 1) ? 1 + (uint32_t)(rnd() % 0x7ffe) : ((rnd() & 1) ? 8200u : 24560u) - 3 + (uint32_t)(rnd() % 7);
        m |= 1ull << 63;
    } else if (k < 60) {     // near the bottom of the range
        e = 1 + (uint32_t)(rnd() % 80);
        m |= 1ull << 63;
    } else if (k < 66) {     // near the top
        e = 0x7ffe - (uint32_t)(rnd() % 40);
        m |= 1ull << 63;
    } else if (k < 72) {     // denormal
        e = 0;
        m &= ~(1ull << 63);
        if (rnd() & 1) m >>= rnd() % 63;
    } else if (k < 75) {     // pseudo-denormal
        e = 0;
        m |= 1ull << 63;
    } else if (k < 79) {     // zero
        e = 0;
        m = 0;
    } else if (k < 83) {     // infinity
        e = 0x7fff;
        m = 1ull << 63;
    } else if (k < 89) {     // quiet NaN
        e = 0x7fff;
        m |= 3ull << 62;
        if (rnd() & 1) m = (3ull << 62) | (rnd() % 4);
    } else if (k < 94) {     // signalling NaN
        e = 0x7fff;
        m = (1ull << 63) | (m & ((1ull << 62) - 1)) | 1;
        if (rnd() & 1) m = (1ull << 63) | (1 + rnd() % 4);
    } else if (k < 97) {     // unnormal
        e = 1 + (uint32_t)(rnd() % 0x7ffe);
        m &= ~(1ull << 63);
    } else {                 // pseudo-infinity / pseudo-NaN
        e = 0x7fff;
        m &= ~(1ull << 63);
        if (rnd() & 1) m = 0;
    }
    v.m = m;
    v.se = (uint16_t)(sign | e);
    return v;
}

static long double to_ld(const x80 &v) {
    long double r;
    memset(&r, 0, sizeof r);
    memcpy(&r, &v, 10);
    return r;
}
static bool same10(const x80 &a, long double b) { return memcmp(&a, &b, 10) == 0; }
static bool is_nan_ld(long double v) { return v != v; }

// host x87 operations, kept out of line so each is one compiled x87 instruction
__attribute__((noinline)) static long double h_add(long double a, long double b) { return a + b; }
__attribute__((noinline)) static long double h_sub(long double a, long double b) { return a - b; }
__attribute__((noinline)) static long double h_mul(long double a, long double b) { return a * b; }
__attribute__((noinline)) static long double _Complex h_cmul(long double _Complex a, long double _Complex b) {
    return a * b;
}

struct Tally {
    const char *name;
    long n = 0, bad = 0;
    void note(bool ok, const x80 &a, const x80 &b, const void *got, const void *want) {
        ++n;
        if (ok) return;
        if (++bad <= 5) {
            uint64_t gm, wm;
            uint16_t gs, ws;
            memcpy(&gm, got, 8); memcpy(&gs, (const char *)got + 8, 2);
            memcpy(&wm, want, 8); memcpy(&ws, (const char *)want + 8, 2);
            fprintf(stderr, "%s mismatch: a=%04x:%016llx b=%04x:%016llx got %04x:%016llx want %04x:%016llx\n", name,
                    a.se, (unsigned long long)a.m, b.se, (unsigned long long)b.m, gs, (unsigned long long)gm, ws,
                    (unsigned long long)wm);
        }
    }
};

int main(int argc, char **argv) {
    const long pairs = argc > 1 ? atol(argv[1]) : 2000000;
    rs = 0x9E3779B97F4A7C15ull ^ (uint64_t)(argc > 2 ? atol(argv[2]) : 1);
    Tally t_add{"add"}, t_sub{"sub"}, t_mul{"mul"}, t_cmp{"compare"}, t_truth{"truth"}, t_cmul{"cmul"};
    for (long i = 0; i < pairs; ++i) {
        x80 a = gen(), b = gen();
        // cluster: make b close to +-a so additions cancel and round
        if ((rnd() % 8) == 0 && x80_class(a) == X80_NORMAL) {
            b = a;
            b.m ^= rnd() >> (rnd() % 64);
            b.m |= 1ull << 63;
            if (rnd() & 1) b.se ^= 0x8000;
        }
        const long double la = to_ld(a), lb = to_ld(b);
        long double w;
        x80 g;
        g = x80_add(a, b, a); w = h_add(la, lb); t_add.note(same10(g, w), a, b, &g, &w);
        g = x80_sub(a, b, a); w = h_sub(la, lb); t_sub.note(same10(g, w), a, b, &g, &w);
        g = x80_mul(a, b, a); w = h_mul(la, lb); t_mul.note(same10(g, w), a, b, &g, &w);
        const int got = (x80_gt(a, b) << 3) | (x80_lt(a, b) << 2) | (x80_ge(a, b) << 1) | (int)x80_le(a, b);
        const int want = ((la > lb) << 3) | ((la < lb) << 2) | ((la >= lb) << 1) | (int)(la <= lb);
        t_cmp.note(got == want, a, b, &got, &want);
        const int gt = x80_truth(a), wt = la != 0;
        t_truth.note(gt == wt, a, a, &gt, &wt);
        // complex: (a + i b) * (c + i d) with c, d fresh
        x80 c = gen(), d = gen(), x, y;
        x80_cmul(a, b, c, d, x, y);
        long double _Complex za, zb, zr;
        __real__ za = la; __imag__ za = lb;
        __real__ zb = to_ld(c); __imag__ zb = to_ld(d);
        zr = h_cmul(za, zb);
        const long double wr = __real__ zr, wi = __imag__ zr;
        const bool ok_r = is_nan_ld(wr) ? x80_isnan(x) : same10(x, wr);
        const bool ok_i = is_nan_ld(wi) ? x80_isnan(y) : same10(y, wi);
        t_cmul.note(ok_r && ok_i, a, c, ok_r ? (const void *)&y : (const void *)&x, ok_r ? (const void *)&wi : (const void *)&wr);
    }
    int rc = 0;
    for (Tally *t : {&t_add, &t_sub, &t_mul, &t_cmp, &t_truth, &t_cmul}) {
        printf("%-8s %ld ops, %ld mismatches\n", t->name, t->n, t->bad);
        rc |= t->bad != 0;
    }
    return rc;
}

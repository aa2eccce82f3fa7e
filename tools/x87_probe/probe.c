#include <stdio.h>
#include <stdint.h>
#include <string.h>
void lsum(long double *restrict a, const long double *restrict b, int n);
void lprod(long double *restrict a, const long double *restrict b, int n) ;
void lmax(long double *restrict a, const long double *restrict b, int n);
typedef struct { uint64_t m; uint16_t se; } x80;
static long double mk(uint16_t se, uint64_t m) { long double v; memset(&v, 0xAB, 16); memcpy(&v, &m, 8); memcpy((char*)&v+8, &se, 2); return v; }
static void show(const char *t, long double v) { unsigned char b[16]; memcpy(b, &v, 16); uint64_t m; uint16_t se; memcpy(&m, b, 8); memcpy(&se, b+8, 2);
  printf("%-34s se=%04x m=%016llx pad=%02x%02x\n", t, se, (unsigned long long)m, b[10], b[15]); }
int main(void) {
  struct { const char *n; long double a, b; } c[] = {
   {"qnan1 + qnan2(larger)", mk(0x7fff, 0xC000000000000001ull), mk(0x7fff, 0xC000000000000002ull)},
   {"qnan2(larger) + qnan1", mk(0x7fff, 0xC000000000000002ull), mk(0x7fff, 0xC000000000000001ull)},
   {"+qnan + -qnan same sig", mk(0x7fff, 0xC000000000000005ull), mk(0xffff, 0xC000000000000005ull)},
   {"-qnan + +qnan same sig", mk(0xffff, 0xC000000000000005ull), mk(0x7fff, 0xC000000000000005ull)},
   {"snan(big) + qnan(small)", mk(0x7fff, 0x8000000000000009ull), mk(0x7fff, 0xC000000000000001ull)},
   {"qnan(small) + snan(big)", mk(0x7fff, 0xC000000000000001ull), mk(0x7fff, 0x8000000000000009ull)},
   {"snan1 + snan2", mk(0x7fff, 0x8000000000000001ull), mk(0x7fff, 0x8000000000000002ull)},
   {"snan2 + snan1", mk(0x7fff, 0x8000000000000002ull), mk(0x7fff, 0x8000000000000001ull)},
   {"1 + snan", mk(0x3fff, 0x8000000000000000ull), mk(0x7fff, 0x8000000000000003ull)},
   {"unnormal + 1", mk(0x3fff, 0x4000000000000000ull), mk(0x3fff, 0x8000000000000000ull)},
   {"1 + unnormal", mk(0x3fff, 0x8000000000000000ull), mk(0x3fff, 0x4000000000000000ull)},
   {"unnormal + qnan", mk(0x3fff, 0x4000000000000000ull), mk(0x7fff, 0xC000000000000007ull)},
   {"pseudo-inf + 1", mk(0x7fff, 0x0000000000000000ull), mk(0x3fff, 0x8000000000000000ull)},
   {"pseudo-nan + 1", mk(0x7fff, 0x4000000000000001ull), mk(0x3fff, 0x8000000000000000ull)},
   {"pseudo-denorm + 0", mk(0x0000, 0x8000000000000001ull), mk(0x0000, 0x0ull)},
   {"pseudo-denorm + tiny", mk(0x0000, 0x8000000000000001ull), mk(0x0000, 0x1ull)},
   {"inf + -inf", mk(0x7fff, 0x8000000000000000ull), mk(0xffff, 0x8000000000000000ull)},
   {"unnormal0(exp>0,m=0) + 1", mk(0x1234, 0x0ull), mk(0x3fff, 0x8000000000000000ull)},
  };
  for (unsigned i = 0; i < sizeof c / sizeof c[0]; i++) {
    long double a = c[i].a, b = c[i].b; lsum(&a, &b, 1); char t[64]; snprintf(t, 64, "SUM %s", c[i].n); show(t, a);
    a = c[i].a; b = c[i].b; lprod(&a, &b, 1); snprintf(t, 64, "PROD %s", c[i].n); show(t, a);
    a = c[i].a; b = c[i].b; lmax(&a, &b, 1); snprintf(t, 64, "MAX %s", c[i].n); show(t, a);
  }
  return 0;
}

#include <stdio.h>
#include <stdint.h>
#include <string.h>
void lsum(long double *restrict a, const long double *restrict b, int n);
void lprod(long double *restrict a, const long double *restrict b, int n) ;
static long double mk(uint16_t se, uint64_t m) { long double v; memset(&v, 0, 16); memcpy(&v, &m, 8); memcpy((char*)&v+8, &se, 2); return v; }
static void show(const char *t, long double v) { uint64_t m; uint16_t se; memcpy(&m, &v, 8); memcpy(&se, (char*)&v+8, 2);
  printf("%-34s se=%04x m=%016llx\n", t, se, (unsigned long long)m); }
int main(void) {
  struct { const char *n; long double a, b; } c[] = {
   {"-snan + +snan same sig", mk(0xffff, 0x8000000000000005ull), mk(0x7fff, 0x8000000000000005ull)},
   {"+snan + -snan same sig", mk(0x7fff, 0x8000000000000005ull), mk(0xffff, 0x8000000000000005ull)},
   {"-qnan + -qnan same sig", mk(0xffff, 0xC000000000000005ull), mk(0xffff, 0xC000000000000005ull)},
   {"-qnan(big) + +qnan(small)", mk(0xffff, 0xC000000000000009ull), mk(0x7fff, 0xC000000000000005ull)},
   {"+qnan(small) + -qnan(big)", mk(0x7fff, 0xC000000000000005ull), mk(0xffff, 0xC000000000000009ull)},
   {"-snan + 1", mk(0xffff, 0x8000000000000005ull), mk(0x3fff, 0x8000000000000000ull)},
   {"denorm*2^k", mk(0x0000, 0x0000000000000003ull), mk(0x3ffe, 0x8000000000000000ull)},
   {"tiny*tiny", mk(0x0001, 0x8000000000000001ull), mk(0x3fbf, 0xC000000000000001ull)},
  };
  for (unsigned i = 0; i < sizeof c / sizeof c[0]; i++) {
    long double a = c[i].a, b = c[i].b; lsum(&a, &b, 1); char t[64]; snprintf(t, 64, "SUM %s", c[i].n); show(t, a);
    a = c[i].a; b = c[i].b; lprod(&a, &b, 1); snprintf(t, 64, "PROD %s", c[i].n); show(t, a);
  }
  return 0;
}

typedef struct { long double value; int loc; } ldi;
void lmax(long double *restrict a, const long double *restrict b, int n) { for (int i = 0; i < n; i++) a[i] = (a[i] > b[i]) ? a[i] : b[i]; }
void lsum(long double *restrict a, const long double *restrict b, int n) { for (int i = 0; i < n; i++) a[i] = a[i] + b[i]; }
void llxor(long double *restrict a, const long double *restrict b, int n) { for (int i = 0; i < n; i++) a[i] = ((a[i] && !b[i]) || (!a[i] && b[i])); }
void lmaxloc(ldi *restrict a, const ldi *restrict b, int n) {
  for (int i = 0; i < n; i++) {
    if (a[i].value < b[i].value) { a[i].value = b[i].value; a[i].loc = b[i].loc; }
    else if (a[i].value <= b[i].value) a[i].loc = (a[i].loc < b[i].loc) ? a[i].loc : b[i].loc;
  }
}
void cprod(long double _Complex *restrict a, const long double _Complex *restrict b, int n) { for (int i = 0; i < n; i++) a[i] = a[i] * b[i]; }
void lprod(long double *restrict a, const long double *restrict b, int n) { for (int i = 0; i < n; i++) a[i] = a[i] * b[i]; }

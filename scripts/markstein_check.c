// Markstein quotient check: y = RN(1/b), q0 = RN(a y), r = fma(-q0, b, a), q = fma(r, y, q0)
// against the IEEE quotient a / b on random fp32 pairs.  gcc -O2 -ffp-contract=off scripts/markstein_check.c -lm
#include <stdlib.h>
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
static uint64_t s = 88172645463325252ull;
static inline uint64_t xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static inline float rf(int emin, int emax) {
  uint32_t m = (uint32_t)(xr() & 0x7fffff);
  int e = emin + (int)(xr() % (uint64_t)(emax - emin + 1));
  uint32_t bits = ((uint32_t)(e + 127) << 23) | m | ((xr() & 1) ? 0x80000000u : 0);
  float f; memcpy(&f, &bits, 4); return f;
}
int main(int argc, char** argv) {
  long n = atol(argv[1]); long bad = 0;
  for (long i = 0; i < n; ++i) {
    float a = rf(-60, 60), b = rf(-60, 60);
    if ((i & 15) == 0) { float t = b; uint32_t u; memcpy(&u, &t, 4); u |= 0x7fffff; memcpy(&b, &u, 4); }  // all-ones mantissas
    if ((i & 15) == 1) { uint32_t u; memcpy(&u, &b, 4); u &= 0xff800000u; memcpy(&b, &u, 4); }             // powers of two
    volatile float y = 1.0f / b;
    float q0 = a * y;
    float r = fmaf(-q0, b, a);
    float q = fmaf(r, y, q0);
    float ref = a / b;
    if (memcmp(&q, &ref, 4) != 0) { if (bad < 10) printf("mismatch a=%a b=%a q=%a ref=%a\n", a, b, q, ref); ++bad; }
  }
  printf("%ld samples, %ld mismatches\n", n, bad);
  return 0;
}

// Exhaustive-ish CPU check that the Markstein division used by the encoder
// (q0 = x*r; two fma corrections; r = RN(1/b)) equals IEEE x/b.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static inline float f(uint32_t u) { float x; memcpy(&x, &u, 4); return x; }
static inline uint32_t b(float x) { uint32_t u; memcpy(&u, &x, 4); return u; }
static uint64_t s = 88172645463325252ull;
static inline uint64_t rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static inline float mdiv(float x, float d, float r) {
  float q = x * r;
  float e = fmaf(-q, d, x);
  q = fmaf(e, r, q);
  e = fmaf(-q, d, x);
  return fmaf(e, r, q);
}
int main(int argc, char** argv) {
  long n = argc > 1 ? atol(argv[1]) : 200000000L;
  long bad = 0, tiny = 0;
  for (long i = 0; i < n; ++i) {
    uint64_t r64 = rnd();
    // divisor: normal, exponent in [-100, 100]
    float d = f(((uint32_t)(127 - 100 + (r64 % 201)) << 23) | ((uint32_t)(r64 >> 20) & 0x7fffff));
    float r = 1.0f / d;
    // numerator: |x| <= ~d mostly, occasionally any exponent down to d*2^-60
    uint64_t r2 = rnd();
    int ex = (int)((b(d) >> 23) & 0xff) - (int)(r2 % 64);
    if (ex < 1) ex = 1;
    float x = f(((uint32_t)ex << 23) | ((uint32_t)(r2 >> 16) & 0x7fffff) | ((r2 >> 63) ? 0x80000000u : 0));
    if (i % 4 == 0) {  // near-halfway quotients: x = d * (k + 0.5 ulp) patterns
      float k = f(0x3f800000u | ((uint32_t)(r2 >> 30) & 0x7fffff));
      x = k * d;
      x = f(b(x) + (uint32_t)((int)(r2 % 5) - 2));
    }
    float want = x / d;
    float got = mdiv(x, d, r);
    if (fabsf(want) < 0x1p-100f || fabsf(x) < 0x1p-96f) { ++tiny; continue; }  // encoder takes x / d there
    if (b(want) != b(got)) { if (bad < 10) printf("x=%a d=%a want=%a got=%a\n", x, d, want, got); ++bad; }
  }
  printf("n=%ld mismatches=%ld tiny-skipped=%ld\n", n, bad, tiny);
  return bad != 0;
}

// spec_check.c — CPU check of the bracketed single-read encoder's decision rule
// (omf_qsgd_spec.hip): for a norm known only to lie in [n_lo, n_hi],
//   dl = fma(|x|, c_lo, -u), dh = fma(|x|, c_hi, -u)   with c_lo = L/n_hi (1 - 2^-20) rounded down,
//   c_hi = L/n_lo (1 + 2^-20) rounded up; the level is decided when ceil(dl) == ceil(dh), and is then
//   ceil(dh) with the sign of x; dl uses max(u, 2^-26) so that an element whose x / n could
//   underflow to 0 where |x| * c does not is left undecided when u == 0.  The bracket needs
//   n_lo >= 2^-90 so that c_hi is finite for L <= 2^30, and L >= 2.
// Claim: for every norm n in [n_lo, n_hi], a decided level equals the reference's exact level
//   vn = RN(x / n); a = |vn * L|; fl = floor(a); m = min(fl + (u < a - fl), L)   (qsgd.py:50-63).
// The check draws brackets, norms inside them, inputs (random, and constructed so that x/n*L
// lands within a few ulps of the decision points j + u) and 24-bit uniforms, and counts
// mismatches (must be 0) and the undecided fraction.  Build: gcc -O2 -o spec_check spec_check.c -lm
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static uint64_t rnd64(void) {
  rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17;
  return rs;
}
static double rnd01(void) { return (double)(rnd64() >> 11) * 0x1p-53; }

static float ref_level(float x, float n, float L, float u) {
  const float vn = x / n;
  const float a = fabsf(vn * L);
  const float fl = floorf(a);
  const float p = a - fl;
  float m = (u < p) ? fl + 1.0f : fl;
  m = fminf(m, L);
  return copysignf(m, vn);
}

// Outward-rounded multipliers of the bracket (the bracket kernel's computation).
static void bracket_c(float n_lo, float n_hi, float L, float* c_lo, float* c_hi) {
  const double lo = (double)L / (double)n_hi * (1.0 - 0x1p-20);
  const double hi = (double)L / (double)n_lo * (1.0 + 0x1p-20);
  *c_lo = nextafterf((float)lo, 0.0f);
  *c_hi = nextafterf((float)hi, INFINITY);
}

int main(int argc, char** argv) {
  const long iters = argc > 1 ? atol(argv[1]) : 20000000L;
  long mism = 0, undec = 0, tested = 0;
  for (long it = 0; it < iters; ++it) {
    const int s = 1 + (int)(rnd64() % 12);  // L >= 2
    const float L = (float)(1u << s);
    // bracket around a centre norm, relative half-width up to 10 %
    const float nc = (float)ldexp(1.0 + rnd01(), (int)(rnd64() % 150) - 88);  // [2^-88, 2^62)
    const double w = rnd01() * 0.1;
    const float n_lo = (float)(nc * (1.0 - w)), n_hi = nextafterf((float)(nc * (1.0 + w)), INFINITY);
    float c_lo, c_hi;
    bracket_c(n_lo, n_hi, L, &c_lo, &c_hi);
    // the true norm: an end point or a random point of the bracket
    const int pick = (int)(rnd64() % 4);
    float n = pick == 0 ? n_lo : pick == 1 ? n_hi : (float)(n_lo + (n_hi - n_lo) * rnd01());
    if (n < n_lo) n = n_lo;
    if (n > n_hi) n = n_hi;
    const float u = (rnd64() % 8 == 0) ? 0.0f : (float)(rnd64() & 0xFFFFFF) * 0x1p-24f;
    float x;
    const int mode = (int)(rnd64() % 4);
    if (mode == 0) {  // random magnitude up to the norm
      x = (float)(n * rnd01() * (rnd64() & 1 ? 1.0 : 1e-3));
    } else if (mode == 1) {  // at a decision point j + u for the TRUE norm, +- a few ulps
      const double j = floor(rnd01() * L);
      float t = (float)((j + u) / L * n);
      const int k = (int)(rnd64() % 9) - 4;
      for (int q = 0; q < abs(k); ++q) t = nextafterf(t, k > 0 ? INFINITY : 0.0f);
      x = t;
    } else if (mode == 2) {  // at a decision point for the bracket's end points
      const double j = floor(rnd01() * L);
      float t = (float)((j + u) / L * (rnd64() & 1 ? n_lo : n_hi));
      const int k = (int)(rnd64() % 9) - 4;
      for (int q = 0; q < abs(k); ++q) t = nextafterf(t, k > 0 ? INFINITY : 0.0f);
      x = t;
    } else {  // tiny magnitudes, down to the subnormal range, relative to the norm
      x = (float)(n * ldexp(rnd01(), -(int)(rnd64() % 160)));
    }
    if (rnd64() & 1) x = -x;
    if (fabsf(x) > n) continue;  // |x| <= norm: the norm is the tensor's own
    ++tested;
    const float ax = fabsf(x);
    // u == 0 is raised to 2^-26 in the lower product only: x / n may underflow to 0 where
    // |x| * c does not, and that element is then left undecided (dl < 0 < dh).  A decided
    // level needs no clamp (ceil(dl) <= the exact level <= L).
    const float dl = fmaf(ax, c_lo, -fmaxf(u, 0x1p-26f)), dh = fmaf(ax, c_hi, -u);
    const float kl = ceilf(dl), kh = ceilf(dh);
    if (kl != kh) {
      ++undec;
      continue;
    }
    const float m = copysignf(kh, x);
    const float r = ref_level(x, n, L, u);
    if ((int)m != (int)r) {
      if (mism < 10)
        printf("MISMATCH x=%a n=%a [%a,%a] L=%g u=%a: spec %g ref %g\n", x, n, n_lo, n_hi, L, u, m, r);
      ++mism;
    }
  }
  printf("tested %ld undecided %ld (%.4f) mismatches %ld\n", tested, undec, (double)undec / tested, mism);
  return mism != 0;
}

// fmx_math.h -- small fp32 math kernels shared by the HIP kernels and the
// host-side accuracy test (tests/cpp/math_test.cpp).
//
// fmx_sincos: sin and cos of one fp32 phase, |x| <= 8 (the NCO phases of the
// stereo PLL, stereo_decoder.cpp:251-253 / 277-278, and the RDS mix-down,
// subcarrier.cpp:158, are wrapped to [-pi, 2pi]).  Three-part Cody-Waite
// reduction by pi/2 with FMA (exact for |q| <= 5) and the cephes sinf/cosf
// minimax polynomials on [-pi/4, pi/4] with the reduced argument carried as
// a float pair: one shared reduction and ~30 VALU
// instead of the libm sincosf path with its large-argument branch.  Max error
// against the correctly rounded result is checked by tests/test_math.py:
// < 1 ulp, ~95 % correctly rounded over [-2pi, 2pi] (the oracle's glibc
// sinf/cosf are the reference; parity bars on the PLL outputs are tolerances).
#ifndef FMX_MATH_H
#define FMX_MATH_H

#include <stdint.h>

#ifdef __HIPCC__
#define FMX_HD __host__ __device__ __forceinline__
#else
#include <cmath>
#define FMX_HD inline
#endif

// The quadrant-swapped polynomials of fmx_sincos_q before their signs:
// sin x = (qi & 2) ? -*s0 : *s0, cos x = ((qi + 1) & 2) ? -*c0 : *c0.  A
// recursion that multiplies by sin x can flip its other factor's sign bit
// off the dependency chain instead (the k_pll feedback loop).
FMX_HD void fmx_sincos_q_abs(float x, float q, int qi, float *s0, float *c0) {
  // r = x - q pi/2 as rh + rl (pi/2 in three parts)
  const float r1 = fmaf(-q, 1.57079637050628662109375f, x);
  const float rh = fmaf(-q, -4.3711388286737929e-08f, r1);
  float rl = fmaf(-q, -4.3711388286737929e-08f, r1 - rh);
  rl = fmaf(-q, -1.7151245100058819e-15f, rl);
  const float z = rh * rh;
  // sin: rh + (rl + rh z P(z)),  degree-9 minimax
  float ps = fmaf(z, 2.6083159809786593541503e-06f, -0.0001981069071916863322258f);
  ps = fmaf(z, ps, 0.00833307858556509017944336f);
  ps = fmaf(z, ps, -0.166666597127914428710938f);
  const float sr = rh + fmaf(rh * z, ps, rl);
  // cos: (1 - z/2) split exactly, + z^2 Q(z) - rh rl
  float pc = fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f);
  pc = fmaf(z, pc, 4.166664568298827e-2f);
  const float hz = 0.5f * z;
  const float w = 1.0f - hz;
  const float tail = (1.0f - w) - hz;
  const float cr = w + (fmaf(z * z, pc, tail) - rh * rl);
  const bool swap = (qi & 1) != 0;
  *s0 = swap ? cr : sr;
  *c0 = swap ? sr : cr;
}

// sin and cos of x given its quadrant count qi (x ~ qi pi/2, |x - qi pi/2|
// <= pi/4 + a few ulp); q = (float)qi.
FMX_HD void fmx_sincos_q(float x, float q, int qi, float *s, float *c) {
  float s0, c0;
  fmx_sincos_q_abs(x, q, qi, &s0, &c0);
  *s = (qi & 2) ? -s0 : s0;
  *c = ((qi + 1) & 2) ? -c0 : c0;
}

FMX_HD void fmx_sincos(float x, float *s, float *c) {
  const float q = rintf(x * 0.636619772367581343f);
  fmx_sincos_q(x, q, (int)q, s, c);
}

// x / c for a constant c with rc = RN(1/c): q = x rc, then one Markstein
// correction with the exact FMA residual -- 3 dependent ops instead of the
// IEEE divide sequence.  Not correctly rounded for every divisor: it is used
// only for the divisors tests/cpp/divconst_test.cpp checks against IEEE x / c
// over every finite float numerator (tests/test_math.py).
FMX_HD float fmx_div_const(float x, float c, float rc) {
  const float q = x * rc;
  const float r = fmaf(-q, c, x);
  return fmaf(r, rc, q);
}

// liquid's NCO constrain (nco.proto.c, as the oracle's lq::nco_constrain):
//   p = (float)((double)x / 2pi);  f = p - truncf(p);  f < 0: f = (float)((double)f + 1);
//   s = f * 2^32;  s >= 2^32 ? 0 : (uint32)s
// restated with one floor: f = p - floorf(p) is the exact value of the
// reference's fpart (+1 when negative) rounded once to float, which equals the
// double add rounded to float (that add is exact unless |fpart| < 2^-29, where
// both round to 1.0).  f == 1.0 is the only s >= 2^32 case and its compare is
// off the dependency chain; the device's v_cvt_u32_f32 maps NaN to 0 as the
// reference's conversion does on the GPU.  Checked bit for bit against the
// reference form over all 2^32 inputs (tests/cpp/ncoconstrain_test.cpp).
FMX_HD uint32_t fmx_cvt_u32(float s) {
#ifdef __HIP_DEVICE_COMPILE__
  return (uint32_t)s;
#else
  return (s != s || s <= 0.0f) ? 0u : (s >= 4294967296.0f ? 0xFFFFFFFFu : (uint32_t)s);
#endif
}
FMX_HD uint32_t fmx_nco_constrain(float x) {
  const float p = (float)((double)x * 0.159154943091895);
  const float f = p - floorf(p);
  const uint32_t u = fmx_cvt_u32(f * 4294967296.0f);
  return (f == 1.0f) ? 0u : u;
}
// liquid's NCO phase of a word as the reference computes it,
// (float)(2 pi (double)(float)theta / 2^32), in float arithmetic: the product
// of (float)theta and the double constant K = 2 pi / 2^32 as Kh + Kl with the
// exact FMA residual, rounded once.  Bit-identical to the double form for all
// 2^32 words (tests/cpp/ncoconstrain_test.cpp); 5 full-rate VALU instead of
// two double conversions and a double multiply.
FMX_HD float fmx_nco_phase(uint32_t theta) {
  const float t = (float)theta;
  const float ph = t * 0x1.921fb6p-30f;
  const float e = fmaf(t, 0x1.921fb6p-30f, -ph);
  return ph + fmaf(t, -0x1.777a5cp-55f, e);
}
FMX_HD float fmx_nco_phase_ref(uint32_t theta) {
  return (float)((double)(float)theta * (6.283185307179586 / 4294967296.0));
}
// the reference form, for the host check
FMX_HD uint32_t fmx_nco_constrain_ref(float x) {
  const float p = (float)((double)x * 0.159154943091895);
  float fpart = p - truncf(p);
  if (fpart < 0.0f) fpart = (float)((double)fpart + 1.0);
  const float s = fpart * 4294967296.0f;
  return (s >= 4294967296.0f) ? 0u : fmx_cvt_u32(s);
}

// Quadrant count of an NCO phase word: round(theta / 2^30) in 0..4, the
// quadrant of the exact phase 2 pi theta / 2^32.  The float phase the
// reference computes from theta is within 0.5 ulp of it, so fmx_sincos_q of
// that phase with this count stays inside the polynomial range; it is known
// as soon as theta is, off the phase's dependency chain (the k_pll loop).
FMX_HD int fmx_nco_quadrant(uint32_t theta) { return (int)((theta >> 30) + ((theta >> 29) & 1u)); }

// sin(2 pi theta / 2^32) for the stereo PLL's feedback chain only (k_pll
// W0, stereo_decoder.cpp:251-256): half-turn reduction on the phase word,
// theta = m 2^31 + d (|d| <= 2^30, m's parity returned in bit 31 of *sg),
// r = d pi / 2^31 (one rounding), and the degree-9 minimax sine on
// [-pi/2, pi/2]; sin = (*sg ? -1 : 1) * the return value.  11 VALU instead
// of the float phase (an f64 multiply) and both quadrant polynomials.  Its
// error against sin of the reference's float phase is measured over all 2^32
// words by tests/cpp/pllsin_test.cpp (tests/golden/pllsin_exhaustive.json).
FMX_HD float pll_sin_word(uint32_t theta, uint32_t *sg) {
  const uint32_t s = (theta + 0x40000000u) & 0x80000000u;
  const float r = (float)(int32_t)(theta ^ s) * 1.4629180792671596e-09f;
  const float z = r * r;
  float u = fmaf(z, 2.6083159809786593541503e-06f, -0.0001981069071916863322258f);
  u = fmaf(u, z, 0.00833307858556509017944336f);
  u = fmaf(u, z, -0.166666597127914428710938f);
  *sg = s;
  return fmaf(z, u * r, r);
}

// RF-level clip pre-test on one 4-byte word of u8 I/Q (signal_level.cpp:
// computeSignalLevel counts samples with a component <= 8 or >= 247): nonzero
// iff some byte b has (b + 9) mod 256 < 18, i.e. b <= 8 or b >= 247.  Bytewise
// add without inter-byte carries, then the classic "some byte < n" test.
// Exact over all 2^32 words (tests/cpp/swar_test.c checks it exhaustively).
FMX_HD uint32_t fmx_word_near_clip(uint32_t w) {
  const uint32_t t = ((w & 0x7F7F7F7Fu) + 0x09090909u) ^ (w & 0x80808080u);
  return (t - 0x12121212u) & ~t & 0x80808080u;
}


// atan2 for the FM discriminator, branch- and compare-free: octant
// reduction a = min/max of |x|, |y| (reciprocal + one Newton step),
// atan(a) = a + a s P(s), s = a^2, with the degree-7 minimax P of the device
// libm (ocml atan), then the octant fix-ups through sign factors
// (copysign) instead of compares and selects.  Within 2 ulp of the exact
// atan2 and 2.5e-7 of atan2f (tests/test_math.py); atan2(+-0, +0) = +-0,
// atan2(+-0, -0) = +-pi as IEEE.
//
// Why no selects: with two k_fe8 workgroups per CU, the libm atan2f (and a
// select-based version) in the discriminator returned wrong values in lanes
// 48-63 of some wave-instructions, nondeterministically (tools/
// gpu_determinism.py: thousands of MPX samples per 4096-channel run, always
// whole 16-lane groups, never with one workgroup per CU or with a
// select-free discriminator).
FMX_HD float fmx_atan2f(float y, float x) {
  const float ax = fabsf(x), ay = fabsf(y);
  const float mx = fmaxf(fmaxf(ax, ay), 1e-37f), mn = fminf(ax, ay);
#ifdef __HIP_DEVICE_COMPILE__
  const float rc = __builtin_amdgcn_rcpf(mx);
#else
  const float rc = 1.0f / mx;
#endif
  float a = mn * rc;
  a = fmaf(fmaf(-mx, a, mn), rc, a); // one Newton step: ~0.5 ulp
  const float s = a * a;
  float p = fmaf(s, 0.002642294391989708f, -0.015280019491910934f);
  p = fmaf(s, p, 0.04149937257170677f);
  p = fmaf(s, p, -0.07413642853498459f);
  p = fmaf(s, p, 0.10605181753635406f);
  p = fmaf(s, p, -0.14197120070457458f);
  p = fmaf(s, p, 0.19992350041866302f);
  p = fmaf(s, p, -0.3333311676979065f);
  const float r = fmaf(a, s * p, a);
  // |y| > |x|: pi/2 - r;  x < 0 (or -0): pi - r1
  const float sw = copysignf(1.0f, ax - ay);           // -1 when |y| > |x|
  const float r1 = fmaf(sw, r, (1.0f - sw) * 0.78539818525314331f);
  const float sx = copysignf(1.0f, x);
  const float r2 = fmaf(sx, r1, (1.0f - sx) * 1.5707963705062866f);
  return copysignf(r2, y);
}

#endif

// fmx_math.h -- small fp32 / integer math shared by the HIP kernels and the
// host-side accuracy tests (tests/cpp/*_test.cpp, tests/hip/pllmath_sweep.hip).
// Every helper here is called by a product kernel; each has an exhaustive or
// swept check against the reference's own arithmetic (tests/test_math.py,
// tests/test_gpu_pllmath.py).
#ifndef FMX_MATH_H
#define FMX_MATH_H

#include <stdint.h>

#ifdef __HIPCC__
#define FMX_HD __host__ __device__ __forceinline__
#else
#include <cmath>
#define FMX_HD inline
#endif

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

#ifdef __HIPCC__
// The stereo PLL's feedback chain (k_pll W0, stereo_decoder.cpp:178-192), one
// sample: vcoQ = sin(phase) of the NCO word theta, then liquid's pll_step
// (dtheta += constrain(e alpha), theta += constrain(e beta)) and step (theta
// += dtheta), e = pilot vcoQ.  These two functions ARE the chain's
// arithmetic: k_pll calls them, and the GPU test kernel
// (tests/hip/pllmath_sweep.hip) sweeps them against the reference's float
// phase / double-precision constrain (tests/test_gpu_pllmath.py,
// tests/golden/pllmath_gpu.json).
//
// fmx_chain_sin: v_sin_f32 takes turns; the word's top 23 bits become the
// mantissa of a float in [1, 2) with one v_alignbit_b32 ({0x7F, theta} >> 9 =
// 0x3F800000 | theta >> 9), so sin(2 pi (1 + theta / 2^32)) = sin(2 pi theta /
// 2^32) up to the truncated 9 bits (< 2^-23 turn) and v_sin's own error.  One
// VALU op instead of a convert and a multiply on the serial chain.
__device__ __forceinline__ float fmx_chain_sin(uint32_t theta) {
  return __builtin_amdgcn_sinf(__builtin_bit_cast(float, __builtin_amdgcn_alignbit(0x7Fu, theta, 9u)));
}
// fmx_word_sincos: sine and cosine of an NCO word (phase 2 pi theta / 2^32)
// by v_sin / v_cos, which take turns: the word as a signed fraction of a
// turn in [-0.5, 0.5) (rounded to 24 bits: < 2^-25 turn).  k_pll's outputs
// (vcoI / vcoQ of the pilot I/Q, cos 2 phase of the L-R mix,
// stereo_decoder.cpp:178-180,194-195,218-220), swept with the chain.
__device__ __forceinline__ void fmx_word_sincos(uint32_t theta, float *s, float *c) {
  const float r = (float)(int32_t)theta * 2.3283064365386963e-10f;
  *s = __builtin_amdgcn_sinf(r);
  *c = __builtin_amdgcn_cosf(r);
}
// fmx_chain_words: the two constrain words of pll_step from the pilot's
// pre-products pa = pilot alpha/2pi 2^32, pb = pilot beta/2pi 2^32 (one packed
// multiply by vcoQ, then truncating converts): for |e k| < 1/2 the word
// constrain(e k) = frac(e k / 2 pi) 2^32 equals (uint32)(int32)(e k / 2 pi 2^32)
// up to the float roundings, which the sweep bounds.
__device__ __forceinline__ void fmx_chain_words(float pa, float pb, float vcoQ, uint32_t *ca, uint32_t *cb) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 x = f2{pa, pb} * f2{vcoQ, vcoQ};
  *ca = (uint32_t)(int32_t)x.x;
  *cb = (uint32_t)(int32_t)x.y;
}
#endif

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

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

// Forms of the stereo PLL's sine / constrain arithmetic (k_pll), chosen at
// compile time; the shipped library is built with the defaults and
// tests/hip/libpllmath.so sweeps whatever forms it is built with.  Round 6
// A/B (profiles/r06a_*): see DESIGN.md section 3.
//   FMX_PLL_CHAIN  W0's feedback sine of the word:
//     0  round 5: the word's top 23 bits truncated (v_alignbit_b32 into a
//        float in [1, 2)), one op; a phase bias of up to -2^-23 turn
//     1  the same with the word carried +256 by W0 (FMX_CHAIN_TOFF): the top
//        23 bits rounded to nearest, still one op
//     2  round 4: (float)(int32)theta 2^-32, a signed 24-bit turn (two ops)
//     3  (float)(uint32)theta 2^-32: the reference's own rounding of the word
//        ((float)theta in nco_crcf_get_phase, as oracle Nco::get_phase) (two ops)
//   FMX_WORD_SINCOS  the P waves' sine / cosine of the word (vcoI / vcoQ,
//     cos 2 phase): 0 signed 24-bit turn, 1 (float)(uint32)theta as the reference
//   FMX_PLL_WORDS  pll_step's constrain words: 0 truncating converts (e < 0:
//     within 130 / 144 words of the reference's 256-word steps); 1 e < 0
//     rounded to the reference's 256-word grid by one f32 add of 2^32
//     (saturating converts, no compare; e >= 0 one word low); 3 the alpha
//     (frequency) word as 1, the beta (phase) word as 0
// Shipped (round 6): FMX_PLL_CHAIN 1 (free: removes the -3.7e-7 rad phase
// bias of the truncated sine) and FMX_PLL_WORDS 3 (the frequency word as the
// reference rounds it: worst PCM RMS against the oracle 3.6e-6 -> 1.4e-6,
// median 9.3e-7 -> 4.3e-7, for +1.1 % / +1.5 % step time at 4096 / 2048
// channels; profiles/r06c_*, r06d_*).  The sine forms alone move no PCM error.
#ifndef FMX_PLL_CHAIN
#define FMX_PLL_CHAIN 1
#endif
#ifndef FMX_WORD_SINCOS
#define FMX_WORD_SINCOS 0
#endif
#ifndef FMX_PLL_WORDS
#define FMX_PLL_WORDS 3
#endif
#if FMX_PLL_CHAIN == 1
#define FMX_CHAIN_TOFF 256u
#else
#define FMX_CHAIN_TOFF 0u
#endif

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
// fmx_chain_sin(theta + FMX_CHAIN_TOFF) = sin(2 pi theta / 2^32): v_sin_f32
// takes turns.  Forms 0 / 1: the word's top 23 bits become the mantissa of a
// float in [1, 2) with one v_alignbit_b32 ({0x7F, w} >> 9 = 0x3F800000 | w >>
// 9), so sin(2 pi (1 + w / 2^32)) = sin(2 pi w / 2^32) up to the dropped 9
// bits and v_sin's own error -- truncated (form 0), or rounded when the word
// is carried + 256 (form 1).  Forms 2 / 3 convert and scale.
__device__ __forceinline__ float fmx_chain_sin(uint32_t w) {
#if FMX_PLL_CHAIN == 2
  return __builtin_amdgcn_sinf((float)(int32_t)w * 2.3283064365386963e-10f);
#elif FMX_PLL_CHAIN == 3
  return __builtin_amdgcn_sinf((float)w * 2.3283064365386963e-10f);
#else
  return __builtin_amdgcn_sinf(__builtin_bit_cast(float, __builtin_amdgcn_alignbit(0x7Fu, w, 9u)));
#endif
}
// fmx_word_sincos: sine and cosine of an NCO word (phase 2 pi theta / 2^32)
// by v_sin / v_cos, which take turns: form 0 the word as a signed fraction of
// a turn in [-0.5, 0.5) (rounded to 24 bits: < 2^-25 turn), form 1 as
// (float)theta 2^-32 in [0, 1], the reference's rounding of the word.
// k_pll's outputs (vcoI / vcoQ of the pilot I/Q, cos 2 phase of the L-R mix,
// stereo_decoder.cpp:178-180,194-195,218-220), swept with the chain.
__device__ __forceinline__ void fmx_word_sincos(uint32_t theta, float *s, float *c) {
#if FMX_WORD_SINCOS == 1
  const float r = (float)theta * 2.3283064365386963e-10f;
#else
  const float r = (float)(int32_t)theta * 2.3283064365386963e-10f;
#endif
  *s = __builtin_amdgcn_sinf(r);
  *c = __builtin_amdgcn_cosf(r);
}
// v_cvt_u32_f32 with its hardware saturation (negative / NaN -> 0, >= 2^32 ->
// 0xFFFFFFFF), which a C++ conversion of an out-of-range float does not promise
__device__ __forceinline__ uint32_t fmx_cvt_u32_sat(float x) {
  uint32_t r;
  asm("v_cvt_u32_f32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}
// fmx_chain_words: the two constrain words of pll_step from the pilot's
// pre-products pa = pilot alpha/2pi 2^32, pb = pilot beta/2pi 2^32 (one packed
// multiply by vcoQ).  Form 0, truncating converts: for |e k| < 1/2 the word
// constrain(e k) = frac(e k / 2 pi) 2^32 equals (uint32)(int32)(e k / 2 pi 2^32)
// up to the float roundings (and, for e < 0, the reference's rounding of
// 1 + frac to 24 bits), which the sweep bounds.  Form 1: x = e k / 2 pi 2^32
// as two saturating converts, cvt(x) + cvt(x + 2^32): for x < 0 the first is
// 0 and the second the f32 sum 2^32 + x rounded to the 256-word grid, which
// is the reference's (float)(fpart + 1) 2^32; for x >= 0 the second
// saturates to 2^32 - 1, so the word is trunc(x) - 1.
// (form 3: the alpha word as form 1, the beta word as form 0)
__device__ __forceinline__ void fmx_chain_words(float pa, float pb, float vcoQ, uint32_t *ca, uint32_t *cb) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 x = f2{pa, pb} * f2{vcoQ, vcoQ};
#if FMX_PLL_WORDS == 1
  const f2 y = x + f2{4294967296.0f, 4294967296.0f};
  *ca = fmx_cvt_u32_sat(x.x) + fmx_cvt_u32_sat(y.x);
  *cb = fmx_cvt_u32_sat(x.y) + fmx_cvt_u32_sat(y.y);
#elif FMX_PLL_WORDS == 3
  *ca = fmx_cvt_u32_sat(x.x) + fmx_cvt_u32_sat(x.x + 4294967296.0f);
  *cb = (uint32_t)(int32_t)x.y;
#else
  *ca = (uint32_t)(int32_t)x.x;
  *cb = (uint32_t)(int32_t)x.y;
#endif
}
// fmx_chain_step: one sample's pll_step + step on the carried words, with
// the words of fmx_chain_words: dtheta += ca; theta += dtheta(new) + cb --
// the reference's order (pll_step adds ca to dtheta and cb to theta, step
// then adds the updated dtheta), so that theta's update is one v_add3_u32 of
// the updated dtheta and no theta + dtheta is formed.  Form 1 / 3 sum the
// saturating converts straight into dtheta with v_add3_u32.
__device__ __forceinline__ void fmx_chain_step(float pa, float pb, float vcoQ, uint32_t &theta, uint32_t &dtheta) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 x = f2{pa, pb} * f2{vcoQ, vcoQ};
  uint32_t tn;
#if FMX_PLL_WORDS == 1
  const f2 y = x + f2{4294967296.0f, 4294967296.0f};
  const uint32_t a0 = fmx_cvt_u32_sat(x.x), a1 = fmx_cvt_u32_sat(y.x);
  const uint32_t b0 = fmx_cvt_u32_sat(x.y), b1 = fmx_cvt_u32_sat(y.y);
  asm("v_add3_u32 %0, %1, %2, %3" : "=v"(dtheta) : "v"(dtheta), "v"(a0), "v"(a1));
  uint32_t s;
  asm("v_add3_u32 %0, %1, %2, %3" : "=v"(s) : "v"(theta), "v"(dtheta), "v"(b0));
  tn = s + b1;
#elif FMX_PLL_WORDS == 3
  const uint32_t a0 = fmx_cvt_u32_sat(x.x), a1 = fmx_cvt_u32_sat(x.x + 4294967296.0f);
  const uint32_t cb = (uint32_t)(int32_t)x.y;
  asm("v_add3_u32 %0, %1, %2, %3" : "=v"(dtheta) : "v"(dtheta), "v"(a0), "v"(a1));
  asm("v_add3_u32 %0, %1, %2, %3" : "=v"(tn) : "v"(theta), "v"(dtheta), "v"(cb));
#else
  const uint32_t ca = (uint32_t)(int32_t)x.x, cb = (uint32_t)(int32_t)x.y;
  dtheta += ca;
  asm("v_add3_u32 %0, %1, %2, %3" : "=v"(tn) : "v"(theta), "v"(dtheta), "v"(cb));
#endif
  theta = tn;
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

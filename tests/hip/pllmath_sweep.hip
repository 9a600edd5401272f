// pllmath_sweep.hip -- TEST CODE, not product: the shipped stereo-PLL chain
// arithmetic of k_pll (fmx_chain_sin, fmx_chain_words, fmx_word_sincos in
// fmtuner-sdr_amd/csrc/fmx_math.h -- the functions k_pll itself calls) swept
// on the GPU against what the reference computes (stereo_decoder.cpp:178-192
// through liquid's nco_crcf, as the oracle restates it: oracle/fmx_oracle.cpp
// lq::Nco):
//
//   sine   every 2^32 NCO word theta: fmx_chain_sin(theta) (W0's feedback
//          sine) and fmx_word_sincos(theta) (the P waves' vcoI / vcoQ / cos
//          2 phase) against sin / cos of the reference's float phase
//          (float)(2 pi (float)theta / 2^32) in double precision, and against
//          the exact phase 2 pi theta / 2^32;
//   words  every float pilot with 2^-30 <= |pilot| < 2 (the MPX, hence the
//          pilot BPF output, stays within +-1.71 at 256 kHz) times a set of
//          vcoQ values, both signs: the chain's two pll_step words
//          (uint32)(int32)(pilot k 2^32 vcoQ) against liquid's constrain
//          frac((double)(e alpha) / 2 pi) 2^32 with e = pilot vcoQ rounded
//          to float, as the reference (fmx_nco_constrain_ref).
//
// Built by tests/hip/Makefile (__graft_entry__.build()) into libpllmath.so;
// tests/test_gpu_pllmath.py calls pllmath_sweep() and compares with
// tests/golden/pllmath_gpu.json.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstring>

#include "../../fmtuner-sdr_amd/csrc/fmx_math.h"

namespace {

constexpr int kNS = 8;   // sine maxima
constexpr int kNW = 8;   // word maxima
constexpr double kTwoPi = 6.283185307179586476925286766559;

__device__ void wave_max(float v, unsigned *dst) {
  for (int d = 32; d >= 1; d >>= 1) v = fmaxf(v, __shfl_xor(v, d));
  if ((threadIdx.x & 63) == 0) atomicMax(dst, __float_as_uint(v)); // non-negative floats order as integers
}
__device__ void wave_sum(double v, double *dst) {
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
  if ((threadIdx.x & 63) == 0) atomicAdd(dst, v);
}

// mx[0] chain sin vs the reference float phase, [1] vs the exact phase,
// [2] / [3] word sin / cos vs the reference float phase, [4] / [5] vs exact;
// sums[0] signed chain-sine error vs exact (its bias), sums[1] |error|,
// sums[2] the error times cos of the exact phase: over all words, sum / 2^31
// is the chain sine's mean PHASE error in radians (a truncated word lags by
// half its dropped bits; the PLL locks to that lag)
__global__ void k_sine(uint64_t w0, uint64_t count, unsigned *mx, double *sums) {
  float m[6] = {0, 0, 0, 0, 0, 0};
  double bias = 0.0, mag = 0.0, pbias = 0.0;
  const uint64_t gsz = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += gsz) {
    const uint32_t th = (uint32_t)(w0 + i);
    const float cs = fmx_chain_sin(th + FMX_CHAIN_TOFF); // the word as W0 carries it
    float ws, wc;
    fmx_word_sincos(th, &ws, &wc);
    const double ph = (double)fmx_nco_phase_ref(th);
    const double rs = sin(ph), rc = cos(ph);
    const double ex = (double)th * (kTwoPi / 4294967296.0);
    const double es = sin(ex), ec = cos(ex);
    m[0] = fmaxf(m[0], (float)fabs((double)cs - rs));
    m[1] = fmaxf(m[1], (float)fabs((double)cs - es));
    m[2] = fmaxf(m[2], (float)fabs((double)ws - rs));
    m[3] = fmaxf(m[3], (float)fabs((double)wc - rc));
    m[4] = fmaxf(m[4], (float)fabs((double)ws - es));
    m[5] = fmaxf(m[5], (float)fabs((double)wc - ec));
    bias += (double)cs - es;
    mag += fabs((double)cs - es);
    pbias += ((double)cs - es) * ec;
  }
  for (int k = 0; k < 6; ++k) wave_max(m[k], mx + k);
  wave_sum(bias, sums);
  wave_sum(mag, sums + 1);
  wave_sum(pbias, sums + 2);
}

// every positive float bit pattern in [b0, b0 + nb) as the pilot, both signs,
// times vq[0 .. nvq): word differences (int32) of ca / cb against the
// reference; mx[0] / [1] |d ca| / |d cb| for e >= 0, [2] / [3] for e < 0,
// [4] / [5] |d| relative to max(|ref word|, 2^10); sums[0] / [1] the sums of
// |d ca| / |d cb| over the e < 0 pairs (their mean: the typical word error,
// where the maxima show only the worst case)
__global__ void k_words(uint32_t b0, uint32_t nb, const float *vq, int nvq, float alpha, float beta, unsigned *mx,
                        double *sums) {
  double sa = 0.0, sb = 0.0;
  const float ka = alpha * 0.159154943091895f, kb = beta * 0.159154943091895f; // as k_pll W0
  const float kaw = ka * 4294967296.0f, kbw = kb * 4294967296.0f;
  float m[6] = {0, 0, 0, 0, 0, 0};
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += gridDim.x * blockDim.x) {
    const float p0 = __uint_as_float(b0 + i);
    for (int sgn = 0; sgn < 2; ++sgn) {
      const float p = sgn ? -p0 : p0;
      const float pa = p * kaw, pb = p * kbw;
      for (int j = 0; j < nvq; ++j) {
        const float v = vq[j];
        uint32_t ca, cb;
        fmx_chain_words(pa, pb, v, &ca, &cb);
        const float e = p * v;
        const uint32_t ra = fmx_nco_constrain_ref(e * alpha), rb = fmx_nco_constrain_ref(e * beta);
        const float da = fabsf((float)(int32_t)(ca - ra)), db = fabsf((float)(int32_t)(cb - rb));
        const int o = (e < 0.0f) ? 2 : 0;
        m[o] = fmaxf(m[o], da);
        m[o + 1] = fmaxf(m[o + 1], db);
        if (e < 0.0f) {
          sa += (double)da;
          sb += (double)db;
        }
        m[4] = fmaxf(m[4], da / fmaxf(fabsf((float)(int32_t)ra), 1024.0f));
        m[5] = fmaxf(m[5], db / fmaxf(fabsf((float)(int32_t)rb), 1024.0f));
      }
    }
  }
  for (int k = 0; k < 6; ++k) wave_max(m[k], mx + k);
  wave_sum(sa, sums);
  wave_sum(sb, sums + 1);
}

} // namespace

extern "C" {

// out[0..5]: sine maxima (see k_sine), out[6]: mean signed chain-sine error,
// out[7]: mean |chain-sine error|, out[8]: words swept; out[9..14]: word
// maxima (see k_words), out[15]: (pilot, vcoQ) pairs checked, out[16]: the
// chain sine's mean phase error (radians, see k_sine), out[17..19]: the forms
// built (FMX_PLL_CHAIN, FMX_WORD_SINCOS, FMX_PLL_WORDS), out[20..21]: the
// mean |d ca| / |d cb| over the e < 0 pairs.  Returns 0, or a negative HIP
// error.
int pllmath_sweep(float alpha, float beta, double *out, int nout) {
  if (nout < 22) return -100;
  unsigned *d_mx = nullptr;
  double *d_sum = nullptr;
  float *d_vq = nullptr;
  // vcoQ values: the extremes, a few interior values, and small ones
  const float vq[] = {1.0f, -1.0f, 0.70710677f, -0.5f, 0.3f, 0.123456f, -0.01f, 1e-3f};
  const int nvq = (int)(sizeof(vq) / sizeof(vq[0]));
  hipError_t e;
  if ((e = hipMalloc(&d_mx, sizeof(unsigned) * (kNS + kNW))) != hipSuccess) return -(int)e;
  if ((e = hipMalloc(&d_sum, sizeof(double) * 5)) != hipSuccess) return -(int)e;
  if ((e = hipMalloc(&d_vq, sizeof(vq))) != hipSuccess) return -(int)e;
  hipMemset(d_mx, 0, sizeof(unsigned) * (kNS + kNW));
  hipMemset(d_sum, 0, sizeof(double) * 5);
  hipMemcpy(d_vq, vq, sizeof(vq), hipMemcpyHostToDevice);
  const uint64_t words = 1ull << 32;
  hipLaunchKernelGGL(k_sine, dim3(8192), dim3(256), 0, 0, (uint64_t)0, words, d_mx, d_sum);
  // |pilot| in [2^-30, 2): exponent fields 97 .. 127
  const uint32_t b0 = 97u << 23, nb = 31u << 23;
  hipLaunchKernelGGL(k_words, dim3(8192), dim3(256), 0, 0, b0, nb, d_vq, nvq, alpha, beta, d_mx + kNS, d_sum + 3);
  if ((e = hipDeviceSynchronize()) != hipSuccess) return -(int)e;
  unsigned mx[kNS + kNW];
  double sums[5];
  hipMemcpy(mx, d_mx, sizeof(mx), hipMemcpyDeviceToHost);
  hipMemcpy(sums, d_sum, sizeof(sums), hipMemcpyDeviceToHost);
  hipFree(d_mx);
  hipFree(d_sum);
  hipFree(d_vq);
  auto f = [&](int i) { float v; std::memcpy(&v, &mx[i], 4); return (double)v; };
  for (int k = 0; k < 6; ++k) out[k] = f(k);
  out[6] = sums[0] / (double)words;
  out[7] = sums[1] / (double)words;
  out[8] = (double)words;
  for (int k = 0; k < 6; ++k) out[9 + k] = f(kNS + k);
  out[15] = (double)nb * 2.0 * nvq;
  out[16] = sums[2] / 2147483648.0;
  out[17] = FMX_PLL_CHAIN;
  out[18] = FMX_WORD_SINCOS;
  out[19] = FMX_PLL_WORDS;
  out[20] = sums[3] / ((double)nb * nvq); // e < 0: half of the 2 nb nvq pairs
  out[21] = sums[4] / ((double)nb * nvq);
  return 0;
}

} // extern "C"

// fmx_kernels.hip -- CDNA4 (gfx950) kernels of the many-channel FM demodulator.
//
// Four hot kernels per reference block:
//
//  k_frontend  one workgroup per channel, 256 threads, the block processed in
//              chunks of 768 DSP samples; every stage is sample-parallel:
//                u8 IQ -> ComplexDecimator (M x 28-tap polyphase FIR, IQ staged
//                in LDS as fp16 pairs in phase-major layout)       liquid_primitives.cpp:461-499
//                -> DC blockers (affine scan over the chunk)        fm_demod.cpp:186-188
//                -> IQ FIR 81/121 taps                              fm_demod.cpp:190-191
//                -> [AGC, serial]  -> discriminator (atan2)         fm_demod.cpp:192-195
//                -> 19 kHz pilot band-pass (305 taps)               stereo_decoder.cpp:229-230
//                -> 240k->171k RDS resampler (host timing schedule) subcarrier.cpp:117-147
//  k_pll       one lane per channel (64 channels per wave): the nonlinear
//              per-sample recurrences of StereoDecoder::processAudio
//              (PLL, envelopes, blend) and the L-R matrix              stereo_decoder.cpp:226-288
//  k_audio     one workgroup per channel: L/R 121-tap FIRs, 32 kHz
//              resampler, de-emphasis + DC block, clamp               af_post_processor.cpp:47-78
//  k_rds       one lane per channel: 57 kHz mix-down, 255-tap FIR as 11
//              streaming partial sums, AGC, symbol sync, PSK2 Costas loop,
//              biphase/delta decoding and redsea block sync            subcarrier.cpp:153-235,
//                                                                      block_sync.cpp:254-313
//
// Build with -ffp-contract=off: wherever the reference's arithmetic order is
// reproduced (IIRs, PLL, resamplers, RDS FIR) products and sums must round
// separately.  The large FIRs use explicit fmaf.
#include <hip/hip_ext.h>
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cstddef>
#include <type_traits>

#include "fmx_internal.h"
#include "fmx_math.h"
#include "fmx_synth.h"

// k_rds's FIR partial sums: one packed FMA per product instead of the
// reference's separate multiply and add (its dotprod order, rounded twice).
// The RDS path is held to bit-exact groups, not to bit-exact floats (its
// mix-down sine is the hardware one).

namespace fmx {

#define FE_T 768       // DSP samples per frontend chunk (256 threads x 3)
#define FE_HALO_IQ 120 // >= longest IQ FIR - 1
#define AU_T 768
#define AU_HALO 120
#define AU_RHALO 32
#define AU_MAXOUT 256

static constexpr float kPiF = 3.14159265358979323846f;

/* ------------------------------------------------------------------ */
// Wave-uniform reads of the design tables (taps) through the scalar cache:
// the constant address space makes the backend emit s_load instead of a
// per-lane global_load + wait in every FIR iteration.  Only for addresses
// that are uniform across the wave.
#define FMX_CONST __attribute__((address_space(4)))
template <typename T> __device__ __forceinline__ const FMX_CONST T *cptr(const T *p) {
  return (const FMX_CONST T *)p;
}

/* ------------------------------------------------------------------ */
// Buffer resource over [base, base + bytes): out-of-range loads return 0.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)bytes, 0x00020000);
}

/* ------------------------------------------------------------------ */
/* liquid NCO fixed-point helpers (nco.proto.c restated)               */
// fmx_nco_constrain (fmx_math.h): one floor instead of trunc / compare / add,
// bit-identical to the reference form for every float (exhaustive host check)
__device__ __forceinline__ uint32_t d_nco_constrain(float x) { return fmx_nco_constrain(x); }
// (2pi * theta) / 2^32 as the reference rounds it, in float (fmx_math.h)
__device__ __forceinline__ float d_nco_phase(uint32_t theta) { return fmx_nco_phase(theta); }
// x / c by fmx_div_const (fmx_math.h), for the divisors whose exactness
// against IEEE x / c tests/cpp/divconst_test.cpp checks exhaustively
__device__ __forceinline__ float d_div_const(float x, float c, float rc) { return fmx_div_const(x, c, rc); }
// unwrapf (liquid_wrappers.cpp / stereo_decoder.cpp): one 2pi step into
// [-pi, pi], as selects (no divergent branches in the sample loops)
__device__ __forceinline__ float d_unwrap(float x) {
  const float dn = x - 2.0f * kPiF, up = x + 2.0f * kPiF;
  return (x > kPiF) ? dn : ((x < -kPiF) ? up : x);
}
__device__ __forceinline__ float d_clamp(float v, float lo, float hi) {
  return (v < lo) ? lo : ((hi < v) ? hi : v);
}

/* ------------------------------------------------------------------ */
// Raw L/R between k_pll and k_audio in pair tiles: sample t of channel c at
// ((c / 2) * (stride / 16) + t / 16) * 32 + (c % 2) * 16 + t % 16, i.e. one
// 128-B line holds 16 consecutive samples of 2 consecutive channels.  A
// k_pll P wave holds 4 channel rows x 16 samples, so each of its store
// instructions writes 2 whole lines; k_audio's loads read 64-B pieces
// (round 2-3: octet tiles of 4 samples x 8 channels for the one-lane-per-
// channel W3; with one row per channel every store instruction wrote a 16-B
// piece of 64 lines and HBM saw ~1.8x the bytes); stride % 16 == 0.
__device__ __forceinline__ size_t lr_tile_idx(int c, int t, int stride) {
  return ((size_t)(c >> 1) * (size_t)(stride >> 4) + (size_t)(t >> 4)) * 32 + (size_t)((c & 1) * 16 + (t & 15));
}
// k_audio's block -> channel order for tiled input: blocks b and b + 8 share
// an XCD (observed round-robin dispatch, MI355X_MICROARCH.md "Workgroup
// dispatch"), so the 8 channels of one octet (4 line pairs) go to blocks 8
// apart and their reads of each shared line hit that XCD's L2 after the first.  Channels past
// the last whole 64 keep b -> b.  Placement only: any order is correct.
__device__ __forceinline__ int au_channel(int b, int C, bool tiled) {
  if (!tiled || b >= (C & ~63)) return b;
  const int x = b & 7, i = b >> 3;
  return ((i >> 3) << 6) | (x << 3) | (i & 7);
}

/* ================================================================== */
/* k_frontend                                                         */
/* ================================================================== */
struct FeShared {
  float carry_i, carry_q; // DC blocker v of the last processed sample
  float carry_n[2];       // k_fe8: the same after the chunk's last sample, by its owner thread
  float2 cold_y[32];      // k_fe8: a cold channel's first outputs, computed in f32 from the bytes
  float fd_re, fd_im;     // discriminator r_prev (last IQ FIR / AGC output)
  float wave_a[4], wave_bi[4], wave_bq[4];
  int clip;
  int e_begin, e_end;
};

// Decimator: outputs j = 3*tid + r of the chunk.  inq is phase-major:
// inq[ph * Q + q] holds input li = q*M + ph; poly[p][qq] = taps[qq*M + p].
// One phase at a time (not unrolled) keeps the live set to ~30 half2 loads.
template <int M, int TPP>
__device__ __forceinline__ void fe_decimate(const __half2 *inq, int Q, const float *__restrict__ poly, int tid,
                                            float (&ai)[3], float (&aq)[3]) {
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    ai[r] = 0.0f;
    aq[r] = 0.0f;
  }
#pragma unroll 1
  for (int p = 0; p < M; ++p) {
    const __half2 *row = inq + (M - 1 - p) * Q + 3 * tid + (TPP - 1);
    const FMX_CONST float *h = cptr(poly) + p * TPP;
#pragma unroll
    for (int s = -(TPP - 1); s <= 2; ++s) {
      const __half2 hv = row[s];
      const float xi = __low2float(hv);
      const float xq = __high2float(hv);
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int qq = r - s;
        if (qq >= 0 && qq < TPP) {
          ai[r] = fmaf(h[qq], xi, ai[r]);
          aq[r] = fmaf(h[qq], xq, aq[r]);
        }
      }
    }
  }
}

// Decimator on natural-order u8 IQ in LDS (VEC path).  raw holds samples
// s = 0.. of the window origin n0*M - L, 2 bytes each; outputs j = 3*tid + r
// need s in [j*M + 1, j*M + L].  Thread t reads dwords (3M/2)*t + e: for
// M = 10 the stride is 15 dwords, conflict-free.  hpad = dec_pad (+PAD);
// (I, Q) pairs go through packed FP32 FMAs on the raw byte values; the
// caller subtracts D->dec_dc = 127.5 * sum(h) per output (the reference's
// per-sample (v - 127.5) offset, factored out of the dot product).
typedef float f32x2 __attribute__((ext_vector_type(2)));
template <int M, int TPP>
__device__ __forceinline__ void fe_decimate_u8(const uint8_t *raw, const float *__restrict__ hpad, int tid,
                                               f32x2 (&acc)[3]) {
  constexpr int L = M * TPP;
  constexpr int NB = TPP + 3;  // blocks of M samples covering s in [0, 2M + L]
  const uint32_t *rw = reinterpret_cast<const uint32_t *>(raw) + (3 * M / 2) * tid;
#pragma unroll
  for (int r = 0; r < 3; ++r) acc[r] = f32x2{0.0f, 0.0f};
#pragma unroll 1
  for (int qb = 0; qb < NB; ++qb) {
    const FMX_CONST float *hq = cptr(hpad) + FMX_DEC_PAD + L - qb * M;  // tap of sample u, output r: hq[r*M - u]
    uint32_t w[M / 2];
#pragma unroll
    for (int e = 0; e < M / 2; ++e) w[e] = rw[qb * (M / 2) + e];
#pragma unroll
    for (int u = 0; u < M; ++u) {
      const uint32_t ww = w[u >> 1];
      f32x2 x;
      const int sh0 = (u & 1) ? 16 : 0;  // v_cvt_f32_ubyte{0..3}
      x.x = (float)((ww >> sh0) & 255u);
      x.y = (float)((ww >> (sh0 + 8)) & 255u);
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const float h = hq[r * M - u];
        acc[r] = __builtin_elementwise_fma(f32x2{h, h}, x, acc[r]);
      }
    }
  }
}

// Real-tap FIR of runtime length L on a complex LDS signal, 3 outputs per
// thread at x[base + r]; hp = taps padded with 5 zeros on each side
// (hp[k + 5] = h[k]), x needs 3 samples of slack past base + 2.
__device__ __forceinline__ void fir_c3(const float2 *x, int base, const float *__restrict__ hp, int L,
                                       float (&zr)[3], float (&zi)[3]) {
  float r0 = 0.0f, r1 = 0.0f, r2 = 0.0f, i0 = 0.0f, i1 = 0.0f, i2 = 0.0f;
#pragma unroll 1
  for (int s = -(L - 1); s <= 2; s += 4) {
    const FMX_CONST float *h = cptr(hp) + 5 - s; // h[r - u] = taps[r - (s + u)]
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float2 v = x[base + s + u];
      r0 = fmaf(h[0 - u], v.x, r0);
      i0 = fmaf(h[0 - u], v.y, i0);
      r1 = fmaf(h[1 - u], v.x, r1);
      i1 = fmaf(h[1 - u], v.y, i1);
      r2 = fmaf(h[2 - u], v.x, r2);
      i2 = fmaf(h[2 - u], v.y, i2);
    }
  }
  zr[0] = r0;
  zr[1] = r1;
  zr[2] = r2;
  zi[0] = i0;
  zi[1] = i1;
  zi[2] = i2;
}

// Real FIR of runtime length P on a real LDS signal, 3 outputs per thread;
// hp padded as above; x needs 3 samples of slack past base + 2.
__device__ __forceinline__ void fir_r3(const float *x, int base, const float *__restrict__ hp, int P,
                                       float (&z)[3]) {
  float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f;
#pragma unroll 1
  for (int s = -(P - 1); s <= 2; s += 4) {
    const FMX_CONST float *h = cptr(hp) + 5 - s;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float v = x[base + s + u];
      a0 = fmaf(h[0 - u], v, a0);
      a1 = fmaf(h[1 - u], v, a1);
      a2 = fmaf(h[2 - u], v, a2);
    }
  }
  z[0] = a0;
  z[1] = a1;
  z[2] = a2;
}

// fir_r3 with the (y0, y1) pair on packed FP32 FMAs: hq[k] = {hp[k], hp[k+1]}.
// Same FMA sequence per output as fir_r3, so bit-identical results.
__device__ __forceinline__ void fir_r3p(const float *x, int base, const float *__restrict__ hp,
                                        const float (*__restrict__ hq)[2], int P, float (&z)[3]) {
  f32x2 a01 = {0.0f, 0.0f};
  float a2 = 0.0f;
#pragma unroll 1
  for (int s = -(P - 1); s <= 2; s += 4) {
    const FMX_CONST float *h = cptr(hp) + 5 - s;
    const FMX_CONST float(*h2)[2] = cptr(hq) + 5 - s;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float v = x[base + s + u];
      const f32x2 hh = {h2[-u][0], h2[-u][1]};  // taps of y0, y1
      a01 = __builtin_elementwise_fma(hh, f32x2{v, v}, a01);
      a2 = fmaf(h[2 - u], v, a2);
    }
  }
  z[0] = a01.x;
  z[1] = a01.y;
  z[2] = a2;
}

// Resampler output from a window accessor; reference dot order (oldest first).
// The boundary case (branch 31 of window i-1 blended with branch 0 of window
// i) only swaps the branch / window indices, so both cases run the same
// loop: no divergence in a wave that mixes them.
template <int SUB, typename Get>
__device__ __forceinline__ float resamp_out(const float *__restrict__ hb, int packed, float mu, Get get) {
  const int i = packed & 0xFFFF;
  const int b = (packed >> 16) & 0xFF;
  const bool boundary = (packed >> 24) & 1;
  const float *h0 = hb + (boundary ? FMX_NPFB - 1 : b) * SUB;
  const float *h1 = hb + (boundary ? 0 : b + 1) * SUB;
  const int i0 = boundary ? i - 1 : i;
  float y0 = 0.0f, y1 = 0.0f;
#pragma unroll
  for (int m = 0; m < SUB; ++m) {
    const float v0 = get(i0 - (SUB - 1) + m);
    const float v1 = get(i - (SUB - 1) + m);
    const float p0 = h0[SUB - 1 - m] * v0;
    const float p1 = h1[SUB - 1 - m] * v1;
    y0 = y0 + p0;
    y1 = y1 + p1;
  }
  const float w0 = (1.0f - mu) * y0;
  const float w1 = mu * y1;
  return w0 + w1;
}

// resamp_out with the two branch dot products as one packed (y0, y1) chain:
// hp[n][b] = {h_b[n], h_(b+1)%32[n]} (branch 31 pairs with branch 0, the
// boundary case), the window pair {x[i0-25+m], x[i-25+m]} from one 8-byte
// read (i0 = i - 1 at a boundary, else the same sample twice).  Products and
// sums are the same IEEE operations in the same order as resamp_out.
template <int SUB>
__device__ __forceinline__ float resamp_out_pair(const float2 (*hp)[FMX_NPFB], int packed, float mu,
                                                 const float *win) {
  const int i = packed & 0xFFFF;
  const int b = (packed >> 16) & 0xFF;
  const bool boundary = (packed >> 24) & 1;
  const int bb = boundary ? FMX_NPFB - 1 : b;
  const float *w = win + (boundary ? i - 1 : i) - (SUB - 1);
  f32x2 y = {0.0f, 0.0f};
#pragma unroll
  for (int m = 0; m < SUB; ++m) {
    const float2 h = hp[SUB - 1 - m][bb];
    const float va = w[m], vb = w[m + 1];
    const f32x2 v = {va, boundary ? vb : va};
    const f32x2 p = f32x2{h.x, h.y} * v;
    y = y + p;
  }
  const float w0 = (1.0f - mu) * y.x;
  const float w1 = mu * y.y;
  return w0 + w1;
}


__device__ __forceinline__ int sched_lower_bound(const FmxSched *s, int n, int i) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((s[mid].packed & 0xFFFF) < i) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// RF level accumulators of the raw u8 IQ (computeSignalLevel,
// signal_level.cpp:145-204): exact integer sums, clip counts per sample.
struct SigAcc {
  // sQ and sQQ are kept as sI + sQ and sII + sQQ (one byte dot product each)
  uint32_t sI = 0, sQ = 0, sII = 0, sQQ = 0, hard = 0, nearc = 0;
  __device__ __forceinline__ void sample(uint32_t i, uint32_t q) {
    sI += i;
    sQ += i + q;
    sII += i * i;
    sQQ += i * i + q * q;
    const uint32_t lo = min(i, q), hi = max(i, q);
    hard += (lo <= 1u || hi >= 254u) ? 1u : 0u;
    nearc += (lo <= 8u || hi >= 247u) ? 1u : 0u;
  }
  __device__ __forceinline__ void flags(uint32_t i, uint32_t q) {
    const uint32_t lo = min(i, q), hi = max(i, q);
    hard += (lo <= 1u || hi >= 254u) ? 1u : 0u;
    nearc += (lo <= 8u || hi >= 247u) ? 1u : 0u;
  }
  // bytes I0 Q0 I1 Q1: the four sums by byte dot products; the clip counters
  // only when some byte is <= 8 or >= 247 (fmx_word_near_clip)
  __device__ __forceinline__ void sums(uint32_t w) {
    sI = __builtin_amdgcn_udot4(w, 0x00010001u, sI, false);
    sQ = __builtin_amdgcn_udot4(w, 0x01010101u, sQ, false);
    sII = __builtin_amdgcn_udot4(w & 0x00FF00FFu, w, sII, false);
    sQQ = __builtin_amdgcn_udot4(w, w, sQQ, false);
  }
  // 16 bytes (8 IQ samples): the near-clip pre-test of the four words ORed,
  // one branch per 16 B
  template <typename V4> __device__ __forceinline__ void word4(const V4 &w) {
    sums(w.x);
    sums(w.y);
    sums(w.z);
    sums(w.w);
    if (fmx_word_near_clip(w.x) | fmx_word_near_clip(w.y) | fmx_word_near_clip(w.z) | fmx_word_near_clip(w.w)) {
      const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        flags(ww[k] & 255u, (ww[k] >> 8) & 255u);
        flags((ww[k] >> 16) & 255u, ww[k] >> 24);
      }
    }
  }
  // the separate sums back from the combined ones
  __device__ __forceinline__ void finish() {
    sQ -= sI;
    sQQ -= sII;
  }
};

// RF-level epilogue of a frontend workgroup: block-reduce the exact byte sums
// of computeSignalLevel (signal_level.cpp:145-204) and store them; the
// reference's double formulas run in k_audio (signal_level_eval), off the
// front end's critical path (one f64 log10 per workgroup tail cost ~0.05 ms
// per k_fe8 launch).
__device__ __forceinline__ void fe_signal_sums(const FeArgs &a, SigAcc sig, unsigned long long *sgp, int c,
                                               int lane, int wave, int tid) {
  sig.finish();
  unsigned long long v[6] = {sig.sI, sig.sQ, sig.sII, sig.sQQ, sig.hard, sig.nearc};
#pragma unroll
  for (int k = 0; k < 6; ++k)
    for (int d = 32; d >= 1; d >>= 1) v[k] += __shfl_xor(v[k], d);
  if (lane == 0)
    for (int k = 0; k < 6; ++k) sgp[wave * 6 + k] = v[k];
  __syncthreads();
  if (tid < 6) a.sig_sums[6 * (size_t)c + tid] = sgp[tid] + sgp[6 + tid] + sgp[12 + tid] + sgp[18 + tid];
}

// computeSignalLevel + smoothSignalLevel (signal_level.cpp:145-214) of one
// channel from its byte sums (t: sum I, sum Q, sum I^2, sum Q^2, hard-clip
// and near-clip counts over `samples` IQ samples), in double as the reference
__device__ __forceinline__ void signal_level_eval(const unsigned long long *sums, long samples, const double *sp,
                                                  float *sm, fmx_signal_level *out) {
  double t[6];
  for (int k = 0; k < 6; ++k) t[k] = (double)sums[k];
  fmx_signal_level r;
  r.level120 = 0.0f;
  r.dbfs = -120.0;
  r.compensated_dbfs = -120.0;
  r.hard_clip_ratio = 0.0;
  r.near_clip_ratio = 0.0;
  if (samples > 0) {
    // sums of (b - 127.5) / 127.5 and its square from the exact byte sums
    const double nn = (double)samples, k1 = 1.0 / 127.5;
    const double sumI = (t[0] - 127.5 * nn) * k1, sumQ = (t[1] - 127.5 * nn) * k1;
    const double sumII = (t[2] - 255.0 * t[0] + 16256.25 * nn) * (k1 * k1);
    const double sumQQ = (t[3] - 255.0 * t[1] + 16256.25 * nn) * (k1 * k1);
    const double meanI = sumI / nn, meanQ = sumQ / nn;
    const double varI = fmax(0.0, (sumII / nn) - (meanI * meanI));
    const double varQ = fmax(0.0, (sumQQ / nn) - (meanQ * meanQ));
    const double rms = sqrt(fmax(1e-15, 0.5 * (varI + varQ)));
    // sp: gain*factor, bias, floor, ceil
    r.dbfs = 20.0 * log10(rms + 1e-12);
    r.compensated_dbfs = r.dbfs - sp[0] + sp[1];
    const double safeCeil = fmax(sp[3], sp[2] + 1.0);
    const double norm = (r.compensated_dbfs - sp[2]) / (safeCeil - sp[2]);
    const float l = (float)(norm * 120.0);
    r.level120 = l < 0.0f ? 0.0f : (l > 120.0f ? 120.0f : l);
    r.hard_clip_ratio = t[4] / nn;
    r.near_clip_ratio = t[5] / nn;
  }
  // smoothSignalLevel (signal_level.cpp:206-214)
  if (sm[1] == 0.0f) {
    sm[0] = r.level120;
    sm[1] = 1.0f;
  } else {
    const float alpha = (r.level120 > sm[0]) ? 0.42f : 0.18f;
    sm[0] += (r.level120 - sm[0]) * alpha;
  }
  r.level120_smoothed = sm[0];
  *out = r;
}

// LDS layout of k_frontend (shared with the launcher's size computation).
// VEC: the decimator input is natural-order u8 IQ (HB halo bytes + the
// chunk); otherwise fp16 pairs in phase-major order.
template <int M, int TPP, bool VEC> struct FeLayout {
  static constexpr int L = (M > 1) ? M * TPP : 1;
  static constexpr int Q = FE_T + ((M > 1) ? TPP : 1);
  static constexpr int HB = ((2 * (L - 1)) + 15) & ~15;       // VEC halo bytes (16-B aligned)
  static constexpr int RAW_BYTES = HB + 2 * FE_T * M + 64;     // + slack read past the chunk
  static constexpr int IN_BYTES = (M > 1) ? (VEC ? RAW_BYTES : M * Q * 4) : 0;
  static constexpr int YB_BYTES = (FE_T + 1) * 8;
  static constexpr int R0 = ((IN_BYTES > YB_BYTES ? IN_BYTES : YB_BYTES) + 15) & ~15;
  static constexpr int XIN = R0;
  static constexpr int MX = XIN + (FE_HALO_IQ + FE_T + 8) * 8;
  static constexpr int RB = MX + (FMX_HIST + FE_T + 8) * 4;   // RDS resampler window: 32 history + chunk
  static constexpr int RSH = RB + (32 + FE_T + 8) * 4;           // RDS resampler filter bank (per-lane branch)
  static constexpr int SG = RSH + FMX_NPFB * FMX_RDS_RS_SUB * 8;  // 4 waves x 6 u64 RF-level partials
  static constexpr int SH = SG + 4 * 6 * 8;
  static constexpr int BYTES = SH + (int)sizeof(FeShared);
  static constexpr int NPF = (M > 1) ? (RAW_BYTES - 64 + 16 * 256 - 1) / (16 * 256) : 1;  // 16-B loads / thread
};

// The next step's RDS schedule slot (FeArgs::next_sched_*): one 16-B word
// per thread of the first workgroups, from the mapped pinned image.  Readers
// are the next front end launch on the same stream (k_fe8 copies at its end,
// k_frontend at its entry).
__device__ __forceinline__ void fe_next_sched_copy(const FeArgs &a) {
  if (a.next_sched_n16 == 0) return;
  const unsigned i = blockIdx.x * 256u + threadIdx.x;
  if (i < a.next_sched_n16) static_cast<uint4 *>(a.next_sched_dst)[i] = static_cast<const uint4 *>(a.next_sched_src)[i];
}

template <int M, int TPP, bool VEC>
__global__ __launch_bounds__(256) void k_frontend(FeArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  fe_next_sched_copy(a);
  using LY = FeLayout<M, TPP, VEC>;
  static_assert(!VEC || LY::HB >= 2 * LY::L, "VEC halo must hold L samples");
  static_assert(!VEC || 3 * M <= FMX_DEC_PAD, "dec_pad too short for this M");
  constexpr int L = LY::L;
  constexpr int Q = LY::Q;
  __half2 *inq = reinterpret_cast<__half2 *>(smem);
  uint8_t *raw = reinterpret_cast<uint8_t *>(smem);
  float2 *yb = reinterpret_cast<float2 *>(smem);
  float2 *xin = reinterpret_cast<float2 *>(smem + LY::XIN);
  float *mx = reinterpret_cast<float *>(smem + LY::MX);
  float *rb = reinterpret_cast<float *>(smem + LY::RB);
  unsigned long long *sgp = reinterpret_cast<unsigned long long *>(smem + LY::SG);
  float *rsh = reinterpret_cast<float *>(smem + LY::RSH);
  FeShared *sh = reinterpret_cast<FeShared *>(smem + LY::SH);
  const bool want_sig = a.sig_sums != nullptr && a.in_mode != FE_IN_CF && a.in_mode != FE_IN_MPX;
  SigAcc sig;
  // diagnostic stage clock (thread 0's view, barrier waits included):
  // compiled only with -DFMX_STAMPS (make STAMPS=1) and read through
  // fmx_debug_stamps when the handle was created with FMX_STAMPS=1
#ifdef FMX_STAMPS
  unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long st_last = (a.dbg && threadIdx.x == 0) ? __builtin_amdgcn_s_memtime() : 0;
#define FE_STAMP(k)                                              \
  if (a.dbg && tid == 0) {                                       \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();  \
    st_acc[k] += t_ - st_last;                                   \
    st_last = t_;                                                \
  }
#else
#define FE_STAMP(k)
#endif

  const int c = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const FmxDesign *__restrict__ D = a.des;
  const int n = a.n;
  const FmxChanParam par = a.par[c];
  const int iqL = D->iq_len[par.iqsel];
  const float *__restrict__ iqh = D->iq_pad[par.iqsel];
  const float iqscale = D->iq_scale[par.iqsel];
  const bool demod = a.do_demod != 0;
  const bool pilot = a.pilot_out != nullptr;
  const bool hist_out = pilot || a.st_hist_out != 0; // the stereo history rows
  const bool rds = a.rds_out != nullptr;
  const float dc_a1 = -1.0f + 0.0005f; // iirfilt_rrrf_create_dc_blocker(0.0005)
  const float dc_c = -dc_a1;

  // zero the FIR slack past the chunk (read against zero-padded taps)
  for (int h = tid; h < FE_HALO_IQ + FE_T + 8; h += 256) xin[h] = make_float2(0.0f, 0.0f);
  for (int h = tid; h < FMX_HIST + FE_T + 8; h += 256) mx[h] = 0.0f;
  __syncthreads();
  // ---- load carried state ----
  if (demod) {
    for (int h = tid; h < FE_HALO_IQ; h += 256) {
      const float2_t v = a.iq_hist[(size_t)c * (FMX_IQ_MAXLEN - 1) + h];
      xin[h] = make_float2(v.x, v.y);
    }
    if (tid == 0) {
      sh->carry_i = a.dc_v[2 * c];
      sh->carry_q = a.dc_v[2 * c + 1];
      sh->fd_re = a.fd_prev[2 * c];
      sh->fd_im = a.fd_prev[2 * c + 1];
    }
  }
  if (hist_out || rds || demod) {
    const float *hist = a.st_hist_rd + (size_t)c * FMX_HIST;
    for (int h = tid; h < FMX_HIST; h += 256) mx[h] = hist_out ? hist[h] : 0.0f;
  }
  if (tid == 0) sh->clip = 0;
  float agc_g = 1.0f, agc_y2p = 1.0f;
  if (demod && par.agc != 0 && tid == 0) {
    agc_g = a.agc[2 * c];
    agc_y2p = a.agc[2 * c + 1];
  }
  const float agc_bw = (par.agc == 1) ? 0.01f : 0.001f;
  int dec_valid = 0;
  if (a.in_mode == FE_IN_U8_DECIM) dec_valid = a.dec_valid[c];
  const uint16_t *iq16 = reinterpret_cast<const uint16_t *>(a.iq + (size_t)c * a.iq_stride);
  const uint8_t *dhist = a.dec_hist + (size_t)c * 2 * FMX_MAX_DEC;
  // RDS schedule of this channel's timing group
  const FmxSched *sched = nullptr;
  int sched_n = 0;
  if (rds) {
    const int g = a.rds_group[c];
    sched = a.rds_sched + (size_t)g * a.rds_sched_stride;
    sched_n = a.rds_sched_n[g];
  }
  const float *rhist = a.rds_hist + (size_t)c * 32;
  if (rds && tid < 32) rb[tid] = rhist[tid];
  // RDS resampler bank as (branch, next branch) pairs: rsp[n][b]
  float2(*rsp)[FMX_NPFB] = reinterpret_cast<float2(*)[FMX_NPFB]>(rsh);
  if (rds)
    for (int k = tid; k < FMX_NPFB * FMX_RDS_RS_SUB; k += 256) {
      const int b = k / FMX_RDS_RS_SUB, nn = k % FMX_RDS_RS_SUB;
      rsp[nn][b] = make_float2(D->rds_rs_h[k], D->rds_rs_h[((b + 1) % FMX_NPFB) * FMX_RDS_RS_SUB + nn]);
    }
  int e_pos = 0;
  // VEC: chunk bytes [2*n0*M - HB, 2*(n0+cnt)*M) are fetched with 16-B loads
  // one chunk ahead into registers (HBM latency hidden behind the previous
  // chunk); the host guarantees 16-B aligned rows and a full decimator history.
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  u32x4 pf[LY::NPF];
  auto prefetch = [&](int n0p) {
    const long nb = LY::HB + 2L * min(FE_T, n - n0p) * M;
    const uint8_t *base = a.iq + (size_t)c * a.iq_stride + 2L * n0p * M - LY::HB;
#pragma unroll
    for (int j = 0; j < LY::NPF; ++j) {
      const long off = 16L * (tid + 256 * j);
      u32x4 v = {0u, 0u, 0u, 0u};
      if (off < nb && (n0p > 0 || off >= LY::HB))  // nb is a multiple of 16 (host check)
        v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(base + off));
      pf[j] = v;
    }
  };
  if constexpr (VEC && M > 1) {
    if (n > 0) prefetch(0);
  }
  __syncthreads();

  for (int n0 = 0; n0 < n; n0 += FE_T) {
    const int cnt = min(FE_T, n - n0);
    if (rds && tid == 0) sh->e_end = e_pos;  // raised by atomicMax in the RDS stage
    FE_STAMP(7)
    // ================= baseband x[j] =================
    if constexpr (VEC && M > 1) {
#pragma unroll
      for (int j = 0; j < LY::NPF; ++j) {
        const int off = 16 * (tid + 256 * j);
        if (off < LY::HB + 2 * FE_T * M && (n0 > 0 || off >= LY::HB))
          *reinterpret_cast<u32x4 *>(raw + off) = pf[j];
        if (want_sig && off >= LY::HB && off < LY::HB + 2 * cnt * M) {
          sig.word4(pf[j]);
        }
      }
      if (n0 == 0) {  // halo = the carried history (dec_valid == L-1 here)
        for (int h = tid; h < LY::HB / 2; h += 256) {
          const int hh = h - (LY::HB / 2 - (L - 1));  // history index, < 0 unused
          uint16_t v = 0;
          if (hh >= 0) v = (uint16_t)dhist[2 * hh] | ((uint16_t)dhist[2 * hh + 1] << 8);
          reinterpret_cast<uint16_t *>(raw)[h] = v;
        }
      }
      if (n0 + FE_T < n) prefetch(n0 + FE_T);
      __syncthreads();
      f32x2 acc[3];
      // window origin in raw: sample HB/2 - L (so that s = j*M + 1 .. j*M + L)
      fe_decimate_u8<M, TPP>(raw + (LY::HB - 2 * L), D->dec_pad, tid, acc);
      int myclip = 0;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int j = 3 * tid + r;
        if (j < cnt) {
          const float yr = (acc[r].x - D->dec_dc) * D->dec_scale;
          const float yi = (acc[r].y - D->dec_dc) * D->dec_scale;
          if (fabsf(yr) >= 0.995f || fabsf(yi) >= 0.995f) myclip++;
          xin[FE_HALO_IQ + j] = make_float2(yr, yi);
          if (a.bb_out) {
            float *o = a.bb_out + (size_t)c * a.bb_stride + 2 * (size_t)(n0 + j);
            o[0] = yr;
            o[1] = yi;
          }
        }
      }
      if (myclip) atomicAdd(&sh->clip, myclip);
      __syncthreads();  // raw aliases yb
    } else if (a.in_mode == FE_IN_U8_DECIM) {
      if constexpr (M > 1) {
        if (want_sig)
          for (int j = tid; j < cnt * M; j += 256) {
            const uint16_t w = iq16[(long)n0 * M + j];
            sig.sample(w & 255u, w >> 8);
          }
        const long g0 = (long)n0 * M - (L - 1);
        const int span = (cnt - 1) * M + L;
        for (int li = tid; li < span; li += 256) {
          const long g = g0 + li;
          float fi = 0.0f, fq = 0.0f;
          if (g >= 0) {
            const uint16_t w = iq16[g];
            fi = (float)(w & 255) - 127.5f;
            fq = (float)(w >> 8) - 127.5f;
          } else {
            const int h = (L - 1) + (int)g;
            if (h >= (L - 1) - dec_valid) {
              fi = (float)dhist[2 * h] - 127.5f;
              fq = (float)dhist[2 * h + 1] - 127.5f;
            }
          }
          inq[(li % M) * Q + li / M] = __floats2half2_rn(fi, fq);
        }
        __syncthreads();
        float ai[3], aq[3];
        fe_decimate<M, TPP>(inq, Q, D->dec_poly, tid, ai, aq);
        int myclip = 0;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          const int j = 3 * tid + r;
          if (j < cnt) {
            const float yr = ai[r] * D->dec_scale;
            const float yi = aq[r] * D->dec_scale;
            if (fabsf(yr) >= 0.995f || fabsf(yi) >= 0.995f) myclip++;
            xin[FE_HALO_IQ + j] = make_float2(yr, yi);
            if (a.bb_out) {
              float *o = a.bb_out + (size_t)c * a.bb_stride + 2 * (size_t)(n0 + j);
              o[0] = yr;
              o[1] = yi;
            }
          }
        }
        if (myclip) atomicAdd(&sh->clip, myclip);
        __syncthreads(); // inq aliases yb
      }
    } else if (a.in_mode == FE_IN_CF) {
      int myclip = 0;
      for (int j = tid; j < cnt; j += 256) {
        const float *p = a.in_f + (size_t)c * a.in_stride + 2 * (size_t)(n0 + j);
        const float xr = p[0], xi = p[1];
        if (fabsf(xr) >= 0.995f || fabsf(xi) >= 0.995f) myclip++;
        xin[FE_HALO_IQ + j] = make_float2(xr, xi);
      }
      if (myclip) atomicAdd(&sh->clip, myclip);
    } else if (a.in_mode == FE_IN_U8_DIRECT) {
      int myclip = 0;
      const uint8_t *p = a.iq + (size_t)c * a.iq_stride;
      for (int j = tid; j < cnt; j += 256) {
        const uint8_t ib = p[2 * (size_t)(n0 + j)], qb = p[2 * (size_t)(n0 + j) + 1];
        if (ib == 0 || ib == 255 || qb == 0 || qb == 255) myclip++;
        if (want_sig) sig.sample(ib, qb);
        xin[FE_HALO_IQ + j] = make_float2(((float)ib - 127.0f) / 127.5f, ((float)qb - 127.0f) / 127.5f);
      }
      if (myclip) atomicAdd(&sh->clip, myclip);
    }
    __syncthreads();

    if (demod) {
      FE_STAMP(0)
      // ================= DC blockers: affine scan =================
      // v_k = x_k - a1 * v_{k-1} (DF-II); y_k = v_k - v_{k-1}
      float A = 1.0f, BI = 0.0f, BQ = 0.0f;
      float2 xv[3];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int j = 3 * tid + r;
        xv[r] = (j < cnt) ? xin[FE_HALO_IQ + j] : make_float2(0.0f, 0.0f);
        if (j < cnt) {
          BI = xv[r].x + dc_c * BI;
          BQ = xv[r].y + dc_c * BQ;
          A = dc_c * A;
        }
      }
      // inclusive wave scan of maps (later o earlier)
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const float pA = __shfl_up(A, d);
        const float pI = __shfl_up(BI, d);
        const float pQ = __shfl_up(BQ, d);
        if (lane >= d) {
          BI = A * pI + BI;
          BQ = A * pQ + BQ;
          A = A * pA;
        }
      }
      if (lane == 63) {
        sh->wave_a[wave] = A;
        sh->wave_bi[wave] = BI;
        sh->wave_bq[wave] = BQ;
      }
      // exclusive within the wave
      float eA = __shfl_up(A, 1), eI = __shfl_up(BI, 1), eQ = __shfl_up(BQ, 1);
      if (lane == 0) {
        eA = 1.0f;
        eI = 0.0f;
        eQ = 0.0f;
      }
      __syncthreads();
      // prefix of earlier waves applied to the chunk carry
      float vI = sh->carry_i, vQ = sh->carry_q;
      for (int w = 0; w < wave; ++w) {
        vI = sh->wave_a[w] * vI + sh->wave_bi[w];
        vQ = sh->wave_a[w] * vQ + sh->wave_bq[w];
      }
      vI = eA * vI + eI;
      vQ = eA * vQ + eQ;
      // serial recompute in the reference order
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int j = 3 * tid + r;
        if (j < cnt) {
          const float tI = dc_a1 * vI;
          const float tQ = dc_a1 * vQ;
          const float nI = xv[r].x - tI;
          const float nQ = xv[r].y - tQ;
          xin[FE_HALO_IQ + j] = make_float2(nI - vI, nQ - vQ);
          vI = nI;
          vQ = nQ;
          if (j == cnt - 1) {
            sh->carry_i = nI;
            sh->carry_q = nQ;
          }
        }
      }
      __syncthreads();
      FE_STAMP(1)
      // ================= IQ FIR =================
      {
        float zr[3], zi[3];
        fir_c3(xin, FE_HALO_IQ + 3 * tid, iqh, iqL, zr, zi);
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          const int j = 3 * tid + r;
          if (j < cnt) yb[1 + j] = make_float2(zr[r] * iqscale, zi[r] * iqscale);
        }
        if (tid == 0) yb[0] = make_float2(sh->fd_re, sh->fd_im);
      }
      __syncthreads();
      // ================= AGC (serial, only when enabled) =================
      if (par.agc != 0) {
        if (tid == 0) {
          for (int j = 0; j < cnt; ++j) {
            const float2 x = yb[1 + j];
            const float yr = x.x * agc_g, yi = x.y * agc_g;
            const float y2 = yr * yr + yi * yi;
            agc_y2p = (float)((1.0 - (double)agc_bw) * (double)agc_y2p + (double)(agc_bw * y2));
            if (agc_y2p > 1e-6f) agc_g *= expf(-0.5f * agc_bw * logf(agc_y2p));
            if (agc_g > 1e6f) agc_g = 1e6f;
            yb[1 + j] = make_float2(yr, yi);
          }
        }
        __syncthreads();
      }
      FE_STAMP(2)
      // ================= discriminator =================
      const float ref = (par.fd_ref != 0.0f) ? par.fd_ref : D->fd_ref; // freqdem 1 / (2 pi kf)
      for (int j = tid; j < cnt; j += 256) {
        const float2 p = yb[j], r = yb[1 + j];
        const float re = p.x * r.x + p.y * r.y;
        const float im = p.x * r.y - p.y * r.x;
        const float m = fmx_atan2f(im, re) * ref; // as k_fe8 (fmx_math.h)
        mx[FMX_HIST + j] = m;
        if (rds) rb[32 + j] = m;
        if (a.mpx_out) a.mpx_out[(size_t)c * a.mpx_stride + n0 + j] = m;
      }
    } else if (a.in_mode == FE_IN_MPX) {
      for (int j = tid; j < cnt; j += 256) {
        const float m = a.in_f[(size_t)c * a.in_stride + n0 + j];
        mx[FMX_HIST + j] = m;
        if (rds) rb[32 + j] = m;
      }
    }
    __syncthreads();

    FE_STAMP(3)
    // RDS resampler schedule entries of this chunk (<= FE_T of them, the
    // rate ratio is < 1), fetched now so their latency hides behind the
    // pilot FIR; the chunk's end index is found from them in parallel.
    FmxSched en3[3];
    if (rds) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int e = e_pos + tid + 256 * k;
        en3[k] = (e < sched_n) ? sched[e] : FmxSched{0xFFFF, 0.0f};
      }
    }
    // ================= 19 kHz pilot band-pass =================
    if (pilot) {
      float z[3];
      fir_r3p(mx, FMX_HIST + 3 * tid, D->pilot_pad, D->pilot_pair, D->pilot_len, z);
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int j = 3 * tid + r;
        if (j < cnt) a.pilot_out[(size_t)c * a.pilot_stride + n0 + j] = z[r];
      }
    }
    FE_STAMP(4)
    // ================= RDS resampler 240k -> 171k =================
    if (rds) {
      int last = -1;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int e = e_pos + tid + 256 * k;
        if (e < sched_n && (en3[k].packed & 0xFFFF) < n0 + cnt) {
          a.rds_out[(size_t)c * a.rds_stride + e] =
              resamp_out_pair<FMX_RDS_RS_SUB>(rsp, en3[k].packed, en3[k].mu, rb + 32 - n0);
          last = e;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (last >= 0) atomicMax(&sh->e_end, last + 1);
    }
    __syncthreads();
    if (rds) e_pos = sh->e_end;
    FE_STAMP(5)
    // ================= carry halos to the next chunk =================
    {
      float2 cx = make_float2(0.0f, 0.0f);
      float cm0 = 0.0f, cm1 = 0.0f;
      if (demod && tid < FE_HALO_IQ) cx = xin[tid + cnt];
      cm0 = mx[tid + cnt];
      cm1 = mx[tid + 256 + cnt];
      const float2 cy = yb[cnt];
      const float crb = (rds && tid < 32) ? rb[cnt + tid] : 0.0f;
      __syncthreads();
      if (rds && tid < 32) rb[tid] = crb;
      if (demod && tid < FE_HALO_IQ) xin[tid] = cx;
      mx[tid] = cm0;
      mx[tid + 256] = cm1;
      if (tid == 0 && demod) {
        sh->fd_re = cy.x;
        sh->fd_im = cy.y;
      }
      __syncthreads();
    }
  }

  // ---- write back state ----
  if (a.in_mode == FE_IN_U8_DECIM && M > 1) {
    // last L-1 input samples (2 bytes each)
    const long total = (long)n * M;
    uint16_t keep[2];
    int cntk = 0;
    for (int h = tid; h < L - 1; h += 256) {
      const long g = total - (L - 1) + h;
      uint16_t v;
      if (g >= 0) v = iq16[g];
      else {
        const int hh = (L - 1) + (int)g; // old history index
        v = (uint16_t)dhist[2 * hh] | ((uint16_t)dhist[2 * hh + 1] << 8);
      }
      keep[cntk++] = v;
    }
    __syncthreads();
    cntk = 0;
    uint8_t *dh = a.dec_hist + (size_t)c * 2 * FMX_MAX_DEC;
    for (int h = tid; h < L - 1; h += 256) {
      const uint16_t v = keep[cntk++];
      dh[2 * h] = (uint8_t)(v & 255);
      dh[2 * h + 1] = (uint8_t)(v >> 8);
    }
    if (tid == 0) {
      long nv = (long)dec_valid + total;
      a.dec_valid[c] = (int)(nv > (L - 1) ? (L - 1) : nv);
    }
  }
  if (demod) {
    for (int h = tid; h < FE_HALO_IQ; h += 256) {
      const float2 v = xin[h];
      a.iq_hist[(size_t)c * (FMX_IQ_MAXLEN - 1) + h] = float2_t{v.x, v.y};
    }
    if (tid == 0) {
      a.dc_v[2 * c] = sh->carry_i;
      a.dc_v[2 * c + 1] = sh->carry_q;
      a.fd_prev[2 * c] = sh->fd_re;
      a.fd_prev[2 * c + 1] = sh->fd_im;
      if (par.agc != 0) {
        a.agc[2 * c] = agc_g;
        a.agc[2 * c + 1] = agc_y2p;
      }
    }
  }
  if (hist_out) {
    float *hist = a.st_hist_wr + (size_t)c * FMX_HIST;
    for (int h = tid; h < FMX_HIST; h += 256) hist[h] = mx[h];
  }
  if (rds) {
    // new RDS resampler window: last 32 MPX samples (carried in rb)
    if (tid < 32) a.rds_hist[(size_t)c * 32 + tid] = rb[tid];
    if (tid == 0) a.rds_count[c] = sched_n;
  }
  FE_STAMP(6)
#ifdef FMX_STAMPS
  if (a.dbg && tid == 0)
    for (int k = 0; k < 8; ++k) atomicAdd(a.dbg + k, st_acc[k]);
#endif
#undef FE_STAMP
  if (tid == 0 && a.clip_out && a.in_mode != FE_IN_MPX)
    a.clip_out[c] = (n > 0) ? (float)sh->clip / (float)n : 0.0f;
  if (want_sig) fe_signal_sums(a, sig, sgp, c, lane, wave, tid);
}

/* ================================================================== */
/* k_pll: StereoDecoder per-sample recurrences                         */
/* ================================================================== */
/* k_pll (round 4): only the two recurrences the reference makes serial stay
 * serial, one channel per lane; everything else runs one item (channel row,
 * sample t) per lane.  A workgroup takes CH = 16 (24) channels in tiles of
 * PLL_T = 16 samples (256 items: one 16-lane DPP row per channel in each of
 * the four P waves), so 2 048 channels are 128 workgroups and 4 096 are 256:
 *   W0 (serial)   the PLL feedback chain only: error = pilot * sin(phase),
 *                 pll_step, step; hands the NCO words on        stereo_decoder.cpp:178-192
 *   P stage A     tile k-1: v_sin / v_cos / float phase of each word, the
 *                 previous sample's by DPP row_ror:1 (t = 0: the previous
 *                 tile's t = 15); PLL frequency (unwrap, clamp), cos(2 phase),
 *                 the pilot I/Q integrator inputs; the four linear recurrences
 *                 x = kS x + u (pilot / MPX envelopes, pilot I / Q) as a
 *                 16-lane inclusive scan (DPP row_shr 1, 2, 4, 8 with kS^d)
 *                 plus kS^(t+1) times the row's carry (ds_bpermute of the
 *                 tile's last sample); |I, Q|^2 and the blend target  :120-205
 *   WB (serial)   the blend smoother (attack / release select)   :226-228
 *   P stage B     tile k-3: the L/R matrix from the delayed MPX and cos(2
 *                 phase) with the blend, the raw L/R stores      :207-231
 * The P waves also move the pilot (3 tiles ahead), MPX and delay-line (1
 * ahead) words into LDS by per-lane LDS-DMA with counted waits.  At
 * iteration k: W0 tile k, A k-1, WB k-2, B k-3.  The chain's sine / NCO
 * constrain are v_sin of the word in turns and an f32 fract (round 3:
 * tools/ubench/chainlat.hip, 72 ticks per sample); the outputs' sine / cosine
 * are v_sin / v_cos of the word (the reference takes cos / sin of the word's
 * float phase: |difference| <= 5e-7); the scans sum the recurrences' terms in
 * a tree instead of one sample at a time (relative differences of a few
 * ulp).  Round 3's seven-wave form kept the envelopes / integrators (W1) and
 * the matrix + blend + stores (W3) in one-lane-per-channel waves, which set
 * its pace (W3 1.73 M, W1 1.67 M, the W0 chain 0.99 M ticks per launch-WG)
 * and gave 2 048 channels only 64 workgroups. */
// One dword per lane from a per-lane global address into LDS m0 + 4 lane
// (LDS-DMA as inline asm: the compiler's wait-count pass does not see it, so
// the issuing wave's own counted s_waitcnt vmcnt are the only waits and the
// moves stay in flight across loop iterations; k_rds, k_pll's first tiles)
__device__ __forceinline__ void dma_dword(const float *src, uint32_t lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds))
               : "memory");
}
// the same from a wave-uniform base plus a per-lane byte offset (saddr form;
// k_pll's P waves): the compiler's LDS-DMA builtin, which sets M0 itself (no
// save / restore around each move) and, in k_pll's loop, adds no wait of its
// own (round 5; in k_rds's loop it adds a vmcnt(0) after the moves: asm there)
__device__ __forceinline__ void dma_dword_s(const float *base, uint32_t voff, uint32_t lds) {
  __builtin_amdgcn_global_load_lds(reinterpret_cast<const char *>(base) + voff,
                                   (__attribute__((address_space(3))) void *)(uintptr_t)__builtin_amdgcn_readfirstlane(lds), 4, 0, 0);
}
// three dwords per lane (12 B, landing at m0 + 12 lane) from a per-lane address
__device__ __forceinline__ void dma_dwordx3(const float *src, uint32_t lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx3 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds))
               : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
  return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char *)p);
}
// sine and cosine of an NCO word (fmx_word_sincos, fmx_math.h)
__device__ __forceinline__ void word_sincos(uint32_t theta, float *s, float *c) { fmx_word_sincos(theta, s, c); }

#include "fmx_pll.inc"

/* ================================================================== */
/* k_audio: L/R FIRs, 32 kHz resampler, de-emphasis, DC block, clamp  */
/* ================================================================== */
/* k_audio: one workgroup (256 threads) per channel, the call in chunks of
 * AU2_T DSP samples, L and R carried together as packed (L, R) pairs:
 *   L/R 121-tap FIRs         v_mfma_f32_16x16x32_f16: the pilot BPF's
 *                            Toeplitz tiles (k_fe8) on f16 hi / lo images
 *                            of the chunk's L and R (x 2^10) and the
 *                            design's tap fragments (FmxDesign::lr_frag,
 *                            x 2^12), three MFMAs per K step   stereo_decoder.cpp:281-282
 *   resampler Fs -> 32 kHz   one output per thread and entry of the host
 *                            timing schedule (branch-transposed bank)   af_post_processor.cpp:56-64
 *   de-emphasis, DC block    block affine scans, 3 outputs per thread,
 *                            then the reference's op order            :66-75, fm_demod.cpp:218-224
 *   clamp (main.cpp:1305-1308), stores.
 * Modes: 0 stereo (FIR + AF), 1 AF only, 2 mono FMDemod::downsampleAudio,
 * 3 mono pipeline (x0.5, L = R), 4 FIR only (fmx_stereo). */
#define AU2_T 2048
#define AU2_PT 8                        // chunk inputs per thread (AU2_T / 256)
#define AU2_MAXOUT (AU2_T / 3 + 16)     // resampler outputs per chunk (ratio >= 3)
#define AU_IMG (AU_HALO + AU2_T + 24) // f16 image: 120 history + the chunk + the last K step's reach
#define AU_FN (AU_RHALO + AU2_T)
struct AuShared {
  // one region, two lives per chunk: the f16 hi / lo images of L and R (120
  // of history first) until the FIR has read them, then the resampler input
  // f (32 of history first)
  float2 xf[AU_IMG > AU_FN ? AU_IMG : AU_FN] __attribute__((aligned(16))); // (4 f16 images = AU_IMG pairs)
  float2 fh[AU_RHALO];                         // f's history between chunks
  float2 o[AU2_MAXOUT];                        // resampler outputs of the chunk
  float hT[FMX_AF_SUB][FMX_NPFB];              // resampler bank transposed: hT[n][b] = h_b[n]
  float2 hf[AU_HALO];                          // the chunk's last 120 (L, R) inputs: the next chunk's FIR history
  float ws[3][4][2];                           // scan scratch (A, BL, BR per wave)
  float iir[4];                                // de_L, de_R, dc_L, dc_R
  int eb, ee, count;
  // the L/R FIR tap window (FmxDesign::lr_q16 [2][2][FMX_LR_QN] u16, whole
  // 64-dword LDS-DMA pieces)
  uint32_t lrq[((2 * FMX_LR_QN + 63) / 64) * 64] __attribute__((aligned(16)));
};

// DPP move of x (CTRL, rows ROWS); lanes that receive nothing get id
template <int CTRL, int ROWS> __device__ __forceinline__ float dpp_or(float x, float id) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, id), __builtin_bit_cast(int, x), CTRL,
                                                               ROWS, 0xF, false));
}
// Inclusive wave64 scan of affine maps v -> A v + (B1, B2), earlier lanes
// applied first, by DPP (no LDS round trip: ds_bpermute per step before
// round 4): row_shr 1, 2, 4, 8 inside each 16-lane row, then row_bcast:15
// into rows 1 and 3 and row_bcast:31 into rows 2 and 3.  Lanes that receive
// nothing combine with the identity (1, 0, 0): exact.
#define WAVE_AFF_STEP(CTRL, ROWS)                                                       \
  {                                                                                   \
    const float pA_ = dpp_or<CTRL, ROWS>(A, 1.0f), p1_ = dpp_or<CTRL, ROWS>(B1, 0.0f); \
    const float p2_ = dpp_or<CTRL, ROWS>(B2, 0.0f);                                     \
    B1 = A * p1_ + B1;                                                                \
    B2 = A * p2_ + B2;                                                                \
    A = A * pA_;                                                                      \
  }
__device__ __forceinline__ void wave_affine_scan(float &A, float &B1, float &B2) {
  WAVE_AFF_STEP(0x111, 0xF)
  WAVE_AFF_STEP(0x112, 0xF)
  WAVE_AFF_STEP(0x114, 0xF)
  WAVE_AFF_STEP(0x118, 0xF)
  WAVE_AFF_STEP(0x142, 0xA)
  WAVE_AFF_STEP(0x143, 0xC)
}
#undef WAVE_AFF_STEP
// the previous lane's map (wave_shr:1; lane 0: the identity)
__device__ __forceinline__ void wave_affine_prev(float A, float B1, float B2, float &eA, float &e1, float &e2) {
  eA = dpp_or<0x138, 0xF>(A, 1.0f);
  e1 = dpp_or<0x138, 0xF>(B1, 0.0f);
  e2 = dpp_or<0x138, 0xF>(B2, 0.0f);
}

// exclusive block scan (256 threads) of per-thread affine maps v -> A v + B
// (B for L and R), applied to the carries: the state before this thread's
// first element.
__device__ __forceinline__ void au_scan_prev(float A, float BL, float BR, float cl, float cr, float (*ws)[4][2],
                                             float &pl, float &pr) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  wave_affine_scan(A, BL, BR);
  if (lane == 63) {
    ws[0][wave][0] = A;
    ws[1][wave][0] = BL;
    ws[2][wave][0] = BR;
  }
  float eA, eL, eR;
  wave_affine_prev(A, BL, BR, eA, eL, eR);
  __syncthreads();
  float vl = cl, vr = cr;
  for (int w = 0; w < wave; ++w) {
    vl = ws[0][w][0] * vl + ws[1][w][0];
    vr = ws[0][w][0] * vr + ws[2][w][0];
  }
  pl = eA * vl + eL;
  pr = eA * vr + eR;
  __syncthreads(); // ws reusable
}

#ifndef FMX_AU_WPE
#define FMX_AU_WPE 1 // k_audio waves per SIMD the register budget allows (A/B switch; 1 = the compiler's choice)
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FMX_AU_WPE))) void k_audio(AudioArgs a) {
  // dynamic LDS, as k_rds: a static 45 KB made the backend pad the VGPR
  // allocation from 111 to 129 (occupancy 3 by LDS)
  extern __shared__ __align__(16) unsigned char au_smem[];
  AuShared &S = *reinterpret_cast<AuShared *>(au_smem);
  const int c = au_channel(blockIdx.x, a.C, a.in_tiled != 0);
  const int tid = threadIdx.x;
  const FmxDesign *__restrict__ D = a.des;
  const FmxChanParam par = a.par[c];
  const int n = a.n;
  const bool mono = (a.mode == 2 || a.mode == 3);
  const bool lrfir = (a.mode == 0 || a.mode == 4);
  const bool af = (a.mode != 4);
  const bool pipe_mono = (a.mode == 3);
  const int deemph = par.deemph;
  const float dalpha = (deemph == 0) ? D->deemph_alpha[0] : ((deemph == 1) ? D->deemph_alpha[1] : par.deemph_alpha);
  const bool de_on = deemph != 2;
  const float dc_alpha = mono ? 0.0008f : 0.005f;
  const float de_a1 = -(1.0f - dalpha);
  const float dc_a1 = -1.0f + dc_alpha;
  // the step's RF levels: workgroup b evaluates channels 256 b .. 256 b + 255
  // from the front end's byte sums (one thread each)
  if (a.sig_out && blockIdx.x * 256 < (unsigned)a.C) {
    const int cs = blockIdx.x * 256 + tid;
    if (cs < a.C)
      signal_level_eval(a.sig_sums + 6 * (size_t)cs, a.sig_samples, a.sig_par + 4 * (size_t)cs,
                        a.sig_smooth + 2 * (size_t)cs, a.sig_out + cs);
  }
  // ---- carried state ----
  float *lrh = a.lr_hist + (size_t)c * 2 * (FMX_LR_LEN - 1);
  float *win = mono ? a.mono_win + (size_t)c * 32 : a.af_win + (size_t)c * 2 * 32;
  float2 *const F = S.xf; // resampler input, after the FIR
  // this thread's pair of the FIR history (threads < 120), across chunks
  float2 cx = make_float2(0.0f, 0.0f);
  if (lrfir && tid < AU_HALO) cx = make_float2(lrh[tid], lrh[(FMX_LR_LEN - 1) + tid]);
  if (af)
    for (int h = tid; h < AU_RHALO; h += 256) S.fh[h] = make_float2(win[h], mono ? 0.0f : win[32 + h]);
  float *iir = mono ? a.mono_iir + (size_t)c * 2 : a.af_iir + (size_t)c * 4;
  if (af && tid == 0) {
    if (mono) {
      S.iir[0] = iir[0];
      S.iir[1] = 0.0f;
      S.iir[2] = iir[1];
      S.iir[3] = 0.0f;
    } else {
      for (int k = 0; k < 4; ++k) S.iir[k] = iir[k];
    }
  }
  const FmxSched *sched = nullptr;
  int sched_n = 0;
  if (af) {
    const int g = a.group[c];
    sched = a.sched + (size_t)g * a.sched_stride;
    sched_n = a.sched_n[g];
    for (int k = tid; k < FMX_NPFB * FMX_AF_SUB; k += 256) {
      const int b = k / FMX_AF_SUB, nn = k % FMX_AF_SUB;
      S.hT[nn][b] = D->af_h[k];
    }
  }
  if (lrfir) { // the L/R FIR tap window by LDS-DMA (waited for before the FIR's barrier)
    static_assert(FMX_LR_QN % 2 == 0, "dword window");
    const float *qs = reinterpret_cast<const float *>(&D->lr_q16[0][0][0]);
    for (int p = tid >> 6; p < (2 * FMX_LR_QN + 63) / 64; p += 4)
      dma_dword(qs + min(64 * p + (tid & 63), 2 * FMX_LR_QN - 1), lds_addr(&S.lrq[64 * p]));
  }
  if (tid == 0) {
    S.eb = 0;
    S.count = 0;
  }
  // tiled input (raw L/R from k_pll): sample j of this channel at tin + ti(j)
  const bool tiled = a.in_tiled != 0;
  const float *inl = a.in_l + (tiled ? lr_tile_idx(c, 0, a.in_stride) : (size_t)c * a.in_stride);
  const float *inr = mono ? nullptr : a.in_r + (tiled ? lr_tile_idx(c, 0, a.in_stride) : (size_t)c * a.in_stride);
  auto ti = [&](int j) __attribute__((always_inline)) { return tiled ? (j >> 4) * 32 + (j & 15) : j; };
  const float sc = D->lr_scale;
  // retune fade/mute of this call (main.cpp:1310-1337): outputs o < mrem
  // get the gain of position (mtot - mrem) + o of the fade-out/mute/fade-in
  int mrem = 0, mtot = 0;
  if (a.mute) {
    mrem = a.mute[2 * c];
    mtot = a.mute[2 * c + 1];
  }
  const int mdone = (mtot > mrem) ? mtot - mrem : 0;
  const int mfade = max(1, min(a.mute_fade, mtot / 2));
  __syncthreads();
  for (int n0 = 0; n0 < n; n0 += AU2_T) {
    const int cnt = min(AU2_T, n - n0);
    FmxSched en3[3];
    if (af) {
      const int eb = S.eb;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int e = eb + tid + 256 * k;
        en3[k] = (e < sched_n) ? sched[e] : FmxSched{0xFFFF, 0.0f};
      }
    }
    // ---- chunk input (all loads issued before the first LDS write) ----
    {
      float vl[AU2_PT], vr[AU2_PT];
#pragma unroll
      for (int k = 0; k < AU2_PT; ++k) {
        const int j = tid + 256 * k;
        vl[k] = (j < cnt) ? inl[ti(n0 + j)] : 0.0f;
        vr[k] = (j < cnt && !mono) ? inr[ti(n0 + j)] : 0.0f;
      }
      if (lrfir) {
        // f16 hi / lo images [L hi | L lo | R hi | R lo], index = chunk sample + 120
        _Float16 *im = reinterpret_cast<_Float16 *>(S.xf);
        auto put = [&](int i, float l, float r) __attribute__((always_inline)) {
          l *= 1024.0f;
          r *= 1024.0f;
          const _Float16 lh = (_Float16)l, rh = (_Float16)r;
          im[i] = lh;
          im[AU_IMG + i] = (_Float16)(l - (float)lh);
          im[2 * AU_IMG + i] = rh;
          im[3 * AU_IMG + i] = (_Float16)(r - (float)rh);
        };
        if (tid < AU_HALO) put(tid, cx.x, cx.y);
#pragma unroll
        for (int k = 0; k < AU2_PT; ++k) put(AU_HALO + tid + 256 * k, vl[k], vr[k]);
        if (tid < AU_IMG - AU_HALO - AU2_T) put(AU_HALO + AU2_T + tid, 0.0f, 0.0f); // zero taps' reach: finite
        // the next chunk's history, exact: inputs cnt - 120 .. cnt - 1 (the
        // older ones, for cnt < 120, from the current history)
#pragma unroll
        for (int k = 0; k < AU2_PT; ++k) {
          const int j = tid + 256 * k;
          if (j >= cnt - AU_HALO && j < cnt) S.hf[j - (cnt - AU_HALO)] = make_float2(vl[k], vr[k]);
        }
        if (tid < AU_HALO && tid >= cnt) S.hf[tid - cnt] = cx;
      } else {
#pragma unroll
        for (int k = 0; k < AU2_PT; ++k) {
          const int j = tid + 256 * k;
          if (j < cnt) F[AU_RHALO + j] = make_float2(vl[k], vr[k]);
        }
      }
      if (!lrfir && af && tid < AU_RHALO) F[tid] = S.fh[tid];
    }
    if (tid == 0) S.ee = S.eb;
    __syncthreads();
    // ---- L/R FIR on MFMA: 16 outputs (rows, A = taps) x 16 blocks of 16
    // outputs (columns, B = inputs), K = the block's 136 inputs from 120
    // before it; each wave two tiles of L and of R (512 outputs each) ----
    if (lrfir) {
      typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
      typedef float f32x4_t __attribute__((ext_vector_type(4)));
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      const int lane = tid & 63, wave = tid >> 6, col = lane & 15, g = lane >> 4;
      const _Float16 *im = reinterpret_cast<const _Float16 *>(S.xf);
      const int xb = 16 * (32 * wave + col) + 8 * g; // image index of block (2 wave) 16 + col's K start, 8-aligned
      const f16x8_t *bLh = reinterpret_cast<const f16x8_t *>(im + xb);
      const f16x8_t *bLl = reinterpret_cast<const f16x8_t *>(im + AU_IMG + xb);
      const f16x8_t *bRh = reinterpret_cast<const f16x8_t *>(im + 2 * AU_IMG + xb);
      const f16x8_t *bRl = reinterpret_cast<const f16x8_t *>(im + 3 * AU_IMG + xb);
      // A fragments from the LDS tap window (round 6; lr_frag's per-K-step
      // L2 loads before): this lane's 8 entries from 32 ks + 8 g + 15 - col
      // in copy (15 - col) & 1, four dwords
      const int qb = 8 * g + 15 - col, qc = qb & 1;
      const uint32_t *qh = &S.lrq[0] + qc * FMX_LR_QN + (qb - qc) / 2;
      const uint32_t *ql = qh + FMX_LR_QN / 2;
      auto frag = [&](int ks, const uint32_t *q) __attribute__((always_inline)) {
        return u32x4{q[16 * ks], q[16 * ks + 1], q[16 * ks + 2], q[16 * ks + 3]};
      };
      f32x4_t aL[2], aR[2];
      aL[0] = aL[1] = aR[0] = aR[1] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
      u32x4 ah = frag(0, qh), al = frag(0, ql);
#pragma unroll
      for (int ks = 0; ks < FMX_LR_KS; ++ks) {
        const f16x8_t ahi = __builtin_bit_cast(f16x8_t, ah), alo = __builtin_bit_cast(f16x8_t, al);
        if (ks + 1 < FMX_LR_KS) {
          ah = frag(ks + 1, qh);
          al = frag(ks + 1, ql);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const f16x8_t lh = bLh[32 * u + 4 * ks], ll = bLl[32 * u + 4 * ks]; // + 256 u + 32 ks samples
          const f16x8_t rh = bRh[32 * u + 4 * ks], rl = bRl[32 * u + 4 * ks];
          // transposed tiles (images as A, taps as B: the same lane
          // registers) -- D[block][output]: a 16-lane group holds 16
          // consecutive outputs
          aL[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(lh, ahi, aL[u], 0, 0, 0);
          aR[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(rh, ahi, aR[u], 0, 0, 0);
          aL[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ll, ahi, aL[u], 0, 0, 0);
          aR[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(rl, ahi, aR[u], 0, 0, 0);
          aL[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(lh, alo, aL[u], 0, 0, 0);
          aR[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(rh, alo, aR[u], 0, 0, 0);
        }
      }
      if (tid < AU_HALO) cx = S.hf[tid];
      __syncthreads(); // the images are read: F takes their place
      if (af && tid < AU_RHALO) F[tid] = S.fh[tid];
      const float osc = sc * (1.0f / 4194304.0f); // taps x 2^12, inputs x 2^10
#pragma unroll
      for (int u = 0; u < 2; ++u) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          // lane: output 256 (2 wave + u) + 16 (4 g + i) + col -- a 16-lane
          // group writes 16 consecutive pairs: conflict-free ds_write_b64
          // (untransposed, 4 consecutive outputs per lane, 16-B writes 128 B
          // apart across an 8-lane group: 8-way)
          const int j = 256 * (2 * wave + u) + 16 * (4 * g + i) + col;
          const float2 y = make_float2(aL[u][i] * osc, aR[u][i] * osc);
          if (af) F[AU_RHALO + j] = y;
          if (a.lr_out_l && j < cnt) {
            a.lr_out_l[(size_t)c * a.lr_out_stride + n0 + j] = y.x;
            a.lr_out_r[(size_t)c * a.lr_out_stride + n0 + j] = y.y;
          }
        }
      }
    }
    __syncthreads();
    if (af) {
      // ---- resampler: one schedule entry per thread ----
      const int eb = S.eb;
      int last = -1;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int e = eb + tid + 256 * k;
        if (e < sched_n && (en3[k].packed & 0xFFFF) < n0 + cnt) {
          const int i = (en3[k].packed & 0xFFFF) - n0;
          const int b = (en3[k].packed >> 16) & 0xFF;
          const bool boundary = (en3[k].packed >> 24) & 1;
          const int b0 = boundary ? FMX_NPFB - 1 : b, b1 = boundary ? 0 : b + 1;
          const int i0 = boundary ? i - 1 : i;
          // scalar multiply-then-add per channel and branch (the reference's
          // two roundings), as asm: the vectoriser's packed-FP32 form put LDS
          // loads right over the sources of a just-issued v_pk_* op (the
          // pattern tests/test_isa_scan.py keeps out of the shipped kernels)
          float y0l = 0.0f, y0r = 0.0f, y1l = 0.0f, y1r = 0.0f;
          auto mac = [](float &y, float h, float x) __attribute__((always_inline)) {
            float t;
            asm("v_mul_f32 %0, %2, %3\n\tv_add_f32 %1, %1, %0" : "=&v"(t), "+v"(y) : "v"(h), "v"(x));
          };
#pragma unroll
          for (int m = 0; m < FMX_AF_SUB; ++m) {
            const float2 v0 = F[AU_RHALO + i0 - (FMX_AF_SUB - 1) + m];
            const float2 v1 = F[AU_RHALO + i - (FMX_AF_SUB - 1) + m];
            const float h0 = S.hT[FMX_AF_SUB - 1 - m][b0], h1 = S.hT[FMX_AF_SUB - 1 - m][b1];
            mac(y0l, h0, v0.x);
            mac(y0r, h0, v0.y);
            mac(y1l, h1, v1.x);
            mac(y1r, h1, v1.y);
          }
          const float mu = en3[k].mu, omu = 1.0f - mu;
          float yl, yr;
          asm("v_mul_f32 %0, %2, %3\n\tv_mul_f32 %1, %2, %4" : "=&v"(yl), "=&v"(yr) : "v"(omu), "v"(y0l), "v"(y0r));
          mac(yl, mu, y1l);
          mac(yr, mu, y1r);
          S.o[e - eb] = make_float2(yl, yr);
          last = e;
        }
      }
      if (last >= 0) atomicMax(&S.ee, last + 1);
      __syncthreads();
      // ---- de-emphasis + DC block over the m outputs, 3 per thread ----
      const int m = S.ee - eb; // <= AU2_MAXOUT
      float xl[3], xr[3];
      bool on[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int q = 3 * tid + k;
        on[k] = q < m;
        const float2 v = on[k] ? S.o[q] : make_float2(0.0f, 0.0f);
        xl[k] = v.x;
        xr[k] = v.y;
      }
      auto compose = [&](float a_, const float *bl, const float *br, float &A, float &BL, float &BR) {
        A = 1.0f;
        BL = 0.0f;
        BR = 0.0f;
#pragma unroll
        for (int k = 0; k < 3; ++k)
          if (on[k]) {
            BL = a_ * BL + bl[k];
            BR = a_ * BR + br[k];
            A = a_ * A;
          }
      };
      if (de_on) {
        float A, BL, BR, pl, pr;
        compose(-de_a1, xl, xr, A, BL, BR);
        au_scan_prev(A, BL, BR, S.iir[0], S.iir[1], S.ws, pl, pr);
#pragma unroll
        for (int k = 0; k < 3; ++k)
          if (on[k]) {
            const float vl = xl[k] - de_a1 * pl, vr = xr[k] - de_a1 * pr;
            if (3 * tid + k == m - 1) {
              S.iir[0] = vl;
              S.iir[1] = vr;
            }
            pl = vl;
            pr = vr;
            xl[k] = dalpha * vl;
            xr[k] = dalpha * vr;
          }
      }
      float A, BL, BR, ql, qr;
      compose(-dc_a1, xl, xr, A, BL, BR);
      au_scan_prev(A, BL, BR, S.iir[2], S.iir[3], S.ws, ql, qr);
      const int o0 = S.count;
#pragma unroll
      for (int k = 0; k < 3; ++k)
        if (on[k]) {
          const float vl = xl[k] - dc_a1 * ql, vr = xr[k] - dc_a1 * qr;
          float yl = vl - ql, yr = vr - qr;
          if (3 * tid + k == m - 1) {
            S.iir[2] = vl;
            S.iir[3] = vr;
          }
          ql = vl;
          qr = vr;
          if (pipe_mono) yl = yl * 0.5f;
          if (a.clamp) {
            yl = d_clamp(yl, -1.0f, 1.0f);
            yr = d_clamp(yr, -1.0f, 1.0f);
          }
          const int o = o0 + 3 * tid + k;
          if (o < mrem) {
            const int idx = mdone + o;
            float gain = 0.0f;
            if (idx < mfade) gain = 1.0f - ((float)idx / (float)mfade);
            else if (idx >= mtot - mfade) gain = (float)(mtot - idx) / (float)mfade;
            gain = d_clamp(gain, 0.0f, 1.0f);
            yl *= gain;
            yr *= gain;
          }
          if (o < a.cap) {
            a.out_l[(size_t)c * a.out_stride + o] = yl;
            if (pipe_mono) a.out_r[(size_t)c * a.out_stride + o] = yl;
            else if (!mono) a.out_r[(size_t)c * a.out_stride + o] = yr;
          }
        }
      __syncthreads();
      if (tid == 0) {
        S.count = o0 + m;
        S.eb = eb + m;
      }
    }
    // ---- carry halos ----
    {
      float2 cf = make_float2(0.0f, 0.0f);
      if (af && tid < AU_RHALO) cf = F[tid + cnt];
      __syncthreads(); // F is dead: the next chunk's images take its place
      if (af && tid < AU_RHALO) S.fh[tid] = cf;
      __syncthreads();
    }
  }
  if (lrfir && tid < AU_HALO) {
    lrh[tid] = cx.x;
    lrh[(FMX_LR_LEN - 1) + tid] = cx.y;
  }
  if (af) {
    for (int h = tid; h < AU_RHALO; h += 256) {
      const float2 v = S.fh[h];
      win[h] = v.x;
      if (!mono) win[32 + h] = v.y;
    }
    if (tid == 0) {
      if (mono) {
        iir[0] = S.iir[0];
        iir[1] = S.iir[2];
      } else {
        for (int k = 0; k < 4; ++k) iir[k] = S.iir[k];
      }
    }
    const int nout = S.count < a.cap ? S.count : a.cap;
    if (tid == 0 && a.out_count) a.out_count[c] = nout;
    if (tid == 0 && a.mute && mrem > 0 && nout > 0) {
      const int mc = min(nout, mrem);
      a.mute[2 * c] = mrem - mc;
      if (mrem - mc == 0) a.mute[2 * c + 1] = 0;
    }
  }
}

/* ================================================================== */
/* k_rds: 57 kHz BPSK demodulator + block sync, one lane per channel   */
/* ================================================================== */
enum { OA = 0, OB = 1, OC = 2, OCP = 3, OD = 4, OINV = 5 };
__device__ __forceinline__ int bs_block_number(int off) {
  return (off == OA) ? 0 : (off == OB) ? 1 : (off == OC || off == OCP) ? 2 : (off == OD) ? 3 : 0;
}
__device__ __forceinline__ int bs_next(int off) {
  return (off == OA) ? OB : (off == OB) ? OC : (off == OC || off == OCP) ? OD : OA;
}
__device__ __forceinline__ int bs_offset_for(uint32_t s) {
  switch (s) {
    case 0x3D8: return OA; // 0b1111011000
    case 0x3D4: return OB; // 0b1111010100
    case 0x25C: return OC; // 0b1001011100
    case 0x3CC: return OCP; // 0b1111001100
    case 0x258: return OD; // 0b1001011000
    default: return OINV;
  }
}
__constant__ uint32_t c_parity[26] = {0x200, 0x100, 0x080, 0x040, 0x020, 0x010, 0x008, 0x004, 0x002,
                                      0x001, 0x2DC, 0x16E, 0x0B7, 0x287, 0x39F, 0x313, 0x355, 0x376,
                                      0x1BB, 0x201, 0x3DC, 0x1EE, 0x0F7, 0x2A7, 0x38F, 0x31B};
__device__ __forceinline__ uint32_t bs_syndrome(uint32_t v) {
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 26; ++k) r ^= ((v >> k) & 1u) ? c_parity[25 - k] : 0u;
  return r;
}
__device__ __forceinline__ bool pulse_follows(uint32_t pos, int off, uint32_t opos, int ooff) {
  const uint32_t d = pos - opos;
  return d % 26 == 0 && d / 26 <= 6 && off != OINV && ooff != OINV &&
         ((uint32_t)bs_block_number(ooff) + d / 26) % 4 == (uint32_t)bs_block_number(off);
}

// k_rds (round 3): RDS_LPC lanes per channel, RDS_CPW channels per
// workgroup (one wave).  The 255-tap low-pass runs as streaming partial sums
// (acc[i]: the i-th next decimation instant) kept PER LANE: the lanes of a
// channel take the samples of a decimation period in turn (period position
// j = lane + 8 q, q = 0..2), each with its own three tap columns, so the
// mix-down and the FIR products of a period run in parallel; the channel's
// output is the sum of its lanes' acc[0] (three DPP butterfly adds, bit-
// identical in every lane).  The NCO word of every sample is exact uint32
// arithmetic (theta_period_start + j * dtheta): between decimation instants
// the reference's NCO only steps (stepPLL runs at symbol instants,
// subcarrier.cpp:195-216).  AGC, symsync and the PSK2 PLL (the serial part,
// once per 24 samples) run redundantly in the channel's lanes; the bit
// decoders (biphase, delta, block sync) in its first lane.
// The mix-down phase of sample k is the NCO word's own phase, v_sin / v_cos
// of theta / 2^32 turns.  The reference mixes with the quad-phase wrapper's
// accumulator phases_[0] (liquid_wrappers.cpp:121-139), which sums
// unwrap(phase_now - prev) * 57000 / 57000 over the NCO's steps (PLL jumps
// included): it is the NCO phase mod 2 pi up to float rounding (a random walk
// of ~1e-7 rad per step); RDS groups stay bit-exact against the oracle
// (which keeps the reference's sum).
#define RDS_LPC 8                  // lanes per channel
#define RDS_CPW (64 / RDS_LPC)     // channels per wave / workgroup
#define RDS_SYMQ 12                // symbols queued per channel before the bit decoders run
#ifndef RDS_PF
#define RDS_PF 3                   // input rounds moved ahead (LDS-DMA)
#endif
#ifndef RDS_NR
#define RDS_NR 4                   // input ring slots (> RDS_PF, a power of two)
#endif
static_assert(RDS_PF < RDS_NR && (RDS_NR & (RDS_NR - 1)) == 0 && 3 * RDS_PF <= 63, "k_rds input ring");
static_assert(FMX_RDS_DECIM == 3 * RDS_LPC, "three samples per lane and decimation period");
// The bit-decoder state of FmxRdsState (biphase, delta, block sync) -- the
// only state k_rds keeps in LDS; the per-sample state lives in registers.
struct RdsBits {
  float bi_prev_re, bi_prev_im, bi_even, bi_odd;
  uint32_t bi_clock, bi_polarity;
  int delta_prev;
  uint32_t bs_bitcount, bs_until_next, bs_reg, bs_err_mask_lo, bs_err_mask_hi;
  int bs_expected, bs_in_sync, bs_err_ptr;
  uint32_t bs_pulse_pos[4];
  int bs_pulse_off[4];
  uint32_t bs_blk_raw[4];
  uint16_t bs_blk_data[4];
  uint8_t bs_blk_flags[4];
  uint32_t bs_bits_since_lost;
};
struct RdsCold {
  RdsBits s;
  uint32_t pad_[(sizeof(RdsBits) / 4) % 2 == 0 ? 1 : 2];
};
static_assert((sizeof(RdsCold) / 4) % 2 == 1, "RdsCold must have an odd dword stride");
__device__ __forceinline__ void rds_bits_load(RdsBits &b, const FmxRdsState &g) {
  b.bi_prev_re = g.bi_prev_re;
  b.bi_prev_im = g.bi_prev_im;
  b.bi_even = g.bi_even;
  b.bi_odd = g.bi_odd;
  b.bi_clock = g.bi_clock;
  b.bi_polarity = g.bi_polarity;
  b.delta_prev = g.delta_prev;
  b.bs_bitcount = g.bs_bitcount;
  b.bs_until_next = g.bs_until_next;
  b.bs_reg = g.bs_reg;
  b.bs_err_mask_lo = g.bs_err_mask_lo;
  b.bs_err_mask_hi = g.bs_err_mask_hi;
  b.bs_expected = g.bs_expected;
  b.bs_in_sync = g.bs_in_sync;
  b.bs_err_ptr = g.bs_err_ptr;
  for (int i = 0; i < 4; ++i) {
    b.bs_pulse_pos[i] = g.bs_pulse_pos[i];
    b.bs_pulse_off[i] = g.bs_pulse_off[i];
    b.bs_blk_raw[i] = g.bs_blk_raw[i];
    b.bs_blk_data[i] = g.bs_blk_data[i];
    b.bs_blk_flags[i] = g.bs_blk_flags[i];
  }
  b.bs_bits_since_lost = g.bs_bits_since_lost;
}
__device__ __forceinline__ void rds_bits_store(FmxRdsState &g, const RdsBits &b) {
  g.bi_prev_re = b.bi_prev_re;
  g.bi_prev_im = b.bi_prev_im;
  g.bi_even = b.bi_even;
  g.bi_odd = b.bi_odd;
  g.bi_clock = b.bi_clock;
  g.bi_polarity = b.bi_polarity;
  g.delta_prev = b.delta_prev;
  g.bs_bitcount = b.bs_bitcount;
  g.bs_until_next = b.bs_until_next;
  g.bs_reg = b.bs_reg;
  g.bs_err_mask_lo = b.bs_err_mask_lo;
  g.bs_err_mask_hi = b.bs_err_mask_hi;
  g.bs_expected = b.bs_expected;
  g.bs_in_sync = b.bs_in_sync;
  g.bs_err_ptr = b.bs_err_ptr;
  for (int i = 0; i < 4; ++i) {
    g.bs_pulse_pos[i] = b.bs_pulse_pos[i];
    g.bs_pulse_off[i] = b.bs_pulse_off[i];
    g.bs_blk_raw[i] = b.bs_blk_raw[i];
    g.bs_blk_data[i] = b.bs_blk_data[i];
    g.bs_blk_flags[i] = b.bs_blk_flags[i];
  }
  g.bs_bits_since_lost = b.bs_bits_since_lost;
}
/* ---- the RDS resampler's MFMA tile (k_rs; round 6: also the producer
 * fused into k_rds, FMX_RDS_FUSED) -- see k_rs below for the band-matrix
 * form ---- */
#define RS_KS 16   // K steps of 4 per 16-output tile: a 64-sample window (fmx_capi.cpp checks that it holds the tile)
// the tile's window, sample s of a channel at [c][RS_XS (s mod 4) + s / 4]:
// a lane's 16 samples of one K column are one 64-B run (4 ds_read_b128
// instead of 16 ds_read_b32 -- those were 2-way on the 32-bank rows), and the
// loader's 4 x 4 register transpose stores 16-B runs; rows 80 floats apart,
// columns 20: 1 extra cycle per read group, stores conflict-free
// (tools/lds_banks.py)
#define RS_XP 80
#define RS_XS 20
typedef float rs_f32x4 __attribute__((ext_vector_type(4)));
// the first window sample of a tile (a multiple of 4) from its row-0 entry
// (lane 0's; wave-uniform)
__device__ __forceinline__ int rs_tile_k0(const FmxSched &e) {
  const uint32_t p0 = __builtin_amdgcn_readlane(e.packed, 0);
  const int i0 = p0 & 0xFFFF;
  return ((((p0 >> 24) & 1) ? i0 - 1 : i0) - (FMX_RDS_RS_SUB - 1)) & ~3;
}
// 16 samples of a channel (quarter lq of the tile's 64) as four 16-B loads
// (4-sample groups lie wholly in the history, the block or past it: k0 and n
// are multiples of 4); unconditional loads (a branch here would make the
// compiler wait for them at the join): samples past the block or a lane
// without a channel read mrow[0] and are zeroed when written to LDS
__device__ __forceinline__ void rs_load_w(const float *mrow, const float *wrow, bool lcv, int n, int lq, int k0,
                                          float4 (&v)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = k0 + 16 * lq + 4 * j;
    const float *p = (!lcv || k >= n) ? mrow : (k < 0 ? wrow + k : mrow + k);
    v[j] = *reinterpret_cast<const float4 *>(p);
  }
}
// ... written to the channel's window row, transposed (samples 16 lq + 4 j + e:
// column e, rows 4 lq + j)
__device__ __forceinline__ void rs_store_w(float *xrow, bool lcv, int n, int lq, int k0, const float4 (&v)[4]) {
  float4 w[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bool ok = lcv && k0 + 16 * lq + 4 * j < n;
    w[j] = ok ? v[j] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  }
  *reinterpret_cast<float4 *>(&xrow[4 * lq]) = make_float4(w[0].x, w[1].x, w[2].x, w[3].x);
  *reinterpret_cast<float4 *>(&xrow[RS_XS + 4 * lq]) = make_float4(w[0].y, w[1].y, w[2].y, w[3].y);
  *reinterpret_cast<float4 *>(&xrow[2 * RS_XS + 4 * lq]) = make_float4(w[0].z, w[1].z, w[2].z, w[3].z);
  *reinterpret_cast<float4 *>(&xrow[3 * RS_XS + 4 * lq]) = make_float4(w[0].w, w[1].w, w[2].w, w[3].w);
}
// one tile: 16 outputs (rows, lane & 15 = r, entry en of row r) x 16
// channel columns (B: the window row xrow of column r), K = the window in
// steps of 4 (lane >> 4 = kk); D: lane (column r, outputs 4 kk .. 4 kk + 3)
__device__ __forceinline__ rs_f32x4 rs_tile(const float (*tab)[FMX_RDS_RS_SUB + 1], const float *xrow,
                                           const FmxSched &en, int kk) {
  const int i = en.packed & 0xFFFF, b = (en.packed >> 16) & 0xFF;
  const bool bnd = (en.packed >> 24) & 1;
  const int s_r = (bnd ? i - 1 : i) - (FMX_RDS_RS_SUB - 1); // the window's oldest sample
  // pair (branch b, branch b + 1) on one window, or at the boundary branch
  // 31 and branch 0 shifted by one
  const int row0 = bnd ? FMX_NPFB - 1 : b, row1 = bnd ? FMX_NPFB : ((b + 1) & (FMX_NPFB - 1));
  const int k0 = rs_tile_k0(en);
  const int m0 = k0 + kk - s_r; // this lane's tap index at K step 0
  // K steps the tile needs: up to the last row's window end (rows past the
  // call repeat the last entry; the schedule's windows only move forward)
  const uint32_t p15 = __builtin_amdgcn_readlane(en.packed, 15);
  const int i15 = p15 & 0xFFFF;
  const int s15 = ((((p15 >> 24) & 1) ? i15 - 1 : i15) - (FMX_RDS_RS_SUB - 1));
  const int ks = min(RS_KS, (s15 + FMX_RDS_RS_SUB - k0 + 3) / 4); // wave-uniform
  // row r's two branch filters combined with its interpolation weight:
  // (1 - mu) h_b + mu h_b+1, one MFMA chain (the reference interpolates the
  // two dot products, (1 - mu) y0 + mu y1: the same sum in another order)
  const float mu = en.mu, mu1 = 1.0f - mu;
  float hv[RS_KS], xv[RS_KS];
#pragma unroll
  for (int q = 0; q < RS_KS / 4; ++q) { // samples 4 st + kk, st = 4 q .. 4 q + 3
    const float4 x4 = *reinterpret_cast<const float4 *>(&xrow[RS_XS * kk + 4 * q]);
    xv[4 * q] = x4.x;
    xv[4 * q + 1] = x4.y;
    xv[4 * q + 2] = x4.z;
    xv[4 * q + 3] = x4.w;
  }
#pragma unroll
  for (int st = 0; st < RS_KS; ++st) {
    const int m = m0 + 4 * st;
    const int mc = min(max(m, 0), FMX_RDS_RS_SUB);
    const bool in = m >= 0 && m <= FMX_RDS_RS_SUB;
    hv[st] = in ? mu1 * tab[row0][mc] + mu * tab[row1][mc] : 0.0f;
  }
  rs_f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int st = 0; st < RS_KS; ++st)
    if (st < ks) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(hv[st], xv[st], acc, 0, 0, 0);
  return acc;
}
// the resampler's tap rows: row b < 32 branch b on the window, row 32
// branch 0 on the window shifted by one (the boundary pair's second branch)
__device__ __forceinline__ void rs_fill_tab(float (*tab)[FMX_RDS_RS_SUB + 1], const FmxDesign *D, int lane, int nl) {
  for (int idx = lane; idx < (FMX_NPFB + 1) * (FMX_RDS_RS_SUB + 1); idx += nl) {
    const int b = idx / (FMX_RDS_RS_SUB + 1), m = idx % (FMX_RDS_RS_SUB + 1);
    const float *hs = D->rds_rs_h; // [branch][26]
    float h;
    if (b < FMX_NPFB) h = m < FMX_RDS_RS_SUB ? hs[b * FMX_RDS_RS_SUB + FMX_RDS_RS_SUB - 1 - m] : 0.0f;
    else h = m >= 1 ? hs[FMX_RDS_RS_SUB - m] : 0.0f;
    tab[b][m] = h;
  }
}

struct RdsLds {
  // tap columns: hq[j0][i][q] = h[23 - (3 j0 + q) + 24 i] (zeros past tap 254),
  // q padded to 4 (one 16-B read per accumulator)
  float hq[RDS_LPC][FMX_RDS_NACC][4] __attribute__((aligned(16)));
  float mf[FMX_NPFB * FMX_SS_SUB];
  float dmf[FMX_NPFB * FMX_SS_SUB];
  // symsync window ring per channel, newest at wp, every sample written at
  // wp and wp + FMX_SS_SUB: the window oldest-first is win[w0 .. w0 + 17],
  // contiguous (constant read offsets, no wrap per tap)
  f32x2 win[2 * FMX_SS_SUB][RDS_CPW];
  float xin[RDS_NR][3][64];        // input ring: round r's sample 3 j0 + q of lane's channel at [r % RDS_NR][q][lane]
  uint32_t ck[RDS_CPW][FMX_RDS_CK][2]; // round 6: the NCO words of each channel's last rounds (round r at r % CK)
};
static_assert(FMX_RDS_DECIM * (FMX_RDS_CK - 1) + 1 >= FMX_RDS_RING, "the checkpoints cover the ring");

// the mix-down of one RDS-rate sample x with NCO word w (subcarrier.cpp:
// 153-160: x e^{-j phase}; the word's phase as a signed fraction of a turn,
// v_sin / v_cos): k_rds's and the ring refill's one formula (bit-identical)
__device__ __forceinline__ f32x2 rds_mix(float x, uint32_t w) {
  const float rr = (float)(int32_t)w * 2.3283064365386963e-10f; // w / 2^32 turns
  const float sn = -__builtin_amdgcn_sinf(rr);
  const float cs = __builtin_amdgcn_cosf(rr);
  return f32x2{x, x} * f32x2{cs, sn};
}
// Round 6: the RDS ring of one channel rebuilt from the checkpoints of its
// last call (FmxRdsState::ck_*, that call >= FMX_RDS_RING samples) and that
// call's RDS-rate input row `prev`: sample t of the call sat in round r
// (t <= o0: round 0, else 1 + (t - o0 - 1) / 24) at period position t -
// base_r and was mixed with ck_thp + (t - base_r) ck_dth of that round --
// k_rds's own words -- and lands where k_rds would have written it
// ((ring_pos - (count - t)) mod RING).  Threads k0, k0 + dk, ... take the
// ring's samples; the state is read from memory (a rare path: a reset, a
// short call after a long one, fmx_diag_rds_ring)
__device__ void rds_ring_fill(const FmxRdsState *sp, const float *prev, float *ring, int k0, int dk) {
  const int count = sp->ck_count, o0 = sp->ck_o0, R = sp->ck_rounds;
  const int first = R > FMX_RDS_CK ? R - FMX_RDS_CK : 0;
  const uint32_t rp = sp->ring_pos;
  for (int k = k0; k < FMX_RDS_RING; k += dk) {
    const int t = count - FMX_RDS_RING + k;
    const int r = t <= o0 ? 0 : 1 + (t - o0 - 1) / FMX_RDS_DECIM;
    const int base = r == 0 ? o0 - (FMX_RDS_DECIM - 1) : o0 + 1 + FMX_RDS_DECIM * (r - 1);
    const int i = min(max(r - first, 0), FMX_RDS_CK - 1);
    const uint32_t w = sp->ck_thp[i] + (uint32_t)(t - base) * sp->ck_dth[i];
    const uint32_t idx = (rp - (uint32_t)(count - t)) & (FMX_RDS_RING - 1);
    *reinterpret_cast<f32x2 *>(ring + 2 * idx) = rds_mix(prev[t], w);
  }
}
// the fused resampler's LDS (FMX_RDS_FUSED, behind RdsLds): k_rs's tap rows,
// its window double buffer for the wave's 8 channels, and a ring of the
// produced 171 kHz samples per channel (output e at [e % RDS_RSR])
#define RDS_RSR 128
struct RdsFusedLds {
  float tab[FMX_NPFB + 1][FMX_RDS_RS_SUB + 1];
  float xs[2][RDS_CPW][RS_XP] __attribute__((aligned(16)));
  float rsr[RDS_CPW][RDS_RSR] __attribute__((aligned(16)));
};
#define RDS_FOFF ((sizeof(RdsLds) + 15) & ~(size_t)15)
// k_bits: the bit decoders' LDS (burst-error tables, one bit state per lane)
struct BitsLds {
  uint32_t esyn[5][52];
  uint32_t eerr[5][52];
  RdsCold cold[64];
};

__device__ __forceinline__ void rds_emit_group(RdsBits &s, const RdsArgs &a, int c, int &ng) {
  fmx_rds_group g;
  uint8_t e[4];
  uint16_t d[4];
  for (int i = 0; i < 4; ++i) {
    const bool rec = s.bs_blk_flags[i] & 1;
    const bool had = (s.bs_blk_flags[i] >> 1) & 1;
    e[i] = rec ? (had ? 1 : 0) : 3;
    d[i] = rec ? s.bs_blk_data[i] : 0;
  }
  g.a = d[0];
  g.b = d[1];
  g.c = d[2];
  g.d = d[3];
  g.errors = (uint8_t)((e[0] << 6) | (e[1] << 4) | (e[2] << 2) | e[3]);
  g.pad = 0;
  g.block_index = a.block_index;
  if (ng < a.groups_stride) a.groups[(size_t)c * a.groups_stride + ng] = g;
  ng++;
}

// BlockStream::pushBit / findBlockInInputRegister / acquireSync
// (block_sync.cpp:235-313) and Group::setBlock (group.cpp:103-128)
__device__ __forceinline__ void rds_push_bit(RdsBits &s, int bit, const BitsLds &L, const RdsArgs &a, int c, int &ng) {
  s.bs_reg = (s.bs_reg << 1u) + (uint32_t)bit;
  s.bs_until_next--;
  s.bs_bitcount++;
  if (s.bs_until_next != 0) return;
  const uint32_t raw = s.bs_reg & ((1u << 26) - 1u);
  const uint32_t syn = bs_syndrome(raw);
  int off = bs_offset_for(syn);
  bool done = false;
  if (!s.bs_in_sync) {
    s.bs_bits_since_lost++;
    if (off != OINV) {
      for (int i = 0; i < 3; ++i) {
        s.bs_pulse_off[i] = s.bs_pulse_off[i + 1];
        s.bs_pulse_pos[i] = s.bs_pulse_pos[i + 1];
      }
      s.bs_pulse_off[3] = off;
      s.bs_pulse_pos[3] = s.bs_bitcount;
      bool found = false;
      for (int i = 0; i < 2; ++i)
        for (int j = i + 1; j < 3; ++j)
          found = found ||
                  (pulse_follows(s.bs_pulse_pos[3], s.bs_pulse_off[3], s.bs_pulse_pos[j], s.bs_pulse_off[j]) &&
                   pulse_follows(s.bs_pulse_pos[j], s.bs_pulse_off[j], s.bs_pulse_pos[i], s.bs_pulse_off[i]));
      if (found) {
        s.bs_in_sync = 1;
        s.bs_expected = off;
        for (int i = 0; i < 4; ++i) {
          s.bs_blk_flags[i] = 0;
          s.bs_blk_data[i] = 0;
          s.bs_blk_raw[i] = 0;
        }
        s.bs_bits_since_lost = 0;
      }
    }
  }
  if (s.bs_in_sync) {
    if (s.bs_expected == OC && off == OCP) s.bs_expected = OCP;
    const bool had = (off != s.bs_expected);
    // RunningSum<int, 50>
    const int p = s.bs_err_ptr;
    if (p < 32) {
      if (had) s.bs_err_mask_lo |= (1u << p);
      else s.bs_err_mask_lo &= ~(1u << p);
    } else {
      if (had) s.bs_err_mask_hi |= (1u << (p - 32));
      else s.bs_err_mask_hi &= ~(1u << (p - 32));
    }
    s.bs_err_ptr = (p + 1) % 50;
    if (__popc(s.bs_err_mask_lo) + __popc(s.bs_err_mask_hi) > 42) {
      s.bs_in_sync = 0;
      s.bs_err_mask_lo = 0;
      s.bs_err_mask_hi = 0;
      done = true;
    }
    if (!done) {
      uint16_t data = (uint16_t)(raw >> 10);
      if (had) {
        const uint32_t *es = L.esyn[s.bs_expected];
        const uint32_t *ee = L.eerr[s.bs_expected];
        for (int i = 0; i < 52; ++i)
          if (es[i] == syn) {
            data = (uint16_t)((raw ^ ee[i]) >> 10);
            off = s.bs_expected;
            break;
          }
      }
      if (off == s.bs_expected) {
        const int bn = bs_block_number(s.bs_expected);
        // (static indices: the state lives in registers in k_bits)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (i == bn) {
            s.bs_blk_raw[i] = raw;
            s.bs_blk_data[i] = data;
            s.bs_blk_flags[i] = (uint8_t)(1 | (had ? 2 : 0));
          }
      }
      const int next = bs_next(s.bs_expected);
      if (next == OA) {
        rds_emit_group(s, a, c, ng);
        for (int i = 0; i < 4; ++i) {
          s.bs_blk_flags[i] = 0;
          s.bs_blk_data[i] = 0;
          s.bs_blk_raw[i] = 0;
        }
      }
      s.bs_expected = next;
    }
  }
  s.bs_until_next = s.bs_in_sync ? 26u : 1u;
}


// the sums of two values over the 8 lanes of a channel group (DPP butterfly:
// quad_perm xor 1, xor 2, then row_half_mirror): every lane of the group
// gets the same bits (each step adds two identical pairs in swapped order).
// Round 5: one v_add_f32_dpp per step and value (a VALU write is read by DPP
// two wait states later: the s_nops) instead of v_mov_dpp + v_add, and never
// packed by the vectoriser beside LDS returns (tests/test_isa_scan.py)
__device__ __forceinline__ f32x2 rds_sum8x2(float x, float y) {
#define RDS_DPP(C) " row_mask:0xf bank_mask:0xf\n\t"
  asm volatile("s_nop 1\n\t"
               "v_add_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2]" RDS_DPP() "v_add_f32_dpp %1, %1, %1 quad_perm:[1,0,3,2]" RDS_DPP()
               "s_nop 0\n\t"
               "v_add_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1]" RDS_DPP() "v_add_f32_dpp %1, %1, %1 quad_perm:[2,3,0,1]" RDS_DPP()
               "s_nop 0\n\t"
               "v_add_f32_dpp %0, %0, %0 row_half_mirror" RDS_DPP() "v_add_f32_dpp %1, %1, %1 row_half_mirror" RDS_DPP()
               : "+v"(x), "+v"(y));
#undef RDS_DPP
  return f32x2{x, y};
}

// k_rds's tap columns (11 per lane, three taps each) held in registers for
// the whole call: the first FMX_RDS_HREG, the rest read from LDS per round
// (round 6: 6 -- 164 VGPRs, still beside two front-end waves; 2048 channels
// 0.3533 -> 0.3418 ms, 1024 0.276 -> 0.273, 4096 unchanged; all 11 at two
// waves per SIMD 0.3428, 8 0.3471: profiles/r06p_ab_rds_tap_registers_*.txt)
#ifndef FMX_RDS_HREG
#define FMX_RDS_HREG 6
#endif
#ifndef FMX_RDS_WPE
#define FMX_RDS_WPE 3 // k_rds waves per SIMD the register budget allows (A/B switch)
#endif
// (FUSED: two waves per SIMD's registers -- the producer's window
// registers; 512 one-wave workgroups at 4096 channels leave it room beside
// two k_fe8 waves)
template <bool FUSED>
__global__ __launch_bounds__(64, FUSED ? 2 : FMX_RDS_WPE) void k_rds(RdsArgs a) {
#ifndef FMX_RDS_PRIO
#define FMX_RDS_PRIO 2
#endif
  __builtin_amdgcn_s_setprio(FMX_RDS_PRIO); // beside the front end's waves (round 1: 1.39 -> 1.375 ms/step)
  // dynamic LDS (sizeof(RdsLds) at launch): with a static size the backend
  // sees an LDS-limited occupancy and pads every wave's register allocation
  // up to it
  extern __shared__ __align__(16) unsigned char rds_smem[];
  RdsLds &L = *reinterpret_cast<RdsLds *>(rds_smem);
#ifdef FMX_STAMPS
  // stage clocks (diagnostics build): 0 setup + state store, 1 input moves
  // and their wait, 2 mix-down, 3 FIR products, 4 FIR output + AGC, 5
  // symsync, 6 PSK2 / NCO update, 7 bit decoders
  unsigned long long rs_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long rs_last = __builtin_amdgcn_s_memtime();
#define RDS_STAMP(k)                                            \
  if (a.dbg) {                                                  \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    rs_acc[k] += t_ - rs_last;                                  \
    rs_last = t_;                                               \
  }
#else
#define RDS_STAMP(k)
#endif
  const int lane = threadIdx.x;
  const int g = lane / RDS_LPC, j0 = lane % RDS_LPC; // channel slot, first period position
  const int c0 = blockIdx.x * RDS_CPW;
  const int c = c0 + g;
  const bool act = c < a.C;
  const bool lead = j0 == 0;
  const FmxDesign *__restrict__ D = a.des;
  // ---- LDS tables ----
  for (int idx = lane; idx < FMX_NPFB * FMX_SS_SUB; idx += 64) {
    L.mf[idx] = D->ss_mf[idx];
    L.dmf[idx] = D->ss_dmf[idx];
  }
  for (int idx = lane; idx < RDS_LPC * FMX_RDS_NACC * 4; idx += 64) {
    const int jj = idx / (FMX_RDS_NACC * 4), i = (idx / 4) % FMX_RDS_NACC, q = idx % 4;
    L.hq[jj][i][q] = (q < 3) ? D->rds_fir[FMX_RDS_DECIM - 1 - (3 * jj + q) + FMX_RDS_DECIM * i] : 0.0f;
  }
  const FmxRdsState G = act ? a.st[c] : FmxRdsState{}; // the compiler loads only the fields used
  const int count = act ? a.in_count[c] : 0;
  float *ring = a.ring + (size_t)(act ? c : 0) * FMX_RDS_RING * 2;
  // round 6: a call of >= FMX_RDS_RING samples leaves the ring to its
  // checkpoints (FmxRdsState::ck_*); a shorter one writes its samples into
  // the ring, which must then hold the previous call's: refilled here first
  // when that call left checkpoints (the channel's 8 lanes, 32 samples each)
  const bool ringw = FUSED || a.ring_always || count < FMX_RDS_RING;
  {
    const bool refill = act && count > 0 && count < FMX_RDS_RING && !G.ring_ok && a.in_prev != nullptr;
    if (__ballot(refill)) {
      if (refill) rds_ring_fill(a.st + c, a.in_prev + (size_t)c * a.in_stride, ring, j0, RDS_LPC);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // before this call's own ring stores
    }
  }
  // ---- hot state -> registers ----
  uint32_t theta = G.theta, dtheta = G.dtheta;
  const uint32_t ssr0 = G.sample_since_reset;
  // this lane's share of the streaming partial sums (the channel's sums in
  // its first lane at entry)
  f32x2 acc[FMX_RDS_NACC];
  for (int i = 0; i < FMX_RDS_NACC; ++i) acc[i] = lead ? f32x2{G.acc_re[i], G.acc_im[i]} : f32x2{0.0f, 0.0f};
  {
    // decimation phase changed by a reset: rebuild the partial sums from the
    // last mixed samples (the reference's FIR window survives the reset).
    // Round 5: the whole wave computes each such channel's 11 sums (terms
    // strided over the 64 lanes, a shuffle tree) -- round 4's serial loop in
    // the channel's first lane, ~2 800 dependent ring loads, held the wave's
    // other seven channels ~80 us at every retune
    // (the sums go through the input ring's LDS, free until the first
    // moves below: a dynamically indexed acc[] would live in scratch)
    static_assert(RDS_CPW * FMX_RDS_NACC * 2 <= RDS_NR * 3 * 64, "rebuild sums fit the input ring");
    f32x2 *rb = reinterpret_cast<f32x2 *>(&L.xin[0][0][0]);
    const bool mine = act && lead && G.rebuild;
    uint64_t need = __ballot(mine);
    while (need) {
      const int src = __ffsll((unsigned long long)need) - 1;
      need &= need - 1;
      const uint32_t rp = (uint32_t)__shfl((int)G.ring_pos, src);
      const float *rg = a.ring + (size_t)(c0 + src / RDS_LPC) * FMX_RDS_RING * 2;
      for (int i = 0; i < FMX_RDS_NACC; ++i) {
        float ar = 0.0f, ai = 0.0f;
        for (int kp = FMX_RDS_FIR - 1 - 24 * i - lane; kp >= 1; kp -= 64) {
          const uint32_t idx = (rp - (uint32_t)kp) & (FMX_RDS_RING - 1);
          const float h = D->rds_fir[24 * i + kp];
          const float pr = h * rg[2 * idx];
          const float pi = h * rg[2 * idx + 1];
          ar = ar + pr;
          ai = ai + pi;
        }
        for (int d = 32; d >= 1; d >>= 1) { // scalar adds as asm: never packed beside the shuffles' LDS returns
          const float tr = __shfl_xor(ar, d), ti = __shfl_xor(ai, d);
          asm("v_add_f32 %0, %0, %2\n\tv_add_f32 %1, %1, %3" : "+v"(ar), "+v"(ai) : "v"(tr), "v"(ti));
        }
        if (lane == src) rb[(src / RDS_LPC) * FMX_RDS_NACC + i] = f32x2{ar, ai};
      }
    }
    if (mine)
#pragma unroll
      for (int i = 0; i < FMX_RDS_NACC; ++i) acc[i] = rb[g * FMX_RDS_NACC + i];
  }
  float agc_g = G.agc_g, agc_y2p = G.agc_y2p;
  float ss_rate = G.ss_rate, ss_del = G.ss_del, ss_tau = G.ss_tau, ss_q_hat = G.ss_q_hat, ss_v1 = G.ss_v1;
  int ss_b = G.ss_b, ss_decim = G.ss_decim, ss_valid = G.ss_mf_valid;
  if (lead)
    for (int m = 0; m < FMX_SS_SUB; ++m) L.win[m][g] = L.win[m + FMX_SS_SUB][g] = f32x2{G.ss_win_re[m], G.ss_win_im[m]};
  int wp = FMX_SS_SUB - 1; // newest window sample at wp
  const f32x2 fscale2 = f32x2{D->rds_fir_scale, D->rds_fir_scale};
  const float agc_bw = D->agc_bw;
  const float ss_b0 = D->ss_b0, ss_a1 = D->ss_a1, ss_adj = D->ss_rate_adj;
  const float psk_xr1 = D->psk_xr1, psk_xi1 = D->psk_xi1;
  const float alpha = D->rds_alpha, beta = D->rds_beta;
  const float dphi_psk = (float)(3.14159265358979323846 * (1.0 - 1.0 / 2));
  const uint32_t ring0 = G.ring_pos;
  // Rounds: round r of a channel ends on its r-th decimation instant of the
  // call (sample o0 + 24 r, sample_since_reset % 24 == 0 there,
  // subcarrier.cpp:186); round 0 holds samples 0..o0, the last round may end
  // before its instant (the tail, carried in acc).  Sample t of round r sits
  // at period position j = t - base_r.
  const int o0 = (int)((FMX_RDS_DECIM - ssr0 % FMX_RDS_DECIM) % FMX_RDS_DECIM);
  const int R = (count <= 0) ? 0 : (o0 >= count ? 1 : 1 + (count - o0 - 1 + FMX_RDS_DECIM - 1) / FMX_RDS_DECIM);
  int rmax = R;
  for (int d = 32; d >= 1; d >>= 1) rmax = max(rmax, __shfl_xor(rmax, d));
  // the NCO word at period position 0 of round 0 (virtual for o0 < 23)
  uint32_t thp = theta - (uint32_t)(FMX_RDS_DECIM - 1 - o0) * dtheta;
  int nsym = 0; // symbols of this call (k_bits decodes them)
  float last_symi = 0.0f;
  float *symrow = a.sym + (size_t)(act ? c : 0) * a.sym_stride;
  // input: the channel rows of this workgroup, sample t of the lane's channel
  // at inb[g * stride + t]; the lane takes the period's positions 3 j0 .. 3 j0
  // + 2 (round 5: contiguous); samples outside [0, count) read the row's
  // first word (every use masks them: vq below).  Each round's three samples
  // per lane are moved by LDS-DMA into the ring L.xin, RDS_PF rounds ahead,
  // and read back when the round runs: the wave's only vector-memory loads,
  // so a counted s_waitcnt finds them (round 3 rotated a register ring, and
  // the rotation waited for the loads of the round before: one memory
  // latency per round)
  const float *inb = a.in + (size_t)c0 * a.in_stride;
  const uint32_t xin0 = lds_addr(&L.xin[0][0][0]);
  auto dma_round = [&](int r) __attribute__((always_inline)) {
    const int base = (r == 0) ? o0 - (FMX_RDS_DECIM - 1) : o0 + 1 + FMX_RDS_DECIM * (r - 1);
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int t = base + 3 * j0 + q;
      const bool v = act && r < R && t >= 0 && t < count;
      dma_dword(inb + (act ? g * a.in_stride : 0) + (v ? t : 0),
                xin0 + (uint32_t)(((r & (RDS_NR - 1)) * 3 + q) * 64 * 4));
    }
  };
  // ---- FUSED: the 240k -> 171k resampler inside (k_rs's MFMA tiles for the
  // wave's 8 channels, columns 8 .. 15 of a tile unused), produced ahead of
  // the round that reads them: tile T (outputs 16 T .. 16 T + 15 of the
  // call, the same schedule entries for every channel) when the latest round
  // position of the wave's channels reaches it.  The window of tile T + 1 is
  // in registers and that of tile T in LDS when tile T is computed (k_rs's
  // two-deep pipeline); the schedule entries two tiles ahead. ----
  RdsFusedLds &F = *reinterpret_cast<RdsFusedLds *>(rds_smem + RDS_FOFF);
  const FmxSched *fsched = nullptr;
  int fns = 0, fntile = 0, ft = 0, o0max = 0;
  FmxSched feC{}, feN{}, feNN{};
  float4 fwN[4];
  const int frr = lane & 15, fkk = lane >> 4, flc = lane >> 2, flq = lane & 3;
  const bool flcv = flc < RDS_CPW && c0 + flc < a.C;
  const float *fmrow = nullptr, *fwrow = nullptr;
  auto f_load_e = [&](int T) __attribute__((always_inline)) { return fsched[min(16 * T + frr, fns - 1)]; };
  if (FUSED) {
    rs_fill_tab(F.tab, D, lane, 64);
    const int fg = a.group[c0];
    fsched = a.sched + (size_t)fg * a.sched_stride;
    fns = a.sched_n[fg];
    fntile = (fns + 15) / 16;
    const int fch = flcv ? c0 + flc : c0;
    fmrow = a.mpx + (size_t)fch * a.mpx_stride;
    fwrow = a.win + (size_t)fch * 32 + 32;
    o0max = o0;
    for (int d = 32; d >= 1; d >>= 1) o0max = max(o0max, __shfl_xor(o0max, d));
    feC = f_load_e(0);
    feN = f_load_e(1);
    feNN = f_load_e(2);
    float4 w0[4];
    rs_load_w(fmrow, fwrow, flcv, a.n, flq, rs_tile_k0(feC), w0);
    if (flc < RDS_CPW) rs_store_w(F.xs[0][flc], flcv, a.n, flq, rs_tile_k0(feC), w0);
    rs_load_w(fmrow, fwrow, flcv, a.n, flq, rs_tile_k0(feN), fwN);
  }
  auto produce = [&]() __attribute__((always_inline)) {
    float4 wNN[4];
    rs_load_w(fmrow, fwrow, flcv, a.n, flq, rs_tile_k0(feNN), wNN); // tile ft + 2
    const rs_f32x4 acc = rs_tile(F.tab, F.xs[ft & 1][frr & (RDS_CPW - 1)], feC, fkk);
    if (frr < RDS_CPW)
      *reinterpret_cast<float4 *>(&F.rsr[frr][(16 * ft + 4 * fkk) & (RDS_RSR - 1)]) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    if (flc < RDS_CPW) rs_store_w(F.xs[(ft + 1) & 1][flc], flcv, a.n, flq, rs_tile_k0(feN), fwN); // tile ft + 1
#pragma unroll
    for (int j = 0; j < 4; ++j) fwN[j] = wNN[j];
    feC = feN;
    feN = feNN;
    feNN = f_load_e(ft + 3);
    ++ft;
  };
  if (!FUSED) {
#pragma unroll
    for (int p = 0; p < RDS_PF; ++p) dma_round(p);
  }
  __syncthreads(); // LDS tables and per-channel state written
  int ckp = 0; // checkpoint slot of round r: r % FMX_RDS_CK
  // the lane's tap columns: the first FMX_RDS_HREG held in registers for
  // the whole call, the others read from LDS every round
  float hr[FMX_RDS_NACC][3];
#pragma unroll
  for (int i = 0; i < FMX_RDS_HREG; ++i) {
    const float4 h = *reinterpret_cast<const float4 *>(&L.hq[j0][i][0]);
    hr[i][0] = h.x;
    hr[i][1] = h.y;
    hr[i][2] = h.z;
  }
  RDS_STAMP(0)
  for (int r = 0; r < rmax; ++r) {
    float xr0[3];
    if (FUSED) {
      // the wave's latest sample this round: o0 + 24 r of its latest channel
      const int eneed = min((r == 0) ? o0max : o0max + FMX_RDS_DECIM * r, fns - 1);
      while (ft < fntile && 16 * ft <= eneed) produce();
      const int fbase = (r == 0) ? o0 - (FMX_RDS_DECIM - 1) : o0 + 1 + FMX_RDS_DECIM * (r - 1);
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int t = fbase + 3 * j0 + q;
        xr0[q] = F.rsr[g][t & (RDS_RSR - 1)]; // t outside [0, count) is masked below (vq)
      }
    } else {
      dma_round(r + RDS_PF);
      // the moves of rounds r + 1 .. r + RDS_PF may stay in flight (anything
      // the compiler issued after them only makes the wait stricter)
      // vmcnt(3 RDS_PF) (its bits 3:0 and 15:14), lgkmcnt / expcnt untouched
      __builtin_amdgcn_s_waitcnt(0x0F70 | ((3 * RDS_PF) & 15) | (((3 * RDS_PF) >> 4) << 14));
#pragma unroll
      for (int q = 0; q < 3; ++q) xr0[q] = L.xin[r & (RDS_NR - 1)][q][lane];
    }
    // this lane's tap columns for the FIR products below: all eleven reads
    // issued here, ahead of the mix-down, which hides their latency (round 4
    // interleaved one read per accumulator with its packed FMAs: eleven LDS
    // latencies per round); the scheduling barrier keeps them together, so
    // none lands over the sources of a packed op (tests/test_isa_scan.py)
#pragma unroll
    for (int i = FMX_RDS_HREG; i < FMX_RDS_NACC; ++i) {
      const float4 h = *reinterpret_cast<const float4 *>(&L.hq[j0][i][0]);
      hr[i][0] = h.x;
      hr[i][1] = h.y;
      hr[i][2] = h.z;
    }
    __builtin_amdgcn_sched_barrier(0);
    RDS_STAMP(1)
    const bool live = r < R;
    const int base = (r == 0) ? o0 - (FMX_RDS_DECIM - 1) : o0 + 1 + FMX_RDS_DECIM * (r - 1);
    // this round's NCO words (the checkpoint a ring refill mixes with)
    if (lead && live) *reinterpret_cast<uint2 *>(&L.ck[g][ckp][0]) = make_uint2(thp, dtheta);
    ckp = (ckp == FMX_RDS_CK - 1) ? 0 : ckp + 1;
    // ---- mix-down and FIR products of this lane's samples (oldest first) ----
    f32x2 mq[3];
    bool vq[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int j = 3 * j0 + q;
      const int t = base + j;
      vq[q] = live && t >= 0 && t < count;
      const uint32_t w = thp + (uint32_t)j * dtheta;
      // samples outside the call contribute nothing (their input reads 0)
      mq[q] = vq[q] ? rds_mix(xr0[q], w) : f32x2{0.0f, 0.0f};
      if (ringw && vq[q] && t >= count - FMX_RDS_RING) {
        const uint32_t idx = (ring0 + (uint32_t)t) & (FMX_RDS_RING - 1);
        *reinterpret_cast<f32x2 *>(ring + 2 * idx) = mq[q];
      }
    }
    RDS_STAMP(2)
    if (live) {
#pragma unroll
      for (int i = 0; i < FMX_RDS_NACC; ++i) {
        // the lane's samples oldest first, as the window dot product (a
        // sample outside the call is 0 and adds +0)
        acc[i] = __builtin_elementwise_fma(f32x2{hr[i][0], hr[i][0]}, mq[0], acc[i]);
        acc[i] = __builtin_elementwise_fma(f32x2{hr[i][1], hr[i][1]}, mq[1], acc[i]);
        acc[i] = __builtin_elementwise_fma(f32x2{hr[i][2], hr[i][2]}, mq[2], acc[i]);
      }
    }
    RDS_STAMP(3)
    const bool has_out = live && base + FMX_RDS_DECIM - 1 < count;
    if (has_out) {
      // ---- FIR output (every 24th sample) -> AGC -> symsync -> PSK2 PLL ----
      const f32x2 f = rds_sum8x2(acc[0].x, acc[0].y) * fscale2;
#pragma unroll
      for (int i = 0; i < FMX_RDS_NACC - 1; ++i) acc[i] = acc[i + 1];
      acc[FMX_RDS_NACC - 1] = f32x2{0.0f, 0.0f};
      const float yr = f.x * agc_g, yi = f.y * agc_g;
      const float y2 = yr * yr + yi * yi;
      agc_y2p = (float)((1.0 - (double)agc_bw) * (double)agc_y2p + (double)(agc_bw * y2));
      if (agc_y2p > 1e-6f) agc_g *= expf(-0.5f * agc_bw * logf(agc_y2p));
      if (agc_g > 1e6f) agc_g = 1e6f;
      RDS_STAMP(4)
      // ---- symsync: push into both MF banks' window ----
      wp = (wp == FMX_SS_SUB - 1) ? 0 : wp + 1;
      if (lead) L.win[wp][g] = L.win[wp + FMX_SS_SUB][g] = f32x2{yr, yi};
      if (ss_valid < FMX_SS_SUB) ss_valid++;
      const int w0 = (wp == FMX_SS_SUB - 1) ? 0 : wp + 1; // oldest
      auto wat = [&](int m) __attribute__((always_inline)) {
        const int i = w0 + m;
        return L.win[i][g];
      };
      int ns = 0;
      f32x2 sym = f32x2{0.0f, 0.0f};
      while (ss_b < FMX_NPFB && ns < 16) {
        const float *hm = L.mf + ss_b * FMX_SS_SUB;
        // the 18-tap matched filter split over the channel's 8 lanes (taps
        // m = j0, j0 + 8, j0 + 16), summed by the DPP butterfly: every lane
        // holds the same total (a tree instead of the reference's sequential
        // sum: a few ulp)
        auto mf_dot = [&](const float *hb) __attribute__((always_inline)) {
          f32x2 p = f32x2{0.0f, 0.0f};
#pragma unroll
          for (int u = 0; u < 3; ++u) {
            const int m = j0 + 8 * u;
            if (u < 2 || m < FMX_SS_SUB) {
              const float h = hb[FMX_SS_SUB - 1 - m];
              p = __builtin_elementwise_fma(f32x2{h, h}, wat(m), p);
            }
          }
          return rds_sum8x2(p.x, p.y);
        };
        const f32x2 acm = mf_dot(hm);
        // x / 3 as fmx_div_const (bit-identical for every normal x,
        // tests/golden/divconst_exhaustive.json), the zero's sign restored
        if (ns == 0)
          sym = f32x2{copysignf(fmx_div_const(acm.x, 3.0f, 1.0f / 3.0f), acm.x),
                      copysignf(fmx_div_const(acm.y, 3.0f, 1.0f / 3.0f), acm.y)};
        if (ss_decim == 1) {
          ss_decim = 0;
          const float *hd = L.dmf + ss_b * FMX_SS_SUB;
          const f32x2 acd = mf_dot(hd);
          float qe = acm.x * acd.x + acm.y * acd.y;
          if (qe > 1.0f) qe = 1.0f;
          else if (qe < -1.0f) qe = -1.0f;
          const float t1 = ss_a1 * ss_v1;
          const float v0 = qe - t1;
          ss_q_hat = ss_b0 * v0;
          ss_v1 = v0;
          ss_rate += ss_adj * ss_q_hat;
          ss_del = ss_rate + ss_q_hat;
        }
        ss_decim++;
        ss_tau += ss_del;
        ss_b = (int)roundf(ss_tau * (float)FMX_NPFB);
        ns++;
      }
      ss_tau -= 1.0f;
      ss_b -= FMX_NPFB;
      RDS_STAMP(5)
      // the NCO word of the instant's sample; step() follows the PLL update
      uint32_t tho = thp + (uint32_t)(FMX_RDS_DECIM - 1) * dtheta;
      if (ns == 1) {
        // ---- PSK2 modem phase error -> NCO PLL ----
        const float symr = sym.x, symi = sym.y;
        // modem_demodulate (PSK2): th = atan2(symi, symr) - pi/2, wrapped
        // below -pi; symbol 1 iff th > 0, i.e. iff the symbol lies left of
        // the imaginary axis.  Away from the axis (|symr| > 1e-5 |symi|:
        // the angle is >= 1e-5 from +-pi/2, far beyond atan2f's error) the
        // sign of symr decides; on it the reference's arithmetic does
        bool s1 = symr < 0.0f;
        if (!(fabsf(symr) > 1e-5f * fabsf(symi))) {
          float th = atan2f(symi, symr) - dphi_psk;
          if ((double)th < -3.14159265358979323846) th = (float)((double)th + 2.0 * 3.14159265358979323846);
          s1 = th > 0.0f;
        }
        const float xr = s1 ? psk_xr1 : 1.0f, xi = s1 ? psk_xi1 : 0.0f;
        float pe = symi * xr - symr * xi;
        pe = d_clamp(pe, -kPiF, kPiF);
        const float dphi = pe * 12.0f;
        dtheta += d_nco_constrain(dphi * alpha);
        tho += d_nco_constrain(dphi * beta);
        // biphase / delta / block sync only consume symbols: they go to
        // HBM and k_bits decodes them (one lane per channel, round 5: the
        // decoders ran in each channel's first lane here, 8 of 64 lanes,
        // ~14 % of this kernel's serial time, profiles/r05i_stamps.txt)
        if (lead && act && nsym < a.sym_stride) symrow[nsym] = symr;
        last_symi = symi;
        nsym++;
      }
      thp = tho + dtheta; // period position 0 of the next round
    } else if (live) {
      // tail: samples base .. count-1 stepped, no decimation instant
      thp = thp + (uint32_t)(count - base) * dtheta;
    }
    RDS_STAMP(6)
  }
  // the channel's partial sums: the lanes' shares added (every lane gets them)
#pragma unroll
  for (int i = 0; i < FMX_RDS_NACC; ++i) acc[i] = rds_sum8x2(acc[i].x, acc[i].y);
  if (!act || !lead) return;
  // ---- registers -> state ----
  FmxRdsState *out = a.st + c;
  // the NCO word of the next sample: after a decimation instant thp is the
  // next period's position 0, after a tail (period start + tail length)
  out->theta = (R > 0) ? thp : theta;
  out->dtheta = dtheta;
  // the wrapper's phases as the reference would hold them (= the NCO phase)
  out->prev_f0 = d_nco_phase(theta);
  out->phase0 = d_unwrap(d_nco_phase(theta));
  out->sample_since_reset = ssr0 + (uint32_t)count;
  out->ring_pos = ring0 + (uint32_t)count;
  out->rebuild = 0;
  if (!ringw) { // the last rounds' words, oldest first (rds_ring_fill)
    const int first = R > FMX_RDS_CK ? R - FMX_RDS_CK : 0;
    int slot = first % FMX_RDS_CK;
    for (int i = 0; i < min(R, FMX_RDS_CK); ++i) {
      out->ck_thp[i] = L.ck[g][slot][0];
      out->ck_dth[i] = L.ck[g][slot][1];
      slot = (slot == FMX_RDS_CK - 1) ? 0 : slot + 1;
    }
    out->ck_o0 = o0;
    out->ck_rounds = R;
    out->ck_count = count;
    out->ring_ok = 0;
  } else if (count > 0) {
    out->ring_ok = 1;
  }
  for (int i = 0; i < FMX_RDS_NACC; ++i) {
    out->acc_re[i] = acc[i].x;
    out->acc_im[i] = acc[i].y;
  }
  out->agc_g = agc_g;
  out->agc_y2p = agc_y2p;
  for (int m = 0; m < FMX_SS_SUB; ++m) {
    const int i = wp + 1 + m;
    const f32x2 w = L.win[i][g];
    out->ss_win_re[m] = w.x;
    out->ss_win_im[m] = w.y;
  }
  out->ss_mf_valid = ss_valid;
  out->ss_rate = ss_rate;
  out->ss_del = ss_del;
  out->ss_tau = ss_tau;
  out->ss_q_hat = ss_q_hat;
  out->ss_v1 = ss_v1;
  out->ss_v2 = G.ss_v2;
  out->ss_b = ss_b;
  out->ss_decim = ss_decim;
  a.sym_count[c] = min(nsym, a.sym_stride);
  a.sym_last_im[c] = last_symi;
  RDS_STAMP(0)
#ifdef FMX_STAMPS
  if (a.dbg && lane == 0)
    for (int k = 0; k < 8; ++k) atomicAdd(a.dbg + k, rs_acc[k]);
#endif
#undef RDS_STAMP
}

// k_bits (round 5): the RDS bit decoders of one call -- BiphaseDecoder::push
// (subcarrier.cpp:50-86), DeltaDecoder (:88-92) and BlockStream::pushBit /
// Group (block_sync.cpp:235-313, group.cpp:103-128) -- over the symbols
// k_rds wrote, one lane per channel (64 channels per wave instead of k_rds's
// 8 first lanes), on the RDS stream right after k_rds.
__global__ __launch_bounds__(64) void k_bits(RdsArgs a) {
  extern __shared__ __align__(16) unsigned char bits_smem[];
  BitsLds &L = *reinterpret_cast<BitsLds *>(bits_smem);
  const int lane = threadIdx.x;
  const int c = blockIdx.x * 64 + lane;
  const bool act = c < a.C;
  // burst-error syndromes per offset word: entry idx < 26 a single-bit error
  // at bit idx, idx >= 26 a two-bit burst at bit idx - 26 (all lanes)
  for (int k = lane; k < 5 * 52; k += 64) {
    const int w = k / 52, idx = k % 52;
    const uint32_t word = w == 0 ? 0x0FCu : w == 1 ? 0x198u : w == 2 ? 0x168u : w == 3 ? 0x350u : 0x1B4u;
    const uint32_t bits = idx < 26 ? 1u : 3u, sh = idx < 26 ? idx : idx - 26;
    const uint32_t e = (bits << sh) & ((1u << 26) - 1u);
    L.esyn[w][idx] = bs_syndrome(e ^ word);
    L.eerr[w][idx] = e;
  }
  __syncthreads();
  if (!act) return;
  RdsBits S; // in registers
  rds_bits_load(S, a.st[c]);
  const int nsym = a.sym_count[c];
  // the symbols four at a time, the next four loaded while these decode (a
  // dependent load per symbol cost a memory latency each)
  const float4 *srow = reinterpret_cast<const float4 *>(a.sym + (size_t)c * a.sym_stride);
  const int nq4 = a.sym_stride / 4;
  float4 nx = nsym > 0 ? srow[0] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  int ng = 0;
  for (int k0 = 0; k0 < nsym; k0 += 4) {
    // this chunk in four scalars (the chunk shifts down one symbol per step:
    // no indexing, no scratch), the next one loading meanwhile
    float q0 = nx.x, q1 = nx.y, q2 = nx.z, q3 = nx.w;
    if (k0 + 4 < nsym && k0 / 4 + 1 < nq4) nx = srow[k0 / 4 + 1];
    const int nj = min(4, nsym - k0);
#pragma unroll 1
    for (int j = 0; j < nj; ++j) {
      const float symr = q0;
      q0 = q1;
      q1 = q2;
      q2 = q3;
      const float bir = (symr - S.bi_prev_re) * 0.5f;
      const int val = bir >= 0.0f;
      const bool has = (S.bi_clock % 2u) == S.bi_polarity;
      S.bi_prev_re = symr;
      if ((S.bi_clock & 1u) == 0) S.bi_even += fabsf(bir);
      else S.bi_odd += fabsf(bir);
      S.bi_clock++;
      if (S.bi_clock == 128u) {
        if (S.bi_even > S.bi_odd) S.bi_polarity = 0;
        else if (S.bi_odd > S.bi_even) S.bi_polarity = 1;
        S.bi_even = 0.0f;
        S.bi_odd = 0.0f;
        S.bi_clock = 0;
      }
      if (has) {
        const int bit = (val != S.delta_prev) ? 1 : 0;
        S.delta_prev = val;
        rds_push_bit(S, bit, L, a, c, ng);
      }
    }
  }
  if (nsym > 0) S.bi_prev_im = a.sym_last_im[c];
  rds_bits_store(a.st[c], S);
  if (a.group_count) a.group_count[c] = ng;
}

/* ================================================================== */
/* state reset / construction                                          */
/* ================================================================== */
// One channel's reset, the parts selected by `parts` (ResetStreamPart): each
// part touches only state that the kernels of ONE stream of process_block
// read or write, so process_block runs it on that stream right before that
// stream's kernel of the step (no cross-stream join, round 5); st_buf: the
// stereo history buffer the step reads (-1: all of them, the joined path).
__device__ void reset_channel(const ResetArgs &a, int c, int m, int parts, int st_buf) {
  const int tid = threadIdx.x;
  const FmxDesign *D = a.des;
  const bool create = m & RS_CREATE;
  if (parts & RSP_FRONT) { // sA: k_fe8 / k_frontend / k_pilot state
    if (create || (m & RS_DECIM)) {
      if (tid == 0) a.dec_valid[c] = 0;
    }
    if (create || (m & (RS_DEMOD | RS_IQFIR))) {
      for (int h = tid; h < FMX_IQ_MAXLEN - 1; h += blockDim.x)
        a.iq_hist[(size_t)c * (FMX_IQ_MAXLEN - 1) + h] = float2_t{0.0f, 0.0f};
    }
    if (tid == 0 && (create || (m & (RS_FREQDEM | RS_DEMOD)))) { // freqdem re-created / reset: r_prev = 0
      a.fd_prev[2 * c] = 0.0f;
      a.fd_prev[2 * c + 1] = 0.0f;
    }
    if (tid == 0 && (create || (m & RS_DEMOD))) {
      a.dc_v[2 * c] = 0.0f;
      a.dc_v[2 * c + 1] = 0.0f;
    }
    if (tid == 0 && (create || (m & RS_AGC))) {
      a.agc[2 * c] = 1.0f;
      a.agc[2 * c + 1] = 1.0f;
    }
    if (create || (m & RS_STEREO)) { // the pilot BPF window / delay line (the previous call's MPX rows)
      for (int h = tid; h < FMX_HIST; h += blockDim.x)
        for (int k = 0; k < FMX_ST_BUFS; ++k)
          if (st_buf < 0 || k == st_buf) a.st_hist[((size_t)k * a.C + c) * FMX_HIST + h] = 0.0f;
    }
    if (create) // the RDS resampler's window (k_fe8 hands it on): a new object only, as the reference
      for (int h = tid; h < 32; h += blockDim.x) a.rds_hist[(size_t)c * 32 + h] = 0.0f;
  }
  if ((parts & RSP_STEREO) && tid == 0 && (create || (m & RS_STEREO))) { // sB: k_pll
    FmxStereoState s{};
    s.theta = 0;
    s.dtheta = D->pll_dtheta0;
    s.pll_freq = D->nominal;
    a.st[c] = s;
  }
  // FmxRdsState in two parts by owner: k_rds's (the fields before
  // bi_prev_re, on sC) and k_bits's (bi_prev_re on, on sD, round 5); each part
  // writes only its own dwords, so a reset on one stream never rewrites the
  // other kernel's fields while that kernel may run
  constexpr int kBitsW = (int)(offsetof(FmxRdsState, bi_prev_re) / 4), kRdsW = (int)(sizeof(FmxRdsState) / 4);
  static_assert(offsetof(FmxRdsState, bi_prev_re) % 4 == 0 && sizeof(FmxRdsState) % 4 == 0, "FmxRdsState parts");
  if ((parts & RSP_RDS) && (create || (m & RS_RDS))) { // sC: k_rds
    // the rebuild reads the ring: refilled first if the last call left
    // checkpoints instead (round 6; every thread reads the state before
    // thread 0 rewrites it)
    if (!create) {
      if (!a.rds[c].ring_ok && a.rds_prev != nullptr)
        rds_ring_fill(a.rds + c, a.rds_prev + (size_t)c * a.rds_stride, a.ring + (size_t)c * 2 * FMX_RDS_RING, tid,
                      blockDim.x);
      __syncthreads();
    }
    if (tid == 0) {
      FmxRdsState s;
      if (create) {
        s = FmxRdsState{};
        s.agc_g = D->agc_g0;
        s.agc_y2p = 1.0f;
        s.rebuild = 0;
      } else {
        s = a.rds[c]; // (the bit decoders' dwords are read but not written back)
        s.rebuild = 1;
      }
      s.ring_ok = 1; // zeroed at creation, refilled above
      s.theta = 0;
      s.dtheta = D->rds_dtheta0;
      s.sample_since_reset = 0;
      // symsync reset (matched filter bank only): firpfb_crcf_reset clears
      // the shared MF / dMF window
      s.ss_mf_valid = 0;
      for (int m = 0; m < FMX_SS_SUB; ++m) {
        s.ss_win_re[m] = 0.0f;
        s.ss_win_im[m] = 0.0f;
      }
      s.ss_rate = 3.0f;
      s.ss_del = 3.0f;
      s.ss_tau = 0.0f;
      s.ss_b = 0;
      s.ss_q_hat = 0.0f;
      s.ss_v1 = 0.0f;
      s.ss_v2 = 0.0f;
      s.ss_decim = 0;
      const uint32_t *src = reinterpret_cast<const uint32_t *>(&s);
      uint32_t *dst = reinterpret_cast<uint32_t *>(a.rds + c);
      for (int w = 0; w < kBitsW; ++w) dst[w] = src[w];
    }
    if (create)
      for (int h = tid; h < 2 * FMX_RDS_RING; h += blockDim.x) a.ring[(size_t)c * 2 * FMX_RDS_RING + h] = 0.0f;
  }
  if ((parts & RSP_BITS) && tid == 0 && (create || (m & RS_RDS))) { // sD: k_bits
    FmxRdsState s;
    if (create) s = FmxRdsState{}; // biphase / delta decoders from zero
    else s = a.rds[c];
    // fresh BlockStream
    s.bs_bitcount = 0;
    s.bs_until_next = 1;
    s.bs_reg = 0;
    s.bs_err_mask_lo = 0;
    s.bs_err_mask_hi = 0;
    s.bs_expected = OA;
    s.bs_in_sync = 0;
    s.bs_err_ptr = 0;
    for (int i = 0; i < 4; ++i) {
      s.bs_pulse_pos[i] = 0;
      s.bs_pulse_off[i] = OINV;
      s.bs_blk_raw[i] = 0;
      s.bs_blk_data[i] = 0;
      s.bs_blk_flags[i] = 0;
    }
    s.bs_bits_since_lost = 0;
    const uint32_t *src = reinterpret_cast<const uint32_t *>(&s);
    uint32_t *dst = reinterpret_cast<uint32_t *>(a.rds + c);
    for (int w = kBitsW; w < kRdsW; ++w) dst[w] = src[w];
  }
  if (parts & RSP_AUDIO) { // sD: k_audio (L/R FIRs, AF post, mono chain, retune mute)
    if (create || (m & RS_STEREO))
      for (int h = tid; h < 2 * (FMX_LR_LEN - 1); h += blockDim.x) a.lr_hist[(size_t)c * 2 * (FMX_LR_LEN - 1) + h] = 0.0f;
    if (create || (m & RS_DEMOD)) {
      if (tid == 0) {
        a.mono_iir[2 * c] = 0.0f;
        a.mono_iir[2 * c + 1] = 0.0f;
      }
      for (int h = tid; h < 32; h += blockDim.x) a.mono_win[(size_t)c * 32 + h] = 0.0f;
    }
    if (create || (m & RS_AF)) {
      for (int h = tid; h < 64; h += blockDim.x) a.af_win[(size_t)c * 64 + h] = 0.0f;
      if (tid < 4) a.af_iir[(size_t)c * 4 + tid] = 0.0f;
    }
    if (tid == 0 && (m & RS_DEEMPH)) {
      a.af_iir[(size_t)c * 4 + 0] = 0.0f;
      a.af_iir[(size_t)c * 4 + 1] = 0.0f;
      a.mono_iir[2 * c] = 0.0f;
    }
    // retune fade/mute (main.cpp:1034-1035): remaining = total = mute length
    if (tid == 0 && (create || (m & RS_MUTE))) {
      const int len = (m & RS_MUTE) ? (int)((uint32_t)m >> 16) : 0;
      a.mute[2 * c] = len;
      a.mute[2 * c + 1] = len;
    }
  }
}
// every part of every channel with a nonzero mask (the joined path: creation,
// stage entry points, resets of many channels at once)
__global__ void k_reset(ResetArgs a) {
  const int c = blockIdx.x;
  const int m = a.mask[c];
  if (m != 0) reset_channel(a, c, m, RSP_ALL, -1);
}
// the listed channels, one part (process_block: on that part's stream)
__global__ void k_reset_list(ResetArgs a, ResetList L, int parts, int st_buf) {
  const int i = blockIdx.x;
  if (i < L.n) reset_channel(a, L.ch[i], L.m[i], parts, st_buf);
}

/* ComplexDecimator::execute's requantisation (liquid_primitives.cpp:448-452):
 * clamp(y * 127.5 + 127.5, 0, 255) truncated to u8, for C rows of n complex
 * outputs (separate multiply and add: the file builds with fp-contract off) */
__global__ void k_iq_to_u8(const float *in, int in_stride, int n, uint8_t *out, size_t out_stride) {
  const int c = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float yr = in[(size_t)c * in_stride + 2 * i], yi = in[(size_t)c * in_stride + 2 * i + 1];
  const float ir = d_clamp((yr * 127.5f) + 127.5f, 0.0f, 255.0f);
  const float qr = d_clamp((yi * 127.5f) + 127.5f, 0.0f, 255.0f);
  out[(size_t)c * out_stride + 2 * i] = (uint8_t)ir;
  out[(size_t)c * out_stride + 2 * i + 1] = (uint8_t)qr;
}

/* ================================================================== */
/* synthetic IQ generator                                              */
/* ================================================================== */
__global__ void k_synth(fmx_synth_config cfg, uint32_t ch0, int n_ch, int64_t sample0, int n_samples,
                        const uint8_t *bits, uint8_t *out, size_t out_stride) {
  const int ci = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (ci >= n_ch || i >= n_samples) return;
  const uint32_t ch = ch0 + (uint32_t)ci;
  const fmx_synth_chan cp = fmx_synth_channel(&cfg, ch);
  const uint8_t *b = bits ? bits + (size_t)ci * cfg.n_bits : nullptr;
  uint8_t iq[2];
  fmx_synth_sample(&cfg, ch, &cp, sample0 + i, b, iq);
  uint16_t w = (uint16_t)iq[0] | ((uint16_t)iq[1] << 8);
  reinterpret_cast<uint16_t *>(out + (size_t)ci * out_stride)[i] = w;
}

/* ================================================================== */
/* k_fe8: the steady-state frontend, 8 consecutive outputs per thread  */
/* ================================================================== */
/* The VEC path of k_frontend (u8 IQ, full decimator history) for calls of
 * whole FE8_T-sample chunks -- every fmx_process_block call of a running
 * receiver and of the bench.  Same stages and per-output arithmetic; each
 * thread owns 8 consecutive DSP samples, so every input sample it reads
 * feeds 8 outputs:
 *   decimator     one 16-B LDS read = 8 IQ samples -> up to 64 packed (I,Q)
 *                 FMAs; the window is fully unrolled, zero taps never issued
 *   DC blockers   8-element affine maps per thread, block scan, recompute
 *   IQ FIR        complex: 1 ds_read_b64 per input -> 8 packed FMAs
 *   pilot BPF     1 ds_read_b32 per input -> 4 packed FMAs (output pairs)
 *   RDS resampler packed (branch, next branch) chain on the MPX image
 * The IQ and MPX images in LDS are padded (element i at i + i/8): lanes 8
 * elements apart read distinct banks.  The complex IQ image and the IQ FIR
 * output alias the u8 input chunk (dead once the decimator's outputs are in
 * registers); only the 120-sample IQ FIR history is carried separately.
 * ~58 KB of LDS per workgroup: two workgroups (8 waves) per CU leave room
 * for a k_pll or k_rds workgroup beside them. */
#define FE8_T 2048
#define FE8_MIN_N 1024 // config.cpp:240 clamps dsp_block_samples to 1024..32768
#ifndef FMX_DEC_UNROLL
#define FMX_DEC_UNROLL 1
#endif
__host__ __device__ constexpr int fe8_i(int i) { return i + (i >> 3); }
// Decimator staging (k_fe8): output o as float2 at o + 2 (o / 32), i.e. one
// 16-B pad per 16 float4 pairs.  The transposed MFMA tiles write 16
// consecutive outputs per 16-lane ds_write_b64 group (conflict-free either
// way); each thread then reads its 8 consecutive outputs as four b128 pairs,
// 64 B apart across the lanes -- 4-way on the 256-B bank row unpadded,
// conflict-free padded (tools/lds_banks.py, the guide's lane groups).
__device__ __forceinline__ int fe8_stg(int o) { return o + 2 * (o >> 5); }
typedef __attribute__((address_space(3))) float lds_f32;
typedef __attribute__((address_space(3))) f32x2 lds_f32x2;

// RS: the RDS resampler runs in k_fe8 (its pair bank in LDS); without it
// (k_rs resamples) the layout is 7 KB smaller
template <int M, int TPP, bool RS = true> struct Fe8Layout {
  static constexpr int L = M * TPP;
  static constexpr int G = (7 * M + L + 1 + 7) / 8;                 // 8-sample groups per thread window
  static constexpr int HB = 2 * L;                                   // halo bytes (L samples)
  static constexpr int RAW_BYTES = HB + 2 * FE8_T * M + 16;
  static constexpr int YB_BYTES = (FE8_T + 1) * 8;
  static constexpr int XN = (FE_HALO_IQ + FE8_T + 16) * 9 / 8 + 8;   // padded complex image
  static constexpr int XIN = 0;                                      // aliases raw
  // FMX_IQ_MFMA: the IQ FIR input instead of the complex image, as f16 hi / lo
  // images of I and Q (x 2^10; history + chunk + zero slack) from XIN
  static constexpr int IQW = FE_HALO_IQ + FE8_T + 32;
  static constexpr int YB = XN * 8;                                  // aliases raw
  static constexpr int NPC = (HB + 2 * FE8_T * M + 1023) / 1024;     // 1-KiB LDS-DMA pieces per chunk
  static constexpr int RAW_ALLOC = NPC * 1024 > RAW_BYTES ? NPC * 1024 : RAW_BYTES;
  static constexpr int R0 = ((RAW_ALLOC > YB + YB_BYTES ? RAW_ALLOC : YB + YB_BYTES) + 15) & ~15;
  // unpadded MPX copy for the RDS resampler (32 history + chunk + 32 slack),
  // at the top of the raw region: the pieces below it are the next chunk's
  // early DMA (during pilot / RDS), the pieces over it the late DMA
  static constexpr int U_FLOATS = 32 + FE8_T + 32;
  static constexpr int UOFF = (R0 - U_FLOATS * 4) & ~15;
  static constexpr int NPC_EARLY = UOFF / 1024 < NPC ? UOFF / 1024 : NPC;
  static constexpr int HX = R0;                                      // IQ FIR history (FE_HALO_IQ)
  // MPX for the MFMA pilot BPF as f16 hi / lo images (history + chunk +
  // zero slack, natural order), the chunk's last FMX_HIST samples in f32
  // (stereo history write-back) and the previous chunk's last 32 in f32
  // (the RDS resampler's window)
  // (RS = false, process_block's variant, runs no pilot BPF -- k_pilot does
  // -- and has no images: 10.4 KB less)
  static constexpr int XW = RS ? FMX_HIST + FE8_T + 32 : 0;
  static constexpr int MX = HX + FE_HALO_IQ * 8;                     // XH: f16 hi [XW]
  static constexpr int XLO = MX + XW * 2;                            // XL: f16 lo [XW]
  // (round 3: no f32 copy of the chunk's last FMX_HIST samples -- the call's
  // last ones go straight to the history rows in HBM -- so that two k_fe8
  // workgroups and a k_pll workgroup fit one CU's 160 KB)
  static constexpr int TL32 = (XLO + XW * 2 + 15) & ~15;             // f32 [32]
  static constexpr int RS_PAIRS = FMX_NPFB + 1;                      // branch pairs (b, b+1), + the boundary pair
  static constexpr int RS_M = FMX_RDS_RS_SUB + 1;                    // 27 terms (leading / trailing zero)
  static constexpr int RST = (TL32 + 32 * 4 + 15) & ~15;             // RDS resampler bank [33][27] float2
  static constexpr int SG = (RST + (RS ? RS_PAIRS * RS_M * 8 : 0) + 15) & ~15;
  static constexpr int SH = SG + 4 * 6 * 8;
  // RS = false (process_block's variant, round 6): the decimator's tap
  // window FmxDesign::dec_q16 (hi, lo: QN entries each) in LDS, read as the
  // A fragments instead of dec_frag from L2 (RS = true keeps dec_frag: no
  // LDS to spare beside its images and resampler bank)
  // Both windows arrive by LDS-DMA behind the first chunk's (whole 64-dword
  // pieces: QDP, QIP; the pad past each window takes copies of its last dword)
  static constexpr int KS = (15 * M + L + 1 + 31) / 32;
  static constexpr int QN = 15 * M + 32 * KS;                        // window entries the K steps reach
  static constexpr int QDP = (FMX_DEC_QN + 63) / 64;                 // [2][FMX_DEC_QN] u16 = FMX_DEC_QN dwords
  static constexpr int QT = (SH + (int)sizeof(FeShared) + 15) & ~15;
  // and the channel's IQ FIR design's window FmxDesign::iq_q16 [2][2][FMX_IQ_QN]
  static constexpr int QIP = (2 * FMX_IQ_QN + 63) / 64;              // 2 FMX_IQ_QN dwords
  static constexpr int QI = QT + (RS ? 0 : QDP * 256);
  // RS = false (round 6): the channel's carried words and decimator history
  // land here by LDS-DMA with the first chunk (1 KB: dwords 0..63 the words,
  // 64..255 the history bytes), so the setup waits on no load
  static constexpr int SU = QI + (RS ? 0 : QIP * 256);
  static constexpr int SU_H = 64;                                    // history dwords from here
  static constexpr int BYTES = SU + (RS ? 0 : 1024);
  static_assert(RS || 2 * (L - 1) <= 4 * (256 - SU_H), "decimator history inside the landing area");
  // (the IQ FIR history lands in hx as 4 x 64 dwords: the 16 past it in tl32,
  // which RS = false does not use)
  static_assert(RS || HX + 1024 <= TL32 + 32 * 4, "IQ FIR history DMA inside hx + tl32");
  static_assert(M % 2 == 0 && FMX_DEC_QN % 2 == 0 && QN <= FMX_DEC_QN, "dword-aligned fragment reads inside the window");
  static constexpr int NPF = (HB + 2 * FE8_T * M + 16 * 256 - 1) / (16 * 256); // 16-B pieces per thread
  // the MFMA decimator's outputs on their way to the 8-per-thread layout
  // (fe8_stg order), in the raw region once every wave has read it; read
  // back before the barrier after which the IQ images take the region
  static constexpr int STG = 0;
  static_assert(STG + (FE8_T + 2 * (FE8_T / 32)) * 8 <= R0, "decimator staging (padded, fe8_stg) inside the raw region");
  // LDS-DMA targets (determinism): the early pieces of
  // the next chunk land below uc while the RDS resampler reads uc; the late
  // pieces cover uc only after the barrier that ends its reads, and no piece
  // reaches the carried images, the resampler bank or the shared words
  static_assert(NPC_EARLY * 1024 <= UOFF, "early DMA pieces end below uc");
  static_assert(NPC * 1024 <= HX && HX <= MX && TL32 + 32 * 4 <= RST, "late DMA pieces end below the carried state");
  // two k_fe8 workgroups beside a 32 x 8 k_pll workgroup (39168 B): 163840 B per CU
  static_assert(M != 10 || 2 * BYTES + 39168 <= 163840, "two front ends and a k_pll workgroup per CU");
  static_assert(XIN + 4 * IQW * 2 <= YB && (IQW * 2) % 16 == 0 && (FE_HALO_IQ * 2) % 16 == 0,
                "IQ images below yb, 16-B aligned rows");
};

// The MFMA FIRs (IQ FIR, pilot BPF) run a P-tap filter as length P8 = P
// rounded up to 8k + 1 (up to 7 zero taps at the oldest end, same sums), so
// every K step starts on an 8-sample boundary.
__device__ __forceinline__ int fir8_len(int P) { return ((P + 6) & ~7) + 1; }
// register budget: two workgroups (8 waves) per CU beside a k_pll / k_rds /
// k_rs wave -- <= 168 VGPRs (3 waves per SIMD); M = 8 (the reference's
// 2.048 MS/s rate) keeps its longer decimator window at 2, and so does the
// RS = true instance (the resampler and the pilot BPF inside: stage entry
// points and RDS steps past k_rs's window, never process_block at 240 / 256
// kHz), which with round 5's per-channel cold start and any-n chunks no
// longer fits 168 without scratch
template <int M, int TPP, bool RS>
#ifndef FMX_FE_PRIO
#define FMX_FE_PRIO 0 // k_fe8's wave priority (s_setprio) beside the other streams' waves
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu((M == 8 || RS) ? 2 : 3))) void k_fe8(FeArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  using LY = Fe8Layout<M, TPP, RS>;
  if (FMX_FE_PRIO > 0) __builtin_amdgcn_s_setprio(FMX_FE_PRIO);
  constexpr int L = LY::L;
  uint8_t *raw = reinterpret_cast<uint8_t *>(smem);
  float2 *yb = reinterpret_cast<float2 *>(smem + LY::YB);
  float2 *hx = reinterpret_cast<float2 *>(smem + LY::HX);
  _Float16 *xh = reinterpret_cast<_Float16 *>(smem + LY::MX);  // MPX hi, index FMX_HIST + j
  _Float16 *xl = reinterpret_cast<_Float16 *>(smem + LY::XLO); // MPX lo
  float *tl32 = reinterpret_cast<float *>(smem + LY::TL32);     // the previous chunk's last 32
  f32x2(*rsb)[LY::RS_M] = reinterpret_cast<f32x2(*)[LY::RS_M]>(smem + LY::RST);
  float *uc = reinterpret_cast<float *>(smem + LY::UOFF); // uc[32 + j]: MPX sample j of the chunk
  unsigned long long *sgp = reinterpret_cast<unsigned long long *>(smem + LY::SG);
  FeShared *sh = reinterpret_cast<FeShared *>(smem + LY::SH);
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
  typedef float f32x4_t __attribute__((ext_vector_type(4)));
  const bool want_sig = a.sig_sums != nullptr;
  // IQ FIR input images (alias xin): I hi, I lo, Q hi, Q lo of the DC blockers'
  // outputs x 2^10, sample i at [i] (i < FE_HALO_IQ: the carried history)
  _Float16 *xih = reinterpret_cast<_Float16 *>(smem + LY::XIN);
  _Float16 *xil = xih + LY::IQW;
  _Float16 *xqh = xih + 2 * LY::IQW;
  _Float16 *xql = xih + 3 * LY::IQW;
  constexpr float kIqIn = 1024.0f;
#ifdef FMX_STAMPS
  unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long st_last = (a.dbg && threadIdx.x == 0) ? __builtin_amdgcn_s_memtime() : 0;
#define FE_STAMP_RAW(k)                                          \
  if (a.dbg && threadIdx.x == 0) {                               \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();  \
    st_acc[k] += t_ - st_last;                                   \
    st_last = t_;                                                \
  }
#ifdef FMX_STAMPS_DECIM // decimator split: 0 staging, 1 RF sums, 2 MFMA loop, 3 dc + IQ FIR + discriminator
#define FE_STAMP(k) FE_STAMP_RAW(((k) == 1 || (k) == 2) ? 3 : (k))
#define FE_STAMP_D(k) FE_STAMP_RAW(k)
#else
#define FE_STAMP(k) FE_STAMP_RAW(k)
#define FE_STAMP_D(k)
#endif
#else
#define FE_STAMP(k)
#define FE_STAMP_D(k)
#endif
  SigAcc sig;
  const int c = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int j0 = 8 * tid;
#ifdef FMX_STAMPS // setup split (dbg[42..47], first chunk only; flushed with the stage clocks)
  unsigned long long su_last = st_last, su_acc[6] = {0, 0, 0, 0, 0, 0}, su_w0 = 0, su_w1 = 0;
#define FE_SETUP_STAMP(k)                                                     \
  if (a.dbg && tid == 0) {                                                    \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();               \
    su_acc[k] += t_ - su_last;                                                \
    su_last = t_;                                                             \
  }
#else
#define FE_SETUP_STAMP(k)
#endif
  const FmxDesign *__restrict__ D = a.des;
  const int n = a.n;
  const FmxChanParam par = a.par[c];
  // u8 IQ chunks arrive by LDS-DMA (the first one issued after the setup
  // loads below: issued before them it costs 26 VGPRs, and vmcnt would make
  // the setup loads wait for it) (16 B per lane, 1-KiB pieces, wave w
  // moving pieces w, w+4, ...): the chunk [n0p*M - L, (n0p + FE8_T)*M) lands
  // in raw while the previous chunk's pilot FIR and RDS resampler run.
  // Bytes before the row (the first chunk's halo) read 0 (out of range) and
  // are replaced by the carried decimator history.
  const __amdgpu_buffer_rsrc_t riq = make_rsrc(a.iq + (size_t)c * a.iq_stride, (uint32_t)(2L * n * M));
  auto dma_chunk = [&](int n0p, auto p_lo_c, auto p_hi_c) __attribute__((always_inline)) {
    constexpr int P_LO = decltype(p_lo_c)::value, P_HI = decltype(p_hi_c)::value;
    uint32_t off = (uint32_t)(2 * n0p * M - LY::HB + 1024 * (P_LO + wave)) + 16u * (uint32_t)lane;
#pragma unroll
    for (int j = 0; j < (P_HI - P_LO + 3) / 4; ++j) {
      const int pc = P_LO + wave + 4 * j;
      if (pc < P_HI)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            riq, (__attribute__((address_space(3))) void *)(smem + 1024 * pc), 16, off, 0, 0, 0);
      off += 4096u;
      asm volatile("" : "+v"(off));
    }
  };
  using PAll0 = std::integral_constant<int, 0>;
  using PEarly = std::integral_constant<int, LY::NPC_EARLY>;
  using PAll = std::integral_constant<int, LY::NPC>;
  const int iqL = D->iq_len[par.iqsel];
  const float iqscale = D->iq_scale[par.iqsel];
  const bool pilot = RS && a.pilot_out != nullptr; // (the launcher never passes a pilot row to RS = false)
  const bool hist_out = pilot || a.st_hist_out != 0; // the stereo history rows
  const bool rds = a.rds_out != nullptr;
  // rs: the resampler runs here (else k_rs does it, from the MPX and the
  // previous call's window this kernel hands over in rds_win_out)
  // (RS = true with rds_win_out set: the pilot BPF here, the resampler in
  // k_rs -- the FMX_FE_PILOT A/B)
  const bool rs = RS && rds && a.rds_win_out == nullptr;
  const float dc_a1 = -1.0f + 0.0005f; // iirfilt_rrrf_create_dc_blocker(0.0005)
  const float dc_c = -dc_a1;
  const float *su = reinterpret_cast<const float *>(smem + LY::SU); // RS = false: the landed words

  // ---- zeroed images, carried state ----
  for (int h = tid; h < LY::XW / 2; h += 256) {
    reinterpret_cast<uint32_t *>(xh)[h] = 0u;
    reinterpret_cast<uint32_t *>(xl)[h] = 0u;
  }
  if (RS) __syncthreads();
  if (RS) {
    for (int h = tid; h < FE_HALO_IQ; h += 256) {
      const float2_t v = a.iq_hist[(size_t)c * (FMX_IQ_MAXLEN - 1) + h];
      hx[h] = make_float2(v.x, v.y);
    }
  }
  FE_SETUP_STAMP(0)
  if (tid == 0) {
    if (RS) {
      sh->carry_i = a.dc_v[2 * c];
      sh->carry_q = a.dc_v[2 * c + 1];
      sh->fd_re = a.fd_prev[2 * c];
      sh->fd_im = a.fd_prev[2 * c + 1];
    }
    sh->clip = 0;
  }
  FE_SETUP_STAMP(1)
  if (RS) {
    const float *hist = a.st_hist_rd + (size_t)c * FMX_HIST;
    for (int h = tid; h < FMX_HIST; h += 256) {
      const float v = pilot ? hist[h] : 0.0f;
      const _Float16 hv = (_Float16)v;
      xh[h] = hv;
      xl[h] = (_Float16)(v - (float)hv);
    }
  }
  FE_SETUP_STAMP(2)
  float agc_g = 1.0f, agc_y2p = 1.0f;
  if (RS && par.agc != 0 && tid == 0) {
    agc_g = a.agc[2 * c];
    agc_y2p = a.agc[2 * c + 1];
  }
  const float agc_bw = (par.agc == 1) ? 0.01f : 0.001f;
  const uint8_t *dhist = a.dec_hist + (size_t)c * 2 * FMX_MAX_DEC;
  const FmxSched *sched = nullptr;
  int sched_n = 0;
  float rds_keep = 0.0f; // the RDS resampler's own window of the previous call (32 samples)
  if (rds) {
    const int g = a.rds_group[c];
    sched = a.rds_sched + (size_t)g * a.rds_sched_stride;
    sched_n = a.rds_sched_n[g];
    if (RS && tid < 32) rds_keep = a.rds_hist[(size_t)c * 32 + tid];
    if (RS && !rs && tid < 32) a.rds_win_out[(size_t)c * 32 + tid] = rds_keep;
  }
  FE_SETUP_STAMP(3)
  if (rs) {
    // pair p < 32: (branch p, branch p+1 mod 32) on the same window; pair 32
    // (boundary): branch 31 on the window, branch 0 on the window shifted by
    // one -- 27 terms, oldest sample first, so every lane runs one chain
    for (int idx = tid; idx < LY::RS_PAIRS * LY::RS_M; idx += 256) {
      const int pr = idx / LY::RS_M, m = idx % LY::RS_M;
      const float *hs = D->rds_rs_h; // [branch][26]
      float h0, h1;
      if (pr < FMX_NPFB) {
        const int b1 = (pr + 1) & (FMX_NPFB - 1);
        h0 = m < FMX_RDS_RS_SUB ? hs[pr * FMX_RDS_RS_SUB + FMX_RDS_RS_SUB - 1 - m] : 0.0f;
        h1 = m < FMX_RDS_RS_SUB ? hs[b1 * FMX_RDS_RS_SUB + FMX_RDS_RS_SUB - 1 - m] : 0.0f;
      } else {
        h0 = m < FMX_RDS_RS_SUB ? hs[(FMX_NPFB - 1) * FMX_RDS_RS_SUB + FMX_RDS_RS_SUB - 1 - m] : 0.0f;
        h1 = m >= 1 ? hs[FMX_RDS_RS_SUB - m] : 0.0f;
      }
      rsb[pr][m] = f32x2{h0, h1};
    }
  }
  // Chunks (round 5): ceil(n / FE8_T) chunks of one size cs (a multiple of 8,
  // <= FE8_T; the last one takes the rest), so any call of n >= FE8_MIN_N
  // (the reference's dsp_block_samples clamp, 1024) has every chunk >= 904
  // samples: the histories the call hands on (IQ FIR 120, stereo rows 512,
  // RDS window 32) always lie inside its last chunk.
  const int nch = (n + FE8_T - 1) / FE8_T;
  const int cs = (((n + nch - 1) / nch) + 7) & ~7;
  // per-channel decimator warmth (round 5): after a reset the reference's
  // window holds complex zeros (ComplexDecimator::reset re-creates the
  // firdecim_crcf, liquid_primitives.cpp:405-420); the coldk oldest history
  // positions of this channel are such zeros (below: bytes 128 in the MFMA,
  // and the 0.5 * taps of the 127.5 centre taken back out of the outputs that
  // reach them).  Read where it is used (first chunk only): SGPRs are scarce.
  auto cold_k = [&]() __attribute__((always_inline)) { return (L - 1) - min(max(a.dec_valid[c], 0), L - 1); };
  dma_chunk(0, PAll0{}, PAll{});
  if (!RS) {
    // the decimator's and the IQ FIR's tap windows by LDS-DMA behind the
    // first chunk's bytes (round 6): no register round trip and no wait here
    // -- they land with the chunk, before its barrier (a copy through
    // registers waited ~5 us for the loads ahead of the chunk's DMA)
    static_assert(FMX_IQ_QN % 2 == 0, "dword windows");
    const float *qs = reinterpret_cast<const float *>(&D->dec_q16[0][0]);
    const float *is = reinterpret_cast<const float *>(&D->iq_q16[par.iqsel][0][0][0]);
    for (int p = wave; p < LY::QDP + LY::QIP; p += 4) {
      const bool dec = p < LY::QDP;
      const int e = 64 * (dec ? p : p - LY::QDP) + lane;
      const float *src = dec ? qs + min(e, FMX_DEC_QN - 1) : is + min(e, 2 * FMX_IQ_QN - 1);
      dma_dword(src, lds_addr(smem + (dec ? LY::QT + 256 * p : LY::QI + 256 * (p - LY::QDP))));
    }
    // ... and the carried state (round 6): the IQ FIR history into hx (one
    // 64-dword piece per wave), the DC / discriminator / AGC words and the
    // RDS window (wave 0) and the decimator's byte history (waves 1..3) into
    // the landing area -- read after the chunk's barrier, no wait of their own
    {
      const float *ih = reinterpret_cast<const float *>(a.iq_hist + (size_t)c * (FMX_IQ_MAXLEN - 1));
      dma_dword(ih + min(tid, 2 * FE_HALO_IQ - 1), lds_addr(smem + LY::HX + 256 * wave));
      const float *w0 = a.dc_v + 2 * c;
      if (wave == 0) {
        const float *src = w0;
        if (lane < 2) src = w0 + lane;
        else if (lane < 4) src = a.fd_prev + 2 * c + (lane - 2);
        else if (lane < 6) src = par.agc != 0 ? a.agc + 2 * c + (lane - 4) : w0;
        else if (lane >= 8 && lane < 40) src = rds ? a.rds_hist + (size_t)c * 32 + (lane - 8) : w0;
        dma_dword(src, lds_addr(smem + LY::SU));
      } else {
        const float *hb = reinterpret_cast<const float *>(dhist);
        dma_dword(hb + min(64 * (wave - 1) + lane, (2 * (L - 1) + 3) / 4 - 1), lds_addr(smem + LY::SU + 4 * LY::SU_H + 256 * (wave - 1)));
      }
    }
  }
  FE_SETUP_STAMP(4)
  int e_pos = 0;
  uint16_t keep[2] = {0, 0}; // the next call's decimator history (L - 1 <= 511 samples: two per thread)

  for (int n0 = 0; n0 < n; n0 += cs) {
    const int cnt = min(cs, n - n0); // samples of this chunk (a multiple of 4)
    if (rs && tid == 0) sh->e_end = e_pos;
    // ================= decimator =================
#ifdef FMX_STAMPS
    // the DMA wait alone (dbg[40] first chunk, dbg[41] later chunks)
    unsigned long long tw0_ = (a.dbg && tid == 0) ? __builtin_amdgcn_s_memtime() : 0;
    if (n0 == 0) { FE_SETUP_STAMP(5) }
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads(); // this chunk's DMA has landed (every wave)
#ifdef FMX_STAMPS
    if (a.dbg && tid == 0) { if (n0 == 0) su_w0 += __builtin_amdgcn_s_memtime() - tw0_; else su_w1 += __builtin_amdgcn_s_memtime() - tw0_; }
#endif
    FE_STAMP(7) // setup / previous chunk's carry + the DMA wait
    if (n0 + cnt >= n) {
      // the call's last L - 1 IQ samples (the next call's decimator history)
      // from this chunk's bytes in raw (sample n M - (L - 1) + h at u16 cnt M + 1 + h)
      int k = 0;
      for (int h = tid; h < L - 1; h += 256) keep[k++] = reinterpret_cast<const uint16_t *>(raw)[cnt * M + 1 + h];
    }
    if (!RS && n0 == 0) {
      if (tid == 0) {
        sh->carry_i = su[0];
        sh->carry_q = su[1];
        sh->fd_re = su[2];
        sh->fd_im = su[3];
        if (par.agc != 0) {
          agc_g = su[4];
          agc_y2p = su[5];
        }
      }
      if (rds && tid < 32) a.rds_win_out[(size_t)c * 32 + tid] = su[8 + tid];
    }
    if (n0 == 0) { // halo: a zero lead sample, then the carried L-1 samples (cold ones: byte 128, i.e. b - 128 = 0)
      const int coldk = cold_k();
      const uint16_t *dh16 = reinterpret_cast<const uint16_t *>(su + LY::SU_H);
      for (int h = tid; h < L; h += 256) {
        const int hh = h - 1;
        uint16_t v = 0;
        if (hh >= 0)
          v = hh < coldk ? (uint16_t)0x8080u
                         : (RS ? (uint16_t)((uint16_t)dhist[2 * hh] | ((uint16_t)dhist[2 * hh + 1] << 8)) : dh16[hh]);
        reinterpret_cast<uint16_t *>(raw)[h] = v;
      }
      __syncthreads();
      if (coldk > 0 && tid < (coldk + M - 1) / M) {
        // the outputs whose window reaches the zeroed positions, in f32 from
        // the bytes (the window's real samples only, oldest first, as the
        // reference's zeroed firdecim window): the MFMA form's 127.5 centre
        // (dec_dc16) is exact only up to its f32 rounding, which these small
        // outputs (the window's taper over a few real samples) feel
        // relatively at weak carriers.  Staged in sh->cold_y, they replace
        // the MFMA outputs at the staging step.
        float sI = 0.0f, sQ = 0.0f;
        for (int d = L; d >= 1; --d) {
          const int t = M * tid + d; // raw position: 1 .. L-1 history, L.. the call
          if (t <= coldk) continue;
          const float h = D->dec_taps[L - d];
          sI = sI + h * ((float)raw[2 * t] - 127.5f);
          sQ = sQ + h * ((float)raw[2 * t + 1] - 127.5f);
        }
        sh->cold_y[tid] = make_float2(sI * D->dec_scale, sQ * D->dec_scale);
      }
    }
    if (want_sig) {
#pragma unroll
      for (int j = 0; j < LY::NPF; ++j) {
        const int off = 16 * (tid + 256 * j);
        if (off >= LY::HB && off < LY::HB + 2 * cnt * M) {
          const u32x4 w = *reinterpret_cast<const u32x4 *>(raw + off);
          sig.word4(w);
        }
      }
    }
    FE_STAMP_D(1)
    float2 xv[8]; // decimator outputs of this thread
    {
      // Decimator as v_mfma_f32_16x16x32_f16 tiles.  Output o = 16 B + r of
      // the chunk (block B, r < 16) uses raw samples 16 M B + t, t in
      // [M r + 1, M r + L], with tap L + M r - t: per block, Y[r] = sum_t
      // T[r][t] X[t] with T[r][t] = q[t - M r] (FmxDesign::dec_q16) -- one
      // 16 x 16 tile is 16 outputs (rows, A = taps) of 16 blocks (columns,
      // B = bytes), K = the block's 15 M + L + 1 input samples in steps of 32.
      // Each wave runs two tiles (512 outputs); the bytes enter exactly as
      // f16 (b - 128), the taps as f16 hi + lo, both products accumulate in
      // f32.  The C layout gives each lane 4 consecutive outputs; they reach
      // the 8-per-thread layout of the stages below through LDS.
      typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
      typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
      typedef float f32x4_t __attribute__((ext_vector_type(4)));
      constexpr int KS = LY::KS;
      static_assert(KS <= FMX_DEC_KS_MAX, "decimator K steps");
      const int col = lane & 15, g = lane >> 4;
      // A fragments, one K step ahead: RS = false from the LDS tap window (8
      // consecutive f16 from 32 ks + 8 g + 15 M - M col, an even index: four
      // dwords, two ds_read2_b32 per half -- round 5 read dec_frag from L2,
      // 2 KB per wave and K step, and every K step waited on that load), RS =
      // true from the design's fragment table (16 B per lane)
      const uint32_t *qh = reinterpret_cast<const uint32_t *>(smem + LY::QT) + (15 * M + 8 * g - M * col) / 2;
      const uint32_t *ql = qh + FMX_DEC_QN / 2;
      const u32x4 *fa = reinterpret_cast<const u32x4 *>(&D->dec_frag[0][0][0][0]) + lane;
      auto frag = [&](int ks, int s) __attribute__((always_inline)) {
        if (RS) return fa[128 * ks + 64 * s];
        const uint32_t *q = (s ? ql : qh) + 16 * ks;
        return u32x4{q[0], q[1], q[2], q[3]};
      };
      u32x4 fh = frag(0, 0), fl = frag(0, 1);
      const unsigned char *rb = raw + 32 * M * (32 * wave + col) + 16 * g;
      f32x4_t acc[2][2];
#pragma unroll
      for (int u = 0; u < 2; ++u) acc[u][0] = acc[u][1] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
      // bytes (I0 Q0 I1 Q1) -> f16 pairs (1024 + b, 1024 + b') by v_perm with
      // the f16 exponent byte 0x64, then - 1152: b - 128 exactly
      auto cvt = [](uint32_t w, uint32_t sel) __attribute__((always_inline)) {
        return __builtin_bit_cast(f16x2_t, __builtin_amdgcn_perm(0x64646464u, w, sel)) -
               f16x2_t{(_Float16)1152.0f, (_Float16)1152.0f};
      };
      // software pipeline (round 6): the next K step's operands -- its bytes
      // (two ds_read_b128) and fragments -- are issued before this step's
      // conversions and MFMAs, which hide their latency (the scheduling
      // barrier keeps the compiler from sinking them back to their uses)
      u32x4 wcur[2], wnxt[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) wnxt[u] = wcur[u] = *reinterpret_cast<const u32x4 *>(rb + 512 * M * u);
#pragma unroll 7
      for (int ks = 0; ks < KS; ++ks) {
        const f16x8_t ahi = __builtin_bit_cast(f16x8_t, fh), alo = __builtin_bit_cast(f16x8_t, fl);
        if (ks + 1 < KS) {
          fh = frag(ks + 1, 0);
          fl = frag(ks + 1, 1);
#pragma unroll
          for (int u = 0; u < 2; ++u) wnxt[u] = *reinterpret_cast<const u32x4 *>(rb + 512 * M * u + 64 * (ks + 1));
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const u32x4 w = wcur[u];
          const f16x2_t i0 = cvt(w.x, 0x04020400u), i1 = cvt(w.y, 0x04020400u);
          const f16x2_t i2 = cvt(w.z, 0x04020400u), i3 = cvt(w.w, 0x04020400u);
          const f16x2_t q0 = cvt(w.x, 0x04030401u), q1 = cvt(w.y, 0x04030401u);
          const f16x2_t q2 = cvt(w.z, 0x04030401u), q3 = cvt(w.w, 0x04030401u);
          const f16x8_t bi = {i0.x, i0.y, i1.x, i1.y, i2.x, i2.y, i3.x, i3.y};
          const f16x8_t bq = {q0.x, q0.y, q1.x, q1.y, q2.x, q2.y, q3.x, q3.y};
          // transposed tile (bytes as A, taps as B: the same lane
          // registers): D[block][output], so the 16 lanes of a group hold 16
          // consecutive outputs
          acc[u][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bi, ahi, acc[u][0], 0, 0, 0);
          acc[u][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bq, ahi, acc[u][1], 0, 0, 0);
          acc[u][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bi, alo, acc[u][0], 0, 0, 0);
          acc[u][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bq, alo, acc[u][1], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < 2; ++u) wcur[u] = wnxt[u];
      }
      FE_STAMP_D(2)
      __syncthreads(); // every wave is past raw: its outputs go to the (aliased) staging area
      float2 *stg = reinterpret_cast<float2 *>(smem + LY::STG);
      const float dc = D->dec_dc16, sc = D->dec_scale16;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        // lane: outputs 256 (2 wave + u) + 16 (4 g + i) + col, i = 0..3
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int o = 256 * (2 * wave + u) + 16 * (4 * g + i) + col;
          stg[fe8_stg(o)] = make_float2((acc[u][0][i] - dc) * sc, (acc[u][1][i] - dc) * sc);
        }
      }
      __syncthreads();
      const int coldk = n0 == 0 ? cold_k() : 0;
      if (coldk > 0) { // workgroup-uniform: a cold channel's first chunk (values from the halo step)
        if (tid < (coldk + M - 1) / M) stg[fe8_stg(tid)] = sh->cold_y[tid];
        __syncthreads();
      }
      int myclip = 0;
#pragma unroll
      for (int r = 0; r < 8; r += 2) {
        const float4 v = *reinterpret_cast<const float4 *>(stg + fe8_stg(j0 + r)); // 16-B aligned: j0 + r even
        xv[r] = make_float2(v.x, v.y);
        xv[r + 1] = make_float2(v.z, v.w);
      }
#pragma unroll
      for (int r = 0; r < 8; ++r)
        if (j0 + r < cnt && (fabsf(xv[r].x) >= 0.995f || fabsf(xv[r].y) >= 0.995f)) myclip++;
      if (myclip) atomicAdd(&sh->clip, myclip);
    }
    __syncthreads(); // raw is dead: xin / yb alias it from here on
    FE_STAMP(0)
    // IQ FIR history and the zero slack past the chunk (read with zero taps)
    if (tid < FE_HALO_IQ) {
      const float2 v = hx[tid];
      const float sI = v.x * kIqIn, sQ = v.y * kIqIn;
      const _Float16 hI = (_Float16)sI, hQ = (_Float16)sQ;
      xih[tid] = hI;
      xil[tid] = (_Float16)(sI - (float)hI);
      xqh[tid] = hQ;
      xql[tid] = (_Float16)(sQ - (float)hQ);
    }
    if (tid < 32) {
      const int i = FE_HALO_IQ + FE8_T + tid;
      xih[i] = xil[i] = xqh[i] = xql[i] = (_Float16)0.0f;
    }
    // ================= DC blockers: affine scan, 8 per thread =================
    {
      float A = 1.0f, BI = 0.0f, BQ = 0.0f;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        BI = xv[r].x + dc_c * BI;
        BQ = xv[r].y + dc_c * BQ;
        A = dc_c * A;
      }
      wave_affine_scan(A, BI, BQ);
      if (lane == 63) {
        sh->wave_a[wave] = A;
        sh->wave_bi[wave] = BI;
        sh->wave_bq[wave] = BQ;
      }
      float eA, eI, eQ;
      wave_affine_prev(A, BI, BQ, eA, eI, eQ);
      __syncthreads();
      float vI = sh->carry_i, vQ = sh->carry_q;
      for (int w = 0; w < wave; ++w) {
        // scalar asm: the vectoriser's packed form of this pair put LDS loads
        // over the sources of a just-issued v_pk_* op (tests/test_isa_scan.py)
        const float wa = sh->wave_a[w], wi = sh->wave_bi[w], wq = sh->wave_bq[w];
        asm("v_mul_f32 %0, %2, %0\n\tv_add_f32 %0, %0, %3\n\tv_mul_f32 %1, %2, %1\n\tv_add_f32 %1, %1, %4"
            : "+v"(vI), "+v"(vQ)
            : "v"(wa), "v"(wi), "v"(wq));
      }
      vI = eA * vI + eI;
      vQ = eA * vQ + eQ;
      // the state before this thread's first element, then the reference's op order
      f16x8_t ih, il, qh, ql;
      const int rlast = (tid == (cnt - 1) >> 3) ? ((cnt - 1) & 7) : -1; // the chunk's last sample
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const float tI = dc_a1 * vI, tQ = dc_a1 * vQ;
        const float nI = xv[r].x - tI, nQ = xv[r].y - tQ;
        const float oI = nI - vI, oQ = nQ - vQ;
        const float sI = oI * kIqIn, sQ = oQ * kIqIn;
        ih[r] = (_Float16)sI;
        il[r] = (_Float16)(sI - (float)ih[r]);
        qh[r] = (_Float16)sQ;
        ql[r] = (_Float16)(sQ - (float)qh[r]);
        // the next chunk's IQ FIR history (f32; read above before the scan's barrier)
        if (j0 + r >= cnt - FE_HALO_IQ && j0 + r < cnt) hx[j0 + r - (cnt - FE_HALO_IQ)] = make_float2(oI, oQ);
        vI = nI;
        vQ = nQ;
        if (r == rlast) {
          sh->carry_n[0] = nI;
          sh->carry_n[1] = nQ;
        }
      }
      *reinterpret_cast<f16x8_t *>(xih + FE_HALO_IQ + j0) = ih;
      *reinterpret_cast<f16x8_t *>(xil + FE_HALO_IQ + j0) = il;
      *reinterpret_cast<f16x8_t *>(xqh + FE_HALO_IQ + j0) = qh;
      *reinterpret_cast<f16x8_t *>(xql + FE_HALO_IQ + j0) = ql;
      __syncthreads();
      if (tid == 0) {
        sh->carry_i = sh->carry_n[0];
        sh->carry_q = sh->carry_n[1];
      }
    }
    __syncthreads();
    FE_STAMP(1)
    // ================= IQ FIR =================
    {
      // v_mfma_f32_16x16x32_f16 tiles as the pilot BPF's: 16 outputs (rows,
      // A = taps, FmxDesign::iq_frag) of 16 blocks of 16 outputs (columns, B
      // = the I or Q images), K = the block's P8 + 15 inputs; three MFMAs per
      // K step and component (hi*hi, hi*lo, lo*hi) into f32 accumulators.
      // Each wave: two tiles (512 outputs) of I and of Q.
      const int P8 = fir8_len(iqL);
      const int KSI = D->iq_ks[par.iqsel];
      const int col = lane & 15, g = lane >> 4;
      const int xb = FE_HALO_IQ + 16 * (32 * wave + col) - (P8 - 1) + 8 * g; // 8-aligned: P8 = 8k + 1
      const f16x8_t *bih = reinterpret_cast<const f16x8_t *>(xih + xb);
      const f16x8_t *bil = reinterpret_cast<const f16x8_t *>(xil + xb);
      const f16x8_t *bqh = reinterpret_cast<const f16x8_t *>(xqh + xb);
      const f16x8_t *bql = reinterpret_cast<const f16x8_t *>(xql + xb);
      const u32x4 *fa = reinterpret_cast<const u32x4 *>(&D->iq_frag[par.iqsel][0][0][0][0]) + lane;
      // RS = false: A fragments from the design's LDS window (round 6), this
      // lane's 8 entries from 32 ks + 8 g + 15 - col in copy (15 - col) & 1
      const int qb = 8 * g + 15 - col, qc = qb & 1;
      const uint32_t *qih = reinterpret_cast<const uint32_t *>(smem + LY::QI) + qc * FMX_IQ_QN + (qb - qc) / 2;
      const uint32_t *qil = qih + FMX_IQ_QN / 2;
      auto ifrag = [&](int ks, int s) __attribute__((always_inline)) {
        if (RS) return fa[128 * ks + 64 * s];
        const uint32_t *q = (s ? qil : qih) + 16 * ks;
        return u32x4{q[0], q[1], q[2], q[3]};
      };
      f32x4_t ai[2], aq[2];
      ai[0] = ai[1] = aq[0] = aq[1] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
      u32x4 ah = ifrag(0, 0), al = ifrag(0, 1);
      for (int ks = 0; ks < KSI; ++ks) {
        const f16x8_t ahi = __builtin_bit_cast(f16x8_t, ah), alo = __builtin_bit_cast(f16x8_t, al);
        if (ks + 1 < KSI) {
          ah = ifrag(ks + 1, 0);
          al = ifrag(ks + 1, 1);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const f16x8_t ihi = bih[32 * u + 4 * ks], ilo = bil[32 * u + 4 * ks]; // + 256 u + 32 ks samples
          const f16x8_t qhi = bqh[32 * u + 4 * ks], qlo = bql[32 * u + 4 * ks];
          // transposed tiles (images as A, taps as B), as the decimator's
          ai[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ihi, ahi, ai[u], 0, 0, 0);
          aq[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(qhi, ahi, aq[u], 0, 0, 0);
          ai[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ilo, ahi, ai[u], 0, 0, 0);
          aq[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(qlo, ahi, aq[u], 0, 0, 0);
          ai[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ihi, alo, ai[u], 0, 0, 0);
          aq[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(qhi, alo, aq[u], 0, 0, 0);
        }
      }
      const float osc = iqscale * (1.0f / (4096.0f * kIqIn)); // exact: a power-of-two rescale
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        // lane: outputs 256 (2 wave + u) + 16 col + 4 g + i, i = 0..3
        // lane: outputs 256 (2 wave + u) + 16 (4 g + i) + col -- 16 lanes,
        // 16 consecutive float2: conflict-free ds_write_b64 (untransposed,
        // 4 outputs per lane 128 B apart across the lanes, it was 16-way)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          yb[1 + 256 * (2 * wave + u) + 16 * (4 * g + i) + col] = make_float2(ai[u][i] * osc, aq[u][i] * osc);
      }
      if (tid == 0) yb[0] = make_float2(sh->fd_re, sh->fd_im);
    }
    __syncthreads();
    // ================= AGC (serial, only when enabled) =================
    if (par.agc != 0) {
      if (tid == 0) {
        for (int j = 0; j < cnt; ++j) {
          const float2 x = yb[1 + j];
          const float yr = x.x * agc_g, yi = x.y * agc_g;
          const float y2 = yr * yr + yi * yi;
          agc_y2p = (float)((1.0 - (double)agc_bw) * (double)agc_y2p + (double)(agc_bw * y2));
          if (agc_y2p > 1e-6f) agc_g *= expf(-0.5f * agc_bw * logf(agc_y2p));
          if (agc_g > 1e6f) agc_g = 1e6f;
          yb[1 + j] = make_float2(yr, yi);
        }
      }
      __syncthreads();
    }
    FE_STAMP(2)
    // ================= discriminator =================
    float mv[8];
    {
      const float ref = (par.fd_ref != 0.0f) ? par.fd_ref : D->fd_ref; // freqdem 1 / (2 pi kf)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int j = tid + 256 * k;
        const float2 p = yb[j], r = yb[1 + j];
        const float re = p.x * r.x + p.y * r.y;
        const float im = p.x * r.y - p.y * r.x;
        const float m = fmx_atan2f(im, re) * ref; // select-free (fmx_math.h)
        mv[k] = m;
        // f16 hi / lo split for the MFMA pilot BPF (m = hi + lo to 22 bits)
        if (pilot) {
          const _Float16 hv = (_Float16)m;
          xh[FMX_HIST + j] = hv;
          xl[FMX_HIST + j] = (_Float16)(m - (float)hv);
        }
        if (a.mpx_out && j < cnt) a.mpx_out[(size_t)c * a.mpx_stride + n0 + j] = m;
      }
      if (tid == 0) {
        sh->fd_re = yb[cnt].x;
        sh->fd_im = yb[cnt].y;
      }
    }
    __syncthreads(); // xin / yb are dead: the next chunk may land in raw (below uc)
    // RDS schedule entries of this chunk, fetched before the early DMA and the
    // resampler's window copy
    FmxSched en[8];
    if (rs) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int e = e_pos + tid + 256 * k;
        en[k] = (e < sched_n) ? sched[e] : FmxSched{0xFFFF, 0.0f};
      }
    }
    if (n0 + cnt < n) dma_chunk(n0 + cnt, PAll0{}, PEarly{});
    const bool last_chunk = n0 + cnt >= n;
    if (rds || hist_out) { // unpadded f32 copy: the RDS resampler's input (its own window history first), the history rows
#pragma unroll
      for (int k = 0; k < 8; ++k) uc[32 + tid + 256 * k] = mv[k];
    }
    if (rs) {
      if (tid < 32) {
        uc[tid] = (n0 == 0) ? rds_keep : tl32[tid];
        uc[32 + cnt + tid] = 0.0f;
      }
    }
    FE_STAMP(3)
    // ================= RDS resampler 240k -> 171k =================
    if (rs) {
      __syncthreads(); // uc complete
      int last = -1;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int e = e_pos + tid + 256 * k;
        if (e < sched_n && (en[k].packed & 0xFFFF) < n0 + cnt) {
          const int i = (en[k].packed & 0xFFFF) - n0;
          const int b = (en[k].packed >> 16) & 0xFF;
          const bool boundary = (en[k].packed >> 24) & 1;
          // the window's oldest sample (one earlier at a boundary), as uc index
          // LDS addresses kept opaque: the reads then use the instruction's
          // offset field (m) instead of one address add per read pair
          uint32_t xa = (uint32_t)(uintptr_t)(lds_f32 *)(uc + 32 + (boundary ? i - 1 : i) - (FMX_RDS_RS_SUB - 1));
          uint32_t ha = (uint32_t)(uintptr_t)(lds_f32x2 *)rsb[boundary ? FMX_NPFB : b];
          asm volatile("" : "+v"(xa), "+v"(ha));
          const lds_f32 *xu = (const lds_f32 *)(uintptr_t)xa;
          const lds_f32x2 *hk = (const lds_f32x2 *)(uintptr_t)ha;
          // two fused multiply-add chains, oldest sample first (the
          // reference's branch dot products, each product fused into its
          // sum: one rounding per tap instead of two, within the PCM / MPX
          // bars of tests/test_gpu_parity.py).  Scalar v_fma_f32 as asm: the
          // packed-FP32 form (v_pk_mul / v_pk_add, which the vectorizer
          // makes of the pair) returned wrong upper-32-lane results,
          // nondeterministically, with two k_fe8 workgroups per CU issuing
          // MFMAs
          float y0 = 0.0f, y1 = 0.0f;
#pragma unroll
          for (int m = 0; m < LY::RS_M; ++m) {
            const float v = xu[m];
            const f32x2 hm = hk[m];
            asm("v_fma_f32 %0, %1, %2, %0" : "+v"(y0) : "v"(hm.x), "v"(v));
            asm("v_fma_f32 %0, %1, %2, %0" : "+v"(y1) : "v"(hm.y), "v"(v));
          }
          const f32x2 y = {y0, y1};
          const float w0f = (1.0f - en[k].mu) * y.x;
          const float w1f = en[k].mu * y.y;
          a.rds_out[(size_t)c * a.rds_stride + e] = w0f + w1f;
          last = e;
        }
      }
      if (last >= 0) atomicMax(&sh->e_end, last + 1);
    }
    if (!rs && last_chunk) __syncthreads(); // uc complete (the resampler's barrier otherwise)
    // the call's last FMX_HIST samples: the next call's stereo history rows,
    // its last 32 the next call's RDS resampler window (HBM); the chunk's last
    // 32 the next chunk's window history (every read of tl32 for this chunk
    // was before the "uc complete" barrier)
    if (last_chunk) {
      if (hist_out) {
        static_assert(FMX_HIST == 512, "two history words per thread");
        const __amdgpu_buffer_rsrc_t rh = make_rsrc(a.st_hist_wr + (size_t)c * FMX_HIST, FMX_HIST * 4);
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, uc[32 + cnt - FMX_HIST + tid]), rh,
                                              4u * tid, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, uc[32 + cnt - 256 + tid]), rh,
                                              4u * tid, 1024, 0);
      }
      if (rds && tid < 32) a.rds_hist[(size_t)c * 32 + tid] = uc[cnt + tid];
    }
    if (rs && tid < 32) tl32[tid] = uc[cnt + tid];
    __syncthreads(); // uc is dead: the rest of the next chunk may land (behind the pilot FIR)
    if (n0 + cnt < n) dma_chunk(n0 + cnt, PEarly{}, PAll{});
    if (rs) e_pos = sh->e_end;
    FE_STAMP(5)
    // ================= 19 kHz pilot band-pass =================
    if (pilot) {
      // v_mfma_f32_16x16x32_f16 tiles as the decimator's: 16 outputs (rows,
      // A = taps) of 16 blocks of 16 outputs (columns, B = MPX), K = the
      // block's P8 + 15 inputs from x[16 B - P8 + 1]; B from the hi / lo
      // images (two 16-B reads), A fragments (FmxDesign::pilot_frag, tap *
      // 2^12 as hi + lo) from global memory, one K step ahead; three MFMAs
      // per K step (hi*hi, hi*lo, lo*hi).  Each wave: two tiles, 512 outputs.
      typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
      typedef float f32x4_t __attribute__((ext_vector_type(4)));
      const int P8 = fir8_len(D->pilot_len);
      const int KSP = D->pilot_ks;
      const int col = lane & 15, g = lane >> 4;
      const int xb = FMX_HIST + 16 * (32 * wave + col) - (P8 - 1) + 8 * g; // 8-aligned: P8 = 8k + 1
      const f16x8_t *bh = reinterpret_cast<const f16x8_t *>(xh + xb);
      const f16x8_t *bl = reinterpret_cast<const f16x8_t *>(xl + xb);
      const u32x4 *fa = reinterpret_cast<const u32x4 *>(&D->pilot_frag[0][0][0][0]) + lane;
      const __amdgpu_buffer_rsrc_t prow = make_rsrc(a.pilot_out + (size_t)c * a.pilot_stride, 4u * (uint32_t)n);
      f32x4_t pacc[2];
      pacc[0] = pacc[1] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
      u32x4 ah = fa[0], al = fa[64];
      for (int ks = 0; ks < KSP; ++ks) {
        const f16x8_t ahi = __builtin_bit_cast(f16x8_t, ah), alo = __builtin_bit_cast(f16x8_t, al);
        if (ks + 1 < KSP) {
          ah = fa[128 * (ks + 1)];
          al = fa[128 * (ks + 1) + 64];
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const f16x8_t xhi = bh[32 * u + 4 * ks], xlo = bl[32 * u + 4 * ks]; // + 256 u + 32 ks samples
          pacc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, xhi, pacc[u], 0, 0, 0);
          pacc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, xlo, pacc[u], 0, 0, 0);
          pacc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo, xhi, pacc[u], 0, 0, 0);
        }
      }
      constexpr float kInv = 1.0f / 4096.0f;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        // lane: outputs 256 (2 wave + u) + 16 col + 4 g + i, i = 0..3, as a
        // buffer store over the call's row: outputs past n (a shorter last
        // chunk; cnt is a multiple of 4) are dropped by the range check, no branch
        const int o = n0 + 256 * (2 * wave + u) + 16 * col + 4 * g;
        const u32x4 pv = u32x4{__builtin_bit_cast(uint32_t, pacc[u][0] * kInv), __builtin_bit_cast(uint32_t, pacc[u][1] * kInv),
                               __builtin_bit_cast(uint32_t, pacc[u][2] * kInv), __builtin_bit_cast(uint32_t, pacc[u][3] * kInv)};
        __builtin_amdgcn_raw_buffer_store_b128(pv, prow, 4u * (uint32_t)o, 0, 0);
      }
    }
    FE_STAMP(4)
    // ================= carry halos to the next chunk =================
    // (RS = false has no images; nothing after the "uc is dead" barrier reads
    // LDS there, so the next chunk needs no barrier here)
    if (RS) {
      // the chunk's last FMX_HIST samples become the f16 images' history
      static_assert(FMX_HIST == 2 * 256, "one f16 pair per thread");
      const uint32_t ch = reinterpret_cast<const uint32_t *>(xh)[cnt / 2 + tid];
      const uint32_t cl = reinterpret_cast<const uint32_t *>(xl)[cnt / 2 + tid];
      __syncthreads();
      reinterpret_cast<uint32_t *>(xh)[tid] = ch;
      reinterpret_cast<uint32_t *>(xl)[tid] = cl;
      __syncthreads();
    }
  }

  // ---- write back state ----
  {
    static_assert(L - 1 <= 512, "two history samples per thread");
    int cntk = 0;
    uint16_t *dh = reinterpret_cast<uint16_t *>(a.dec_hist + (size_t)c * 2 * FMX_MAX_DEC);
    for (int h = tid; h < L - 1; h += 256) dh[h] = keep[cntk++];
    if (tid == 0) a.dec_valid[c] = L - 1; // n M >= 1024 M > L - 1 new samples
  }
  for (int h = tid; h < FE_HALO_IQ; h += 256) {
    const float2 v = hx[h];
    a.iq_hist[(size_t)c * (FMX_IQ_MAXLEN - 1) + h] = float2_t{v.x, v.y};
  }
  if (tid == 0) {
    a.dc_v[2 * c] = sh->carry_i;
    a.dc_v[2 * c + 1] = sh->carry_q;
    a.fd_prev[2 * c] = sh->fd_re;
    a.fd_prev[2 * c + 1] = sh->fd_im;
    if (par.agc != 0) {
      a.agc[2 * c] = agc_g;
      a.agc[2 * c + 1] = agc_y2p;
    }
  }
  if (rds && tid == 0) a.rds_count[c] = sched_n;
  if (tid == 0 && a.clip_out) a.clip_out[c] = (float)sh->clip / (float)n;
  FE_STAMP(6)
#ifdef FMX_STAMPS
  if (a.dbg && tid == 0) {
    for (int k = 0; k < 8; ++k) atomicAdd(a.dbg + k, st_acc[k]);
    for (int k = 0; k < 6; ++k) atomicAdd(a.dbg + 42 + k, su_acc[k]);
    atomicAdd(a.dbg + 40, su_w0);
    atomicAdd(a.dbg + 41, su_w1);
  }
#endif
#undef FE_STAMP
#undef FE_STAMP_D
#undef FE_STAMP_RAW
  if (want_sig) fe_signal_sums(a, sig, sgp, c, lane, wave, tid);
  // at the end, where registers are free (at the entry it cost 28 VGPRs)
  fe_next_sched_copy(a);
}

// the events of set_launch_events, consumed by the next fmx_launch
static thread_local hipEvent_t t_ev_start = nullptr, t_ev_stop = nullptr;
void set_launch_events(void *start, void *stop) {
  t_ev_start = static_cast<hipEvent_t>(start);
  t_ev_stop = static_cast<hipEvent_t>(stop);
}
template <typename K, typename... Args>
static int fmx_launch(K kernel, dim3 grid, dim3 block, size_t smem, hipStream_t st, Args... args) {
  hipEvent_t e0 = t_ev_start, e1 = t_ev_stop;
  t_ev_start = t_ev_stop = nullptr;
  if (e0 || e1) hipExtLaunchKernelGGL(kernel, grid, block, (uint32_t)smem, st, e0, e1, 0u, args...);
  else hipLaunchKernelGGL(kernel, grid, block, smem, st, args...);
  return hipGetLastError() == hipSuccess ? FMX_OK : FMX_E_HIP;
}

template <int M, int TPP, bool RS> static int fe8_launch_rs(const FeArgs &a, hipStream_t st) {
  // 160 KB per CU: two k_fe8 workgroups (512-B allocation granules) beside one
  // k_pll or k_rds workgroup (36 KB each, 36 864 B allocated)
  static_assert(Fe8Layout<M, TPP, RS>::BYTES <= (160 * 1024 - 36864) / 2, "k_fe8: two workgroups per CU plus a k_pll / k_rds workgroup");
  static_assert(Fe8Layout<M, TPP, RS>::UOFF >= Fe8Layout<M, TPP, RS>::YB, "RDS copy above the IQ image");
  const size_t smem = (size_t)Fe8Layout<M, TPP, RS>::BYTES;
  static bool configured = false;
  if (!configured) {
    if (hipFuncSetAttribute(reinterpret_cast<const void *>(&k_fe8<M, TPP, RS>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem) != hipSuccess)
      return FMX_E_HIP;
    configured = true;
  }
  return fmx_launch(k_fe8<M, TPP, RS>, dim3(a.C), dim3(256), smem, st, a);
}
// the resampler in the kernel, or (rds_win_out set) left to k_rs
// (process_block's variant, RS = false, has no pilot BPF: k_pilot runs it)
template <int M, int TPP> static int fe8_launch(const FeArgs &a, hipStream_t st) {
  if (a.rds_out && a.rds_win_out && !a.pilot_out) return fe8_launch_rs<M, TPP, false>(a, st);
  return fe8_launch_rs<M, TPP, true>(a, st);
}

/* ================================================================== */
/* launchers                                                           */
/* ================================================================== */
template <int M, int TPP, bool VEC> static int fe_launch(const FeArgs &a, hipStream_t st) {
  const size_t smem = (size_t)FeLayout<M, TPP, VEC>::BYTES;
  static bool configured = false;
  if (!configured) {
    if (hipFuncSetAttribute(reinterpret_cast<const void *>(&k_frontend<M, TPP, VEC>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem) != hipSuccess)
      return FMX_E_HIP;
    configured = true;
  }
  return fmx_launch(k_frontend<M, TPP, VEC>, dim3(a.C), dim3(256), smem, st, a);
}

} // namespace fmx

// The decimation factor is a host-known constant of the handle; expose
// explicit launchers so fmx_capi can pick the instantiation.
namespace fmx {
// steady state: whole 2048-sample chunks, full history, no complex
// decimator output, 16-B pilot rows, RDS rate ratio < 0.9 (<= 8 resampler
// outputs per thread and chunk) -> k_fe8
// k_fe8 takes any call of n >= FE8_MIN_N samples with n % 4 == 0 (chunks
// of one size, a multiple of 8, see k_fe8: the last chunk's length is n mod
// 8 off a multiple of 8, and its 16-B pilot stores and f16-pair history carry
// need a multiple of 4) on 16-B aligned IQ rows, cold or warm decimator
// history per channel; other n (e.g. 1025 at M = 8, where every n passes the
// IQ alignment test) take k_frontend
static bool fe8_ok(const FeArgs &a, int M) {
  if (a.in_mode != FE_IN_U8_DECIM) return false;
  const bool aligned = ((((uintptr_t)a.iq) | (uintptr_t)a.iq_stride) & 15) == 0 && ((2L * a.n * M) & 15) == 0;
  return aligned && a.n >= FE8_MIN_N && (a.n & 3) == 0 && a.do_demod && !a.bb_out &&
         (!a.pilot_out || ((((uintptr_t)a.pilot_out) | (uintptr_t)a.pilot_stride * 4) & 15) == 0) &&
         a.des_fs >= 190000;
}
bool frontend_is_fe8(const FeArgs &a, int M, int tpp) {
  return fe8_ok(a, M) && ((M == 10 && tpp == 28) || (M == 8 && tpp == 28) || (M == 4 && tpp == 20) ||
                               (M == 2 && tpp == 12));
}
int launch_frontend_m(const FeArgs &a, int M, int tpp, void *stream, bool vec) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (a.in_mode != FE_IN_U8_DECIM) return fe_launch<1, 1, false>(a, st);
  const bool fe8 = fe8_ok(a, M);
  vec = vec && ((((uintptr_t)a.iq) | (uintptr_t)a.iq_stride) & 15) == 0 && ((2L * a.n * M) & 15) == 0;
  if (fe8) {
    if (M == 10 && tpp == 28) return fe8_launch<10, 28>(a, st);
    if (M == 8 && tpp == 28) return fe8_launch<8, 28>(a, st);
    if (M == 4 && tpp == 20) return fe8_launch<4, 20>(a, st);
    if (M == 2 && tpp == 12) return fe8_launch<2, 12>(a, st);
  }
  if (M == 10 && tpp == 28) return vec ? fe_launch<10, 28, true>(a, st) : fe_launch<10, 28, false>(a, st);
  if (M == 8 && tpp == 28) return vec ? fe_launch<8, 28, true>(a, st) : fe_launch<8, 28, false>(a, st);
  if (M == 4 && tpp == 20) return vec ? fe_launch<4, 20, true>(a, st) : fe_launch<4, 20, false>(a, st);
  if (M == 2 && tpp == 12) return vec ? fe_launch<2, 12, true>(a, st) : fe_launch<2, 12, false>(a, st);
  return FMX_E_INVALID;
}

int launch_pll(const PllArgs &a, void *stream) {
  // 16 channels per workgroup while that leaves at least half the CUs
  // without one, else 24: eight waves, two per SIMD, and a third fewer
  // workgroups beside the other streams' (round 5: 4096 channels 0.635 ->
  // 0.618 ms per step, 8192 1.170 -> 1.134; at 2048 24 was 0.357 -> 0.363,
  // profiles/r05za_ab_pll_ch24.txt); the CU count is the handle's device's
  // (PllArgs::n_cu, queried once per handle at create)
  const int n_cu = a.n_cu > 0 ? a.n_cu : 256;
  hipStream_t st = static_cast<hipStream_t>(stream);
#ifndef FMX_PLL_CH_FORCE // A/B variants only
  const int ch = 2 * ((a.C + 15) / 16) <= n_cu ? 16 : 24;
#else
  const int ch = FMX_PLL_CH_FORCE;
#endif
  if (ch == 16) return fmx_launch(k_pll<16>, dim3((a.C + 15) / 16), dim3(64 * PLL_WAVES(16)), 0, st, a);
#if defined(FMX_PLL_CH_FORCE) && FMX_PLL_CH_FORCE != 16 && FMX_PLL_CH_FORCE != 24
  return fmx_launch(k_pll<FMX_PLL_CH_FORCE>, dim3((a.C + FMX_PLL_CH_FORCE - 1) / FMX_PLL_CH_FORCE),
                    dim3(64 * PLL_WAVES(FMX_PLL_CH_FORCE)), 0, st, a);
#endif
  return fmx_launch(k_pll<24>, dim3((a.C + 23) / 24), dim3(64 * PLL_WAVES(24)), 0, st, a);
}
int launch_audio(const AudioArgs &a, void *stream) {
  return fmx_launch(k_audio, dim3(a.C), dim3(256), sizeof(AuShared), static_cast<hipStream_t>(stream), a);
}
/* ================================================================== */
/* k_pilot: the 19 kHz pilot band-pass (stereo_decoder.cpp:229-230)    */
/* ================================================================== */
/* k_fe8's pilot stage as its own kernel on the front-end stream, after
 * k_fe8 (which then writes only the MPX and the stereo history rows).  In
 * k_fe8 the stage waited on one tap-fragment load per K step with two
 * workgroups (8 waves) per CU to hide it; here a workgroup is 6.3 KB of LDS
 * and 4 small waves, so many are resident and the loads overlap.  The sums
 * are k_fe8's: the same f16 hi / lo images of the same samples, the same
 * 8-aligned windows, the same three MFMAs per K step in the same order
 * (a tile of 256 outputs starts on a 256-sample boundary in both).
 * Workgroup = 4096 outputs of one channel (4 waves x 4 tiles of 16 x 16:
 * the fragments, 22 KB per K sweep from L2, are loaded once per 4 tiles); the
 * block -> (channel, segment) map keeps a channel's segments on one XCD, so
 * the window halo a neighbour loaded is an L2 hit. */
#define PIL_TPW 4                  // 256-output tiles per wave: one tap-fragment load feeds PIL_TPW MFMA chains
#define PIL_SEG (4 * 256 * PIL_TPW) // outputs per workgroup
#ifndef FMX_PILOT_QLDS
#define FMX_PILOT_QLDS 1 // A fragments from the LDS tap window (round 6; 0: pilot_frag from L2, A/B)
#endif
#define PIL_QP ((2 * FMX_PILOT_QN + 63) / 64) // 64-dword pieces of the [2][2][FMX_PILOT_QN] u16 window
struct PilLds {
  // sample s0 - FMX_HIST + i at [i]: the history (previous call's MPX rows
  // for s < 0), the segment, 32 zero-slack samples (read by K steps past the
  // filter, against zero taps)
  _Float16 xh[FMX_HIST + PIL_SEG + 32] __attribute__((aligned(16)));
  _Float16 xl[FMX_HIST + PIL_SEG + 32] __attribute__((aligned(16)));
  // the tap window FmxDesign::pilot_q16 ([copy][hi, lo][entry]; whole 64-dword
  // LDS-DMA pieces, the pad past it copies of its last dword)
  uint32_t q[FMX_PILOT_QLDS ? PIL_QP * 64 : 1] __attribute__((aligned(16)));
};
#ifndef FMX_PILOT_PRIO
#define FMX_PILOT_PRIO 0 // k_pilot's wave priority (s_setprio) beside the other streams' waves
#endif
__global__ __launch_bounds__(256) void k_pilot(PilotArgs a) {
  __shared__ PilLds L;
  if (FMX_PILOT_PRIO > 0) __builtin_amdgcn_s_setprio(FMX_PILOT_PRIO);
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
  typedef _Float16 f16x4_t __attribute__((ext_vector_type(4)));
  typedef float f32x4_t __attribute__((ext_vector_type(4)));
  const FmxDesign *__restrict__ D = a.des;
  const int nseg = (a.n + PIL_SEG - 1) / PIL_SEG;
  const int units = a.C * nseg;
  const int per = (units + 7) / 8; // units per XCD (workgroups go round-robin over the 8 XCDs)
  const int u = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  if (u >= units) return;
  const int c = u / nseg, s0 = (u % nseg) * PIL_SEG;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int P8 = fir8_len(D->pilot_len);
  const int KSP = D->pilot_ks;
  const float *mrow = a.mpx + (size_t)c * a.mpx_stride;
  const float *hrow = a.st_hist_rd + (size_t)c * FMX_HIST + FMX_HIST; // hrow[s], s < 0
  if (FMX_PILOT_QLDS) { // the tap window by LDS-DMA, ahead of the image loads (it lands before their wait)
    static_assert(FMX_PILOT_QN % 2 == 0, "dword window");
    const float *qs = reinterpret_cast<const float *>(&D->pilot_q16[0][0][0]);
    for (int p = wave; p < PIL_QP; p += 4)
      dma_dword(qs + min(64 * p + lane, 2 * FMX_PILOT_QN - 1), lds_addr(&L.q[64 * p]));
  }
  // the images from the window's first sample (8-aligned: P8 = 8k + 1), 4
  // samples per thread and pass
  const int i0 = FMX_HIST - (P8 - 1);
  // (every pass's loads issued before the first conversion)
  constexpr int NPASS = (FMX_HIST + PIL_SEG + 32 + 1023) / 1024;
  float4 v[NPASS];
#pragma unroll
  for (int q = 0; q < NPASS; ++q) {
    const int i = i0 + 4 * tid + 1024 * q, s = s0 - FMX_HIST + i;
    if (i >= FMX_HIST + PIL_SEG + 32) continue;
    if (a.vec && s >= 0 && s + 4 <= a.n) {
      v[q] = *reinterpret_cast<const float4 *>(mrow + s);
    } else {
      float w[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) w[k] = (s + k < 0) ? hrow[s + k] : (s + k < a.n ? mrow[s + k] : 0.0f);
      v[q] = make_float4(w[0], w[1], w[2], w[3]);
    }
  }
#pragma unroll
  for (int q = 0; q < NPASS; ++q) {
    const int i = i0 + 4 * tid + 1024 * q;
    if (i >= FMX_HIST + PIL_SEG + 32) continue;
    const float w[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
    f16x4_t hv, lv;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      hv[k] = (_Float16)w[k];
      lv[k] = (_Float16)(w[k] - (float)hv[k]);
    }
    *reinterpret_cast<f16x4_t *>(&L.xh[i]) = hv;
    *reinterpret_cast<f16x4_t *>(&L.xl[i]) = lv;
  }
  if (FMX_PILOT_QLDS) asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // the window's moves landed (before the barrier)
  __syncthreads();
  // tiles PIL_TPW w + u: 16 outputs (rows, A = taps, FmxDesign::pilot_frag)
  // of 16 blocks of 16 outputs (columns, B = MPX), K = P8 + 15 inputs
  const int col = lane & 15, g = lane >> 4;
  const int xb = FMX_HIST + 256 * PIL_TPW * wave + 16 * col - (P8 - 1) + 8 * g;
  const f16x8_t *bh = reinterpret_cast<const f16x8_t *>(&L.xh[xb]);
  const f16x8_t *bl = reinterpret_cast<const f16x8_t *>(&L.xl[xb]);
  const u32x4 *fa = reinterpret_cast<const u32x4 *>(&D->pilot_frag[0][0][0][0]) + lane;
  // (FMX_PILOT_QLDS) this lane's 8 window entries from 32 ks + 8 g + 15 - col:
  // in copy (15 - col) & 1 they start on an even entry, four dwords
  const int qb = 8 * g + 15 - col, qc = qb & 1;
  const uint32_t *qh = &L.q[0] + qc * FMX_PILOT_QN + (qb - qc) / 2;
  const uint32_t *ql = qh + FMX_PILOT_QN / 2;
  auto frag = [&](int ks, int s) __attribute__((always_inline)) {
    if (!FMX_PILOT_QLDS) return fa[128 * ks + 64 * s];
    const uint32_t *q = (s ? ql : qh) + 16 * ks;
    return u32x4{q[0], q[1], q[2], q[3]};
  };
  f32x4_t acc[PIL_TPW];
#pragma unroll
  for (int u = 0; u < PIL_TPW; ++u) acc[u] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
  u32x4 ah = frag(0, 0), al = frag(0, 1);
  for (int ks = 0; ks < KSP; ++ks) {
    const f16x8_t ahi = __builtin_bit_cast(f16x8_t, ah), alo = __builtin_bit_cast(f16x8_t, al);
    if (ks + 1 < KSP) {
      ah = frag(ks + 1, 0);
      al = frag(ks + 1, 1);
    }
#pragma unroll
    for (int u = 0; u < PIL_TPW; ++u) {
      const f16x8_t xhi = bh[32 * u + 4 * ks], xlo = bl[32 * u + 4 * ks]; // + 256 u + 32 ks samples
      acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, xhi, acc[u], 0, 0, 0);
      acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, xlo, acc[u], 0, 0, 0);
      acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo, xhi, acc[u], 0, 0, 0);
    }
  }
  // lane: outputs 16 col + 4 g + i of a tile's 256 (1 KB per store, contiguous)
  constexpr float kInv = 1.0f / 4096.0f;
#pragma unroll
  for (int u = 0; u < PIL_TPW; ++u) {
    const int o = s0 + 256 * (PIL_TPW * wave + u) + 16 * col + 4 * g;
    float *po = a.out + (size_t)c * a.out_stride + o;
    if (a.vec && o + 4 <= a.n) {
      *reinterpret_cast<float4 *>(po) =
          make_float4(acc[u][0] * kInv, acc[u][1] * kInv, acc[u][2] * kInv, acc[u][3] * kInv);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (o + k < a.n) po[k] = acc[u][k] * kInv;
    }
  }
}
int launch_pilot(const PilotArgs &a0, void *stream) {
  PilotArgs a = a0;
  if (a.C <= 0 || a.n <= 0) return FMX_OK;
  if (((a.des_pilot_len + 6) & ~7) > FMX_HIST) return FMX_E_INVALID; // the images' history holds the reach (fir8_len - 1)
  a.vec = ((((uintptr_t)a.mpx) | ((uintptr_t)a.mpx_stride * 4) | ((uintptr_t)a.out) | ((uintptr_t)a.out_stride * 4)) &
           15) == 0;
  const long units = (long)a.C * ((a.n + PIL_SEG - 1) / PIL_SEG);
  return fmx_launch(k_pilot, dim3((unsigned)(8 * ((units + 7) / 8))), dim3(256), 0, static_cast<hipStream_t>(stream), a);
}
/* ================================================================== */
/* k_rs: the RDS resampler 240k -> 171k (subcarrier.cpp:117-147) on MFMA */
/* ================================================================== */
/* Output e of a call is y_e = (1 - mu_e) y0_e + mu_e y1_e, with y0 / y1 the
 * 27-term dot products of the MPX window x[s_e .. s_e + 26] (s_e = i_e - 25,
 * one earlier at a boundary) with the entry's (branch, next branch) taps
 * (the pair table k_fe8 used).  Every channel of a handle follows one RDS
 * timing schedule (the RDS set is never reset per channel), so the windows
 * of 16 consecutive outputs form one band matrix A (16 rows, 27 nonzero
 * taps each) shared by all channels: v_mfma_f32_16x16x4f32 multiplies it,
 * 4 columns per K step, with the MPX of 16 channels (B = 4 samples x 16
 * channels).  FP32 products, sums in blocks of 4 (the reference sums
 * sequentially; k_fe8's FMA chains it replaces differed the same way, by a
 * few ulp).  One wave per workgroup; workgroup (x, y) takes channels
 * 16 x .. 16 x + 15 and the y-th contiguous run of 16-output tiles.  With it,
 * k_fe8 leaves out the resampler: a front end without it ran 0.777 against
 * 0.847 ms per pipelined step (profiles/r03h_ab_lds_history_nors.txt). */
#define RS_TMAX FMX_RS_TMAX // output tiles per workgroup at most (fmx_capi.cpp sizes parts)
// <= 96 VGPRs (five waves per SIMD): a k_rs wave beside two k_fe8 waves (168
// each) and a k_pll wave (80)
struct RsLds {
  float tab[FMX_NPFB + 1][FMX_RDS_RS_SUB + 1]; // branch rows, 27 terms oldest sample first
  // the tile's MPX window [buffer][channel][column-major samples - k0]:
  // 16.5 KB in all, so a k_rs workgroup fits beside two k_fe8 (52.4 KB each)
  // and one k_pll workgroup (31.2 KB) on a CU
  float xs[2][16][RS_XP] __attribute__((aligned(16)));
};
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(5))) void k_rs(RsArgs a) {
  // dynamic LDS (as k_rds): with a static size the backend sees an
  // LDS-limited occupancy and ignores the occupancy attribute's budget
  extern __shared__ __align__(16) unsigned char rs_smem[];
  RsLds &RL = *reinterpret_cast<RsLds *>(rs_smem);
  auto &tab = RL.tab;
  auto &xs = RL.xs;
  const int lane = threadIdx.x;
  const int c0 = blockIdx.x * 16;
  const FmxDesign *__restrict__ D = a.des;
  rs_fill_tab(tab, D, lane, 64);
  // one schedule for every channel (the RDS timing set is never reset per
  // channel: SubcarrierSet::reset leaves the resampler alone,
  // subcarrier.cpp:108; process_block launches k_rs only with one group)
  const int g = a.group[c0];
  const FmxSched *sched = a.sched + (size_t)g * a.sched_stride;
  const int ns = a.sched_n[g];
  const int ntile = (ns + 15) / 16;
  const int per = (ntile + a.parts - 1) / a.parts;
  const int ta = blockIdx.y * per, tb = min(ntile, ta + per);
  __syncthreads();
  // a tile's 16 schedule entries (rows past the call repeat the last), lane l
  // holding row l & 15, loaded from L2 two tiles ahead of their window's
  // load (round 6: no LDS staging of the workgroup's entries, so a workgroup
  // may take any number of tiles); row 0 / row 15 to the wave by readlane
  auto load_e = [&](int T) __attribute__((always_inline)) {
    return sched[min(16 * T + (lane & 15), ns - 1)];
  };
  const int r = lane & 15, kk = lane >> 4; // A: row r, K column kk; B: K row kk, channel column r
  // window loads: lane (channel lc, quarter lq) moves samples k0 + 16 lq .. + 15
  const int lc = lane >> 2, lq = lane & 3;
  const int cl = c0 + lc;
  const bool lcv = cl < a.C;
  const float *mrow = a.mpx + (size_t)(lcv ? cl : c0) * a.mpx_stride; // mrow[k], 0 <= k < n
  const float *wrow = a.win + (size_t)(lcv ? cl : c0) * 32 + 32;       // wrow[k], -32 <= k < 0
  auto load_w = [&](const FmxSched &e, float4 (&v)[4]) __attribute__((always_inline)) {
    rs_load_w(mrow, wrow, lcv, a.n, lq, rs_tile_k0(e), v);
  };
  auto store_w = [&](const FmxSched &e, int buf, const float4 (&v)[4]) __attribute__((always_inline)) {
    rs_store_w(xs[buf][lc], lcv, a.n, lq, rs_tile_k0(e), v);
  };
  auto tile = [&](int T, const FmxSched &en, int buf) __attribute__((always_inline)) {
    const rs_f32x4 acc = rs_tile(tab, xs[buf][r], en, kk);
    // D: lane (channel column r, output rows 4 kk .. 4 kk + 3)
    const int cb = c0 + r;
    if (cb < a.C) {
      float *dst = a.out + (size_t)cb * a.out_stride + 16 * T + 4 * kk;
      if (16 * T + 4 * kk + 3 < ns) {
        *reinterpret_cast<float4 *>(dst) = make_float4(acc[0], acc[1], acc[2], acc[3]);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (16 * T + 4 * kk + q < ns) dst[q] = acc[q];
      }
    }
  };
  // tile T's window is loaded at tile T-2 (registers), written to LDS at the
  // end of tile T-1: two register sets alternating (static indices)
  // (schedule entries: tiles T, T + 1 in e0c / e1c, T + 2, T + 3 in e0n / e1n)
  FmxSched e0c = load_e(ta), e1c = load_e(ta + 1), e0n = load_e(ta + 2), e1n = load_e(ta + 3);
  float4 wa[4], wb[4];
  if (ta < tb) load_w(e0c, wa);
  if (ta + 1 < tb) load_w(e1c, wb);
  if (ta < tb) store_w(e0c, 0, wa);
  for (int T = ta; T < tb; T += 2) {
    if (T + 2 < tb) load_w(e0n, wa);
    tile(T, e0c, 0);
    if (T + 1 < tb) store_w(e1c, 1, wb);
    if (T + 1 < tb) {
      if (T + 3 < tb) load_w(e1n, wb);
      tile(T + 1, e1c, 1);
      if (T + 2 < tb) store_w(e0n, 0, wa);
    }
    e0c = e0n;
    e1c = e1n;
    e0n = load_e(T + 4);
    e1n = load_e(T + 5);
  }
}

int launch_rs(const RsArgs &a, void *stream) {
  static_assert(sizeof(RsLds) <= 17 * 1024, "k_rs LDS");
  static_assert(RS_XS >= RS_KS && RS_XP >= 4 * RS_XS && RS_XS % 4 == 0, "k_rs window layout");
  return fmx_launch(k_rs, dim3((a.C + 15) / 16, a.parts), dim3(64), sizeof(RsLds), static_cast<hipStream_t>(stream), a);
}
int launch_rds_sym(const RdsArgs &a, void *stream) {
  // two k_fe8 workgroups (2 x 62.5 KB) leave 35 KB of a CU's 160 KB: several
  // k_rds workgroups fit beside them
  static_assert(sizeof(RdsLds) <= 16 * 1024, "k_rds LDS");
  static_assert(RDS_FOFF + sizeof(RdsFusedLds) <= 28 * 1024, "fused k_rds LDS");
#if FMX_RDS_FUSED
  if (a.fused)
    return fmx_launch(k_rds<true>, dim3((a.C + RDS_CPW - 1) / RDS_CPW), dim3(64), RDS_FOFF + sizeof(RdsFusedLds),
                      static_cast<hipStream_t>(stream), a);
#endif
  return fmx_launch(k_rds<false>, dim3((a.C + RDS_CPW - 1) / RDS_CPW), dim3(64), sizeof(RdsLds), static_cast<hipStream_t>(stream), a);
}
int launch_bits(const RdsArgs &a, void *stream) {
  static_assert(sizeof(BitsLds) <= 16 * 1024, "k_bits LDS");
  return fmx_launch(k_bits, dim3((a.C + 63) / 64), dim3(64), sizeof(BitsLds), static_cast<hipStream_t>(stream), a);
}
int launch_rds(const RdsArgs &a, void *stream) {
  // the bound events (set_launch_events): the start on k_rds, the stop on
  // k_bits, so that the timer and a completion event span both
  hipEvent_t e0 = t_ev_start, e1 = t_ev_stop;
  t_ev_start = t_ev_stop = nullptr;
  set_launch_events(e0, nullptr);
  int rc = launch_rds_sym(a, stream);
  if (rc != FMX_OK) return rc;
  set_launch_events(nullptr, e1);
  return launch_bits(a, stream);
}
// 16-B words src -> dst (the schedule upload from mapped pinned memory)
__global__ void k_copy16(const uint4 *src, uint4 *dst, size_t n16) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n16) dst[i] = src[i];
}
int launch_copy16(const void *src, void *dst, size_t n16, void *stream) {
  if (n16 == 0) return FMX_OK;
  hipLaunchKernelGGL(k_copy16, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint4 *>(src), static_cast<uint4 *>(dst), n16);
  return hipGetLastError() == hipSuccess ? FMX_OK : FMX_E_HIP;
}
int launch_iq_to_u8(const float *in, int in_stride, int C, int n, uint8_t *out, size_t out_stride, void *stream) {
  if (C <= 0 || n <= 0) return FMX_OK;
  hipLaunchKernelGGL(k_iq_to_u8, dim3((n + 255) / 256, C), dim3(256), 0, static_cast<hipStream_t>(stream), in,
                     in_stride, n, out, out_stride);
  return hipGetLastError() == hipSuccess ? FMX_OK : FMX_E_HIP;
}
// every channel whose ring is left to checkpoints: refilled (fmx_diag_rds_ring)
__global__ void k_ring_fill(ResetArgs a) {
  const int c = blockIdx.x;
  if (c >= a.C || a.rds[c].ring_ok || a.rds_prev == nullptr) return;
  rds_ring_fill(a.rds + c, a.rds_prev + (size_t)c * a.rds_stride, a.ring + (size_t)c * 2 * FMX_RDS_RING, threadIdx.x,
                blockDim.x);
  __syncthreads();
  if (threadIdx.x == 0) a.rds[c].ring_ok = 1;
}
int launch_ring_fill(const ResetArgs &a, void *stream) {
  hipLaunchKernelGGL(k_ring_fill, dim3(a.C), dim3(256), 0, static_cast<hipStream_t>(stream), a);
  return hipGetLastError() == hipSuccess ? FMX_OK : FMX_E_HIP;
}
int launch_reset(const ResetArgs &a, void *stream) {
  hipLaunchKernelGGL(k_reset, dim3(a.C), dim3(256), 0, static_cast<hipStream_t>(stream), a);
  return hipGetLastError() == hipSuccess ? FMX_OK : FMX_E_HIP;
}
int launch_reset_list(const ResetArgs &a, const ResetList &L, int parts, int st_buf, void *stream) {
  if (L.n <= 0) return FMX_OK;
  hipLaunchKernelGGL(k_reset_list, dim3(L.n), dim3(256), 0, static_cast<hipStream_t>(stream), a, L, parts, st_buf);
  return hipGetLastError() == hipSuccess ? FMX_OK : FMX_E_HIP;
}
int launch_synth(const fmx_synth_config &cfg, uint32_t ch0, int n_ch, int64_t sample0, int n_samples,
                 const uint8_t *bits, uint8_t *out, size_t out_stride, void *stream) {
  if (n_ch <= 0 || n_samples <= 0) return FMX_OK;
  dim3 grid((n_samples + 255) / 256, n_ch);
  hipLaunchKernelGGL(k_synth, grid, dim3(256), 0, static_cast<hipStream_t>(stream), cfg, ch0, n_ch, sample0,
                     n_samples, bits, out, out_stride);
  return hipGetLastError() == hipSuccess ? FMX_OK : FMX_E_HIP;
}
} // namespace fmx

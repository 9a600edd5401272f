// fmx_design.cpp -- host-side filter design and resampler timing for the
// MI355X FM demodulator.  Computes, once per handle, every constant the
// reference objects compute in their constructors and setters:
//
//   ComplexDecimator::init        src/dsp/liquid_primitives.cpp:370-403
//   FIRFilter::init (+center)     src/dsp/liquid_primitives.cpp:62-113
//   FMDemod ctor / setters        src/fm_demod.cpp:29-71, 99-147
//   StereoDecoder ctor            src/stereo_decoder.cpp:25-63, 98-117
//   AFPostProcessor               src/af_post_processor.cpp:7-45
//   SubcarrierSet ctor            src/redsea_port/dsp/subcarrier.cpp:94-106
//
// The liquid-dsp design routines they call (firdes_kaiser, rrcos, resamp
// prototype, symsync derivative filter) follow liquid's published algorithms
// (DESIGN.md section 3).  The resampler timing loop of resamp_rrrf is
// data-independent, so it is simulated here on the host and handed to the
// kernels as an output schedule.
//
// Compiled with -ffp-contract=off: the float sequences below must round
// exactly like the reference's.
#include "fmx_internal.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

namespace fmx {

static constexpr double kPiD = 3.14159265358979323846;
static constexpr float kPiF = 3.14159265358979323846f;

// IEEE binary16 <-> binary32 (round to nearest even) for the MFMA tap tables
static float f16_bits_to_f32(uint16_t h) {
  const int e = (h >> 10) & 31;
  const uint32_t m = h & 0x3FFu;
  float v;
  if (e == 0) v = std::ldexp(static_cast<float>(m), -24);
  else if (e == 31) v = m ? std::numeric_limits<float>::quiet_NaN() : std::numeric_limits<float>::infinity();
  else v = std::ldexp(static_cast<float>(m | 0x400u), e - 25);
  return (h & 0x8000u) ? -v : v;
}
static uint16_t f32_to_f16_bits(float f) {
  uint32_t x;
  std::memcpy(&x, &f, 4);
  const uint16_t sign = static_cast<uint16_t>((x >> 16) & 0x8000u);
  const uint32_t ax = x & 0x7FFFFFFFu;
  if (ax > 0x7F800000u) return sign | 0x7E00u;
  if (ax >= 0x477FF000u) return sign | 0x7C00u; // >= 65520 rounds to infinity
  if (ax <= 0x33000000u) return sign;           // <= 2^-25 rounds to zero
  const int e = static_cast<int>(ax >> 23) - 127;
  const uint32_t m = (ax & 0x7FFFFFu) | 0x800000u;
  const int shift = (e < -14) ? 13 + (-14 - e) : 13;
  uint32_t r = m >> shift;
  const uint32_t rem = m & ((1u << shift) - 1u), half = 1u << (shift - 1);
  if (rem > half || (rem == half && (r & 1u))) ++r;
  if (e < -14) return sign | static_cast<uint16_t>(r); // subnormal (a carry lands on the smallest normal)
  return sign | static_cast<uint16_t>((static_cast<uint32_t>(e + 15) << 10) + (r - 0x400u));
}

static float kaiser_beta_As(float As) {
  As = std::fabs(As);
  if (As > 50.0f) return 0.1102f * (As - 8.7f);
  if (As > 21.0f)
    return static_cast<float>(0.5842 * std::pow(static_cast<double>(As - 21.0f), 0.4) +
                              0.07886 * static_cast<double>(As - 21.0f));
  return 0.0f;
}

static double bessel_i0(double z) {
  if (z == 0.0) return 1.0;
  double y = 0.0, t = 1.0, h = 0.5 * z;
  for (int k = 0; k < 64; ++k) {
    if (k > 0) t *= h / k;
    y += t * t;
  }
  return y;
}

void firdes_kaiser(unsigned n, float fc, float As, float mu, float *h) {
  const double beta = kaiser_beta_As(As);
  const double i0b = bessel_i0(beta);
  for (unsigned i = 0; i < n; ++i) {
    const double t = static_cast<double>(i) - static_cast<double>(n - 1) / 2.0 + mu;
    const double x = 2.0 * fc * t;
    const double s = (std::fabs(x) < 1e-12) ? 1.0 : std::sin(kPiD * x) / (kPiD * x);
    const double tw = static_cast<double>(i) - static_cast<double>(n - 1) / 2.0;
    const double r = 2.0 * tw / static_cast<double>(n);
    const double w = bessel_i0(beta * std::sqrt(std::max(0.0, 1.0 - r * r))) / i0b;
    h[i] = static_cast<float>(s * w);
  }
}

static void firdes_rrcos(unsigned k, unsigned m, float beta, float *h) {
  const unsigned n = 2 * k * m + 1;
  const double b = beta;
  for (unsigned i = 0; i < n; ++i) {
    const double t = static_cast<double>(i) / k - static_cast<double>(m);
    double v;
    if (std::fabs(t) < 1e-3) {
      v = 1.0 - b + 4.0 * b / kPiD;
    } else if (std::fabs(1.0 - 16.0 * b * b * t * t) < 1e-3) {
      v = (b / std::sqrt(2.0)) * ((1.0 + 2.0 / kPiD) * std::sin(kPiD / (4.0 * b)) +
                                  (1.0 - 2.0 / kPiD) * std::cos(kPiD / (4.0 * b)));
    } else {
      const double num = std::cos((1.0 + b) * kPiD * t) * 4.0 * b / kPiD +
                         std::sin((1.0 - b) * kPiD * t) / (kPiD * t);
      v = num / (1.0 - 16.0 * b * b * t * t);
    }
    h[i] = static_cast<float>(v);
  }
}

// FIRFilter::init(length, cutoff, As, center) -> taps + scale
static void design_fir(float *taps, float &scale, unsigned length, float cutoff, float As, float center) {
  firdes_kaiser(length, cutoff, As, 0.0f, taps);
  if (std::fabs(center) < 1e-6f) {
    scale = 2.0f * cutoff;
    return;
  }
  const int mid = static_cast<int>(length / 2);
  constexpr float kTwoPi = 6.28318530717958647692f;
  for (unsigned n = 0; n < length; ++n) {
    const float phase = kTwoPi * center * static_cast<float>(static_cast<int>(n) - mid);
    taps[n] = 2.0f * taps[n] * std::cos(phase);
  }
  double sumAbs = 0.0;
  for (unsigned n = 0; n < length; ++n) sumAbs += std::fabs(taps[n]);
  if (sumAbs > 1e-12) {
    const float inv = static_cast<float>(1.0 / sumAbs);
    for (unsigned n = 0; n < length; ++n) taps[n] *= inv;
  }
  scale = 1.0f;
}

// resamp_rrrf prototype: 2*m*npfb+1 Kaiser taps at fc/npfb, gain npfb/sum;
// the filter bank uses the first 2*m*npfb taps, branch b = proto[b + n*npfb].
static void design_resamp(unsigned m, float fc, float As, unsigned npfb, float *branch_major,
                          std::vector<float> *proto_out) {
  const unsigned n = 2 * m * npfb + 1;
  std::vector<float> hf(n);
  firdes_kaiser(n, fc / static_cast<float>(npfb), As, 0.0f, hf.data());
  float gain = 0.0f;
  for (unsigned i = 0; i < n; ++i) gain += hf[i];
  gain = static_cast<float>(npfb) / gain;
  std::vector<float> h(n);
  for (unsigned i = 0; i < n; ++i) h[i] = hf[i] * gain;
  const unsigned sub = (n - 1) / npfb;
  for (unsigned b = 0; b < npfb; ++b)
    for (unsigned k = 0; k < sub; ++k) branch_major[b * sub + k] = h[b + k * npfb];
  if (proto_out) *proto_out = h;
}

// liquid nco_crcf phase/frequency constrain (fixed-point NCO)
uint32_t nco_constrain(float theta) {
  const float p = static_cast<float>(static_cast<double>(theta) * 0.159154943091895);
  float fpart = p - std::trunc(p);
  if (fpart < 0.0f) fpart = static_cast<float>(static_cast<double>(fpart) + 1.0);
  const float s = fpart * 4294967296.0f;
  if (s >= 4294967296.0f) return 0u;
  return static_cast<uint32_t>(s);
}

static const int kXdrFmBwHz[30] = {309000, 298000, 281000, 263000, 246000, 229000, 211000, 194000,
                                   177000, 159000, 142000, 125000, 108000, 95000,  90000,  83000,
                                   73000,  63000,  55000,  48000,  42000,  36000,  32000,  27000,
                                   24000,  20000,  17000,  15000,  9000,   0};

int bandwidth_select(int bw_hz, int w0) {
  const int eff = (bw_hz <= 0) ? w0 : bw_hz;
  int selected = 29;
  if (eff > 0) {
    int minDiff = std::numeric_limits<int>::max();
    for (int i = 0; i < 29; ++i) {
      const int diff = std::abs(kXdrFmBwHz[i] - eff);
      if (diff < minDiff) {
        minDiff = diff;
        selected = i;
      }
    }
  }
  return selected;
}

int tef_bandwidth_hz(int mode) {
  static const int kTef[] = {311000, 287000, 254000, 236000, 217000, 200000, 184000, 168000, 151000,
                             133000, 114000, 97000,  84000,  72000,  64000,  56000,  0};
  return kTef[std::clamp(mode, 0, 16)];
}

int design_build(const fmx_config &cfg, FmxDesign *d, DesignExtras *ex, std::string *err) {
  std::memset(d, 0, sizeof(*d));
  if (cfg.dsp_rate <= 0 || cfg.iq_rate <= 0 || cfg.out_rate <= 0 || cfg.iq_rate % cfg.dsp_rate != 0) {
    *err = "iq_rate must be a positive integer multiple of dsp_rate";
    return FMX_E_INVALID;
  }
  const int M = cfg.iq_rate / cfg.dsp_rate;
  const int fs = cfg.dsp_rate;
  d->M = M;
  d->fs = fs;
  d->out_rate = cfg.out_rate;
  d->block = cfg.block;
  // ---- ComplexDecimator: main.cpp:670-674 ----
  const unsigned tpp = (M >= 8) ? 28u : ((M >= 4) ? 20u : 12u);
  d->dec_tpp = static_cast<int>(std::max(4u, tpp));
  d->dec_len = (M > 1) ? M * d->dec_tpp : 1;
  if (d->dec_len > FMX_MAX_DEC) {
    *err = "decimation factor too large";
    return FMX_E_INVALID;
  }
  if (M > 1) {
    const float cutoff = std::clamp(0.45f / static_cast<float>(M), 0.01f, 0.45f);
    firdes_kaiser(static_cast<unsigned>(d->dec_len), cutoff, 80.0f, 0.0f, d->dec_taps_raw);
    d->dec_scale = 2.0f * cutoff;
    constexpr float kScale = 1.0f / 127.5f;
    for (int i = 0; i < d->dec_len; ++i) d->dec_taps[i] = d->dec_taps_raw[i] * kScale;
    for (int p = 0; p < M; ++p)
      for (int q = 0; q < d->dec_tpp; ++q) d->dec_poly[p * d->dec_tpp + q] = d->dec_taps[q * M + p];
    for (int i = 0; i < d->dec_len; ++i) d->dec_pad[FMX_DEC_PAD + i] = d->dec_taps[i];
    double dc = 0.0;
    for (int i = 0; i < d->dec_len; ++i) dc += static_cast<double>(d->dec_taps[i]);
    d->dec_dc = static_cast<float>(127.5 * dc);
    // f16 MFMA decimator tables (k_fe8): taps x 2^16, reversed, as f16 hi +
    // lo in the A-fragment layout
    const int L = d->dec_len;
    const int KS = (15 * M + L + 1 + 31) / 32;
    if (KS > FMX_DEC_KS_MAX) {
      *err = "decimator too long for the MFMA fragment table";
      return FMX_E_INVALID;
    }
    for (int ks = 0; ks < FMX_DEC_KS_MAX; ++ks)
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 8; ++j) {
          const int dd = 32 * ks + 8 * (l >> 4) + j - M * (l & 15);
          const float q = (ks < KS && dd >= 1 && dd <= L) ? d->dec_taps[L - dd] * 65536.0f : 0.0f;
          const uint16_t hi = f32_to_f16_bits(q);
          d->dec_frag[ks][0][l][j] = hi;
          d->dec_frag[ks][1][l][j] = f32_to_f16_bits(q - f16_bits_to_f32(hi));
        }
    for (int i = 0; i < FMX_DEC_QN; ++i) {
      const int dd = i - 15 * M;
      const float q = (dd >= 1 && dd <= L) ? d->dec_taps[L - dd] * 65536.0f : 0.0f;
      const uint16_t hi = f32_to_f16_bits(q);
      d->dec_q16[0][i] = hi;
      d->dec_q16[1][i] = f32_to_f16_bits(q - f16_bits_to_f32(hi));
    }
    d->dec_dc16 = static_cast<float>(-0.5 * 65536.0 * dc);
    d->dec_scale16 = d->dec_scale * (1.0f / 65536.0f);
  } else {
    d->dec_scale = 1.0f;
    d->dec_dc = 0.0f;
  }
  // ---- FMDemod IQ filters ----
  for (int i = 0; i < 30; ++i) {
    const int sel = kXdrFmBwHz[i];
    const double head = 0.45 * static_cast<double>(fs);
    const double cut = (sel > 0) ? std::clamp(static_cast<double>(sel) * 0.5, 9000.0, head) : head;
    const float cn = std::clamp(static_cast<float>(cut / static_cast<double>(fs)), 0.01f, 0.45f);
    const unsigned len = (sel > 0 && sel <= 73000) ? 121U : 81U;
    const float As = (sel > 0 && sel <= 42000) ? 70.0f : 60.0f;
    d->iq_len[i] = static_cast<int>(len);
    design_fir(d->iq_taps[i], d->iq_scale[i], len, cn, As, 0.0f);
  }
  {
    const float cn = std::clamp(110000.0f / static_cast<float>(fs), 0.01f, 0.45f);
    d->iq_len[FMX_IQ_CTOR] = 81;
    design_fir(d->iq_taps[FMX_IQ_CTOR], d->iq_scale[FMX_IQ_CTOR], 81, cn, 60.0f, 0.0f);
  }
  {
    const float kf = static_cast<float>(75000.0 / static_cast<double>(fs));
    d->fd_ref = static_cast<float>(1.0 / (2.0 * kPiD * static_cast<double>(kf)));
  }
  for (int k = 0; k < 2; ++k) {
    const int us = (k == 0) ? 50 : 75;
    const float tau = static_cast<float>(us) * 1e-6f;
    const float dt = 1.0f / static_cast<float>(cfg.out_rate);
    d->deemph_alpha[k] = dt / (tau + dt);
  }
  // ---- StereoDecoder ----
  {
    int taps = static_cast<int>(std::ceil(3.8 * static_cast<double>(fs) / 3000.0));
    taps = std::clamp(taps, 63, 511);
    if ((taps % 2) == 0) taps++;
    const float centerNorm = std::clamp(19000.0f / static_cast<float>(fs), 0.001f, 0.49f);
    const float cutNorm = std::clamp(250.0f / static_cast<float>(fs), 0.0005f, 0.45f);
    float sc = 1.0f;
    design_fir(d->pilot_taps, sc, static_cast<unsigned>(taps), cutNorm, 60.0f, centerNorm);
    d->pilot_len = taps;
    d->delay_len = std::max(1, std::max(0, (taps - 1) / 2) + 1);
    const float audioCut = std::clamp(15000.0f / static_cast<float>(fs), 0.01f, 0.45f);
    design_fir(d->lr_taps, d->lr_scale, FMX_LR_LEN, audioCut, 60.0f, 0.0f);
    d->nominal = 2.0f * kPiF * 19000.0f / static_cast<float>(fs);
    d->pll_min = 2.0f * kPiF * 18750.0f / static_cast<float>(fs);
    d->pll_max = 2.0f * kPiF * 19250.0f / static_cast<float>(fs);
    d->pll_alpha = 0.01f;
    d->pll_beta = std::sqrt(0.01f);
    d->pll_dtheta0 = nco_constrain(d->nominal);
    const float atk[3] = {0.090f, 0.120f, 0.180f};
    const float rel[3] = {0.040f, 0.030f, 0.015f};
    const float gate[3] = {0.75f, 0.85f, 0.95f};
    for (int m = 0; m < 3; ++m) {
      d->blend_attack[m] = 1.0f - std::exp(-1.0f / (atk[m] * static_cast<float>(fs)));
      d->blend_release[m] = 1.0f - std::exp(-1.0f / (rel[m] * static_cast<float>(fs)));
      d->gate[m] = gate[m];
    }
  }
  // ---- resamplers ----
  std::vector<float> proto_af, proto_rds;
  design_resamp(12, 0.47f, 60.0f, FMX_NPFB, d->af_h, &proto_af);
  design_resamp(13, 0.47f, 60.0f, FMX_NPFB, d->rds_rs_h, &proto_rds);
  {
    const float ratio = static_cast<float>(cfg.out_rate) / static_cast<float>(fs);
    if (ratio < 0.005f || ratio > 8.0f) {
      *err = "audio resampler ratio out of range";
      return FMX_E_INVALID;
    }
    d->af_del = 1.0f / ratio;
    const float rr = 171000.0f / static_cast<float>(fs);
    if (rr < 0.005f || rr > 2.0f) {
      *err = "RDS resampler ratio out of range";
      return FMX_E_INVALID;
    }
    d->rds_del = 1.0f / rr;
  }
  // ---- RDS subcarrier ----
  {
    constexpr float kTarget = 171000.0f;
    float sc = 1.0f;
    design_fir(d->rds_fir, sc, FMX_RDS_FIR, 2400.0f / kTarget, 60.0f, 0.0f);
    d->rds_fir_scale = sc;
    for (int jp = 0; jp < FMX_RDS_DECIM; ++jp)
      for (int i = 0; i < 12; ++i) {
        const int k = jp + FMX_RDS_DECIM * i;
        d->rds_rows[jp][i] = (i < FMX_RDS_NACC && k < FMX_RDS_FIR) ? d->rds_fir[k] : 0.0f;
      }
    d->agc_bw = 500.0f / kTarget;
    d->agc_g0 = 0.08f;
    const float k2Pi = 2.f * kPiF;
    d->rds_dtheta0 = nco_constrain(57000.f * k2Pi / kTarget);
    d->rds_alpha = 0.03f / kTarget;
    d->rds_beta = std::sqrt(d->rds_alpha);
    // symsync_crcf_create_rnyquist(RRC, k=3, m=3, beta=0.8, 32)
    const unsigned hlen = 2 * 32 * 3 * 3 + 1;
    std::vector<float> h(hlen), dh(hlen);
    firdes_rrcos(32 * 3, 3, 0.8f, h.data());
    float hdh_max = 0.0f;
    for (unsigned i = 0; i < hlen; ++i) {
      if (i == 0) dh[i] = h[i + 1] - h[hlen - 1];
      else if (i == hlen - 1) dh[i] = h[0] - h[i - 1];
      else dh[i] = h[i + 1] - h[i - 1];
      if (std::fabs(h[i] * dh[i]) > hdh_max || i == 0) hdh_max = std::fabs(h[i] * dh[i]);
    }
    for (unsigned i = 0; i < hlen; ++i) dh[i] *= 0.06f / hdh_max;
    for (unsigned b = 0; b < FMX_NPFB; ++b)
      for (unsigned k = 0; k < FMX_SS_SUB; ++k) {
        d->ss_mf[b * FMX_SS_SUB + k] = h[b + k * FMX_NPFB];
        d->ss_dmf[b * FMX_SS_SUB + k] = dh[b + k * FMX_NPFB];
      }
    // symsync_set_lf_bw(2200/171000)
    const float bt = 2200.0f / kTarget;
    const float alpha = 1.000f - bt;
    const float beta = 0.220f * bt;
    const float A0 = 1.00f - 0.500f * alpha;
    const float A1 = -0.495f * alpha;
    const float A2 = 0.0f;
    d->ss_b0 = beta / A0;
    d->ss_a1 = A1 / A0;
    d->ss_a2 = A2 / A0;
    d->ss_rate_adj = static_cast<float>(0.5 * static_cast<double>(bt));
    const float alphaPsk = static_cast<float>(kPiD / 2.0);
    const float arg = 1.0f * 2.0f * alphaPsk;
    d->psk_xr1 = std::cos(arg);
    d->psk_xi1 = std::sin(arg);
    if (ex) {
      ex->rrc = h;
      ex->rrc_d = dh;
    }
  }
  for (int i = 0; i < FMX_IQ_DESIGNS; ++i)
    for (int k = 0; k < d->iq_len[i]; ++k) d->iq_pad[i][k + 5] = d->iq_taps[i][k];
  for (int i = 0; i < FMX_IQ_DESIGNS; ++i)
    for (int k = 0; k < d->iq_len[i]; ++k) d->iq_z16[i][k + 16] = d->iq_taps[i][k];
  for (int i = 0; i < FMX_IQ_DESIGNS; ++i) {
    // MFMA IQ FIR fragments (k_fe8), as the pilot BPF's below
    const int P = d->iq_len[i], P8 = ((P + 6) & ~7) + 1;
    d->iq_ks[i] = (P8 + 15 + 31) / 32;
    for (int ks = 0; ks < FMX_IQ_KS_MAX; ++ks)
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 8; ++j) {
          const int dd = 32 * ks + 8 * (l >> 4) + j - (l & 15);
          const int k = P8 - 1 - dd;
          const float q = (ks < d->iq_ks[i] && k >= 0 && k < P) ? d->iq_taps[i][k] * 4096.0f : 0.0f;
          const uint16_t hi = f32_to_f16_bits(q);
          d->iq_frag[i][ks][0][l][j] = hi;
          d->iq_frag[i][ks][1][l][j] = f32_to_f16_bits(q - f16_bits_to_f32(hi));
        }
    for (int c = 0; c < 2; ++c)
      for (int e = 0; e < FMX_IQ_QN; ++e) {
        const int dd = e + c - 15;
        const int k = P8 - 1 - dd;
        const float q = (dd < 32 * d->iq_ks[i] && k >= 0 && k < P) ? d->iq_taps[i][k] * 4096.0f : 0.0f;
        const uint16_t hi = f32_to_f16_bits(q);
        d->iq_q16[i][c][0][e] = hi;
        d->iq_q16[i][c][1][e] = f32_to_f16_bits(q - f16_bits_to_f32(hi));
      }
  }
  for (int k = 0; k < d->pilot_len; ++k) d->pilot_z16[k + 16] = d->pilot_taps[k];
  for (int k = 0; k < d->pilot_len; ++k) d->pilot_pad[k + 5] = d->pilot_taps[k];
  {
    // MFMA pilot BPF fragments (k_fe8): taps * 2^12 (all f16-normal), hi/lo split
    const int P = d->pilot_len, P8 = ((P + 6) & ~7) + 1;
    d->pilot_ks = (P8 + 15 + 31) / 32;
    for (int ks = 0; ks < FMX_PILOT_KS_MAX; ++ks)
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 8; ++j) {
          const int dd = 32 * ks + 8 * (l >> 4) + j - (l & 15);
          const int k = P8 - 1 - dd;
          const float q = (ks < d->pilot_ks && k >= 0 && k < P) ? d->pilot_taps[k] * 4096.0f : 0.0f;
          const uint16_t hi = f32_to_f16_bits(q);
          d->pilot_frag[ks][0][l][j] = hi;
          d->pilot_frag[ks][1][l][j] = f32_to_f16_bits(q - f16_bits_to_f32(hi));
        }
    for (int c = 0; c < 2; ++c)
      for (int i = 0; i < FMX_PILOT_QN; ++i) {
        const int dd = i + c - 15;
        const int k = P8 - 1 - dd;
        const float q = (dd < 32 * d->pilot_ks && k >= 0 && k < P) ? d->pilot_taps[k] * 4096.0f : 0.0f;
        const uint16_t hi = f32_to_f16_bits(q);
        d->pilot_q16[c][0][i] = hi;
        d->pilot_q16[c][1][i] = f32_to_f16_bits(q - f16_bits_to_f32(hi));
      }
  }
  for (int k = 0; k + 1 < FMX_PILOT_MAX + FMX_PAD; ++k) {
    d->pilot_pair[k][0] = d->pilot_pad[k];
    d->pilot_pair[k][1] = d->pilot_pad[k + 1];
  }
  for (int k = 0; k < FMX_LR_LEN; ++k) d->lr_pad[k + 5] = d->lr_taps[k];
  {
    // MFMA L/R FIR fragments (k_audio): taps * 2^12, hi/lo split; P = 121 is
    // already 8k + 1, so the window starts 120 samples before the output
    constexpr int P = FMX_LR_LEN, P8 = P;
    static_assert((P8 + 15 + 31) / 32 == FMX_LR_KS, "L/R FIR K steps");
    for (int ks = 0; ks < FMX_LR_KS; ++ks)
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 8; ++j) {
          const int dd = 32 * ks + 8 * (l >> 4) + j - (l & 15);
          const int k = P8 - 1 - dd;
          const float q = (k >= 0 && k < P) ? d->lr_taps[k] * 4096.0f : 0.0f;
          const uint16_t hi = f32_to_f16_bits(q);
          d->lr_frag[ks][0][l][j] = hi;
          d->lr_frag[ks][1][l][j] = f32_to_f16_bits(q - f16_bits_to_f32(hi));
        }
    for (int c = 0; c < 2; ++c)
      for (int e = 0; e < FMX_LR_QN; ++e) {
        const int k = P8 - 1 - (e + c - 15);
        const float q = (k >= 0 && k < P) ? d->lr_taps[k] * 4096.0f : 0.0f;
        const uint16_t hi = f32_to_f16_bits(q);
        d->lr_q16[c][0][e] = hi;
        d->lr_q16[c][1][e] = f32_to_f16_bits(q - f16_bits_to_f32(hi));
      }
  }
  for (int k = 0; k + 1 < FMX_LR_LEN + FMX_PAD; ++k) {
    d->lr_pair[k][0] = d->lr_pad[k];
    d->lr_pair[k][1] = d->lr_pad[k + 1];
  }
  if (ex) {
    ex->proto_af = proto_af;
    ex->proto_rds = proto_rds;
  }
  return FMX_OK;
}

/* ---- resamp_rrrf timing (float tau, interp/boundary states) ---- */
void timing_reset(ResampTiming &t) {
  t.tau = 0.0f;
  t.bf = 0.0f;
  t.b = 0;
  t.mu = 0.0f;
  t.state = 0;
}

static inline void timing_update(ResampTiming &t) {
  t.tau += t.del;
  t.bf = t.tau * static_cast<float>(FMX_NPFB);
  t.b = static_cast<int>(std::floor(t.bf));
  t.mu = t.bf - static_cast<float>(t.b);
}

int timing_run(ResampTiming &t, int n_in, FmxSched *out, int cap) {
  int n = 0;
  const int npfb = FMX_NPFB;
  for (int i = 0; i < n_in; ++i) {
    while (t.b < npfb) {
      if (t.state == 1) {
        if (out && n < cap) {
          out[n].packed = i | ((npfb - 1) << 16) | (1 << 24);
          out[n].mu = t.mu;
        }
        n++;
        timing_update(t);
        t.state = 0;
      } else {
        if (t.b == npfb - 1) {
          t.state = 1;
          t.b = npfb;
        } else {
          if (out && n < cap) {
            out[n].packed = i | (t.b << 16);
            out[n].mu = t.mu;
          }
          n++;
          timing_update(t);
        }
      }
    }
    t.tau -= 1.0f;
    t.bf -= static_cast<float>(npfb);
    t.b -= npfb;
  }
  return n;
}

bool timing_equal(const ResampTiming &a, const ResampTiming &b) {
  return a.tau == b.tau && a.bf == b.bf && a.b == b.b && a.mu == b.mu && a.state == b.state &&
         a.del == b.del;
}

} // namespace fmx

/*
 * fmx_oracle.cpp -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the per-channel FM demod hot path of bkram/fmtuner-sdr
 * (fm-sdr-tuner v1.3.0).  It is the parity checker for the HIP path and the
 * timed CPU baseline ("kind": "port") of bench.py; nothing in the product
 * (fmtuner-sdr_amd/) links or calls it.
 *
 * Structure:
 *   namespace lq   -- restatement of the liquid-dsp objects the reference calls
 *                     (SURVEY.md 2.1).  liquid-dsp is NOT in this image and its
 *                     version is unpinned by the reference, so each object
 *                     follows liquid's published algorithm with the choices
 *                     written down in DESIGN.md section 3 ("parity unpinned"
 *                     against a real liquid build).
 *   namespace ref  -- the reference's own classes restated line by line:
 *                     ComplexDecimator (src/dsp/liquid_primitives.cpp:370-499),
 *                     FMDemod (src/fm_demod.cpp), StereoDecoder
 *                     (src/stereo_decoder.cpp), AFPostProcessor
 *                     (src/af_post_processor.cpp), SubcarrierSet
 *                     (src/redsea_port/dsp/subcarrier.cpp), BlockStream
 *                     (src/redsea_port/block_sync.cpp), RDSDecoder
 *                     (src/rds_decoder.cpp) and the per-block body of
 *                     main.cpp:1232-1308.
 *
 * Build with -ffp-contract=off: the reference (liquid built for generic x86-64)
 * rounds every product and sum separately.
 */
#include "fmx_oracle.h"

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <complex>
#include <cstdint>
#include <cstring>
#include <functional>
#include <limits>
#include <memory>
#include <stdexcept>
#include <thread>
#include <vector>

using cf = std::complex<float>;

namespace lq {

constexpr double kPiD = 3.14159265358979323846;

/* ---------------- filter design (liquid firdes.c / window.c) ------------- */
// kaiser_beta_As: [Vaidyanathan:1993] as used by liquid_firdes_kaiser.
static float kaiser_beta_As(float As) {
  As = std::fabs(As);
  if (As > 50.0f) return 0.1102f * (As - 8.7f);
  if (As > 21.0f)
    return static_cast<float>(0.5842 * std::pow(static_cast<double>(As - 21.0f), 0.4) +
                              0.07886 * static_cast<double>(As - 21.0f));
  return 0.0f;
}
// I0 by its power series, evaluated in double (liquid evaluates a log-gamma
// form in float; DESIGN.md 3: taps agree to ~1e-6 relative).
static double besseli0(double z) {
  if (z == 0.0) return 1.0;
  double y = 0.0, t = 1.0, h = 0.5 * z;
  for (int k = 0; k < 64; ++k) {
    if (k > 0) t *= h / k;
    y += t * t;
  }
  return y;
}
// liquid_kaiser(i, wlen, beta): r = 2t/wlen with t = i - (wlen-1)/2.
static double kaiser(unsigned i, unsigned n, double beta) {
  double t = static_cast<double>(i) - static_cast<double>(n - 1) / 2.0;
  double r = 2.0 * t / static_cast<double>(n);
  double a = besseli0(beta * std::sqrt(std::max(0.0, 1.0 - r * r)));
  return a / besseli0(beta);
}
static double sinc(double x) {
  if (std::fabs(x) < 1e-12) return 1.0;
  return std::sin(kPiD * x) / (kPiD * x);
}
// liquid_firdes_kaiser(n, fc, As, mu, h): h[i] = sinc(2 fc t) * kaiser, no
// normalisation.  Evaluated in double, rounded to float once.
void firdes_kaiser(unsigned n, float fc, float As, float mu, float *h) {
  double beta = kaiser_beta_As(As);
  for (unsigned i = 0; i < n; ++i) {
    double t = static_cast<double>(i) - static_cast<double>(n - 1) / 2.0 + mu;
    h[i] = static_cast<float>(sinc(2.0 * fc * t) * kaiser(i, n, beta));
  }
}
// liquid_firdes_rrcos(k, m, beta, dt, h): square-root raised cosine, length
// 2km+1, unnormalised (h(0) = 1 - beta + 4 beta / pi).
void firdes_rrcos(unsigned k, unsigned m, float beta, float dt, float *h) {
  unsigned n = 2 * k * m + 1;
  double b = beta;
  for (unsigned i = 0; i < n; ++i) {
    double t = static_cast<double>(i) / k - static_cast<double>(m) + dt;
    double v;
    if (std::fabs(t) < 1e-3) {
      v = 1.0 - b + 4.0 * b / kPiD;
    } else if (std::fabs(1.0 - 16.0 * b * b * t * t) < 1e-3) {
      v = (b / std::sqrt(2.0)) * ((1.0 + 2.0 / kPiD) * std::sin(kPiD / (4.0 * b)) +
                                  (1.0 - 2.0 / kPiD) * std::cos(kPiD / (4.0 * b)));
    } else {
      double num = std::cos((1.0 + b) * kPiD * t) * 4.0 * b / kPiD +
                   std::sin((1.0 - b) * kPiD * t) / (kPiD * t);
      v = num / (1.0 - 16.0 * b * b * t * t);
    }
    h[i] = static_cast<float>(v);
  }
}

/* ---------------- dot products (liquid dotprod portable order) ----------- */
// window w holds oldest..newest; h_rev = taps reversed; sequential order.
static inline cf dot_cf(const float *hrev, const cf *w, unsigned n) {
  float re = 0.0f, im = 0.0f;
  for (unsigned i = 0; i < n; ++i) {
    float pr = hrev[i] * w[i].real();
    float pi = hrev[i] * w[i].imag();
    re = re + pr;
    im = im + pi;
  }
  return cf(re, im);
}
static inline float dot_rf(const float *hrev, const float *w, unsigned n) {
  float r = 0.0f;
  for (unsigned i = 0; i < n; ++i) {
    float p = hrev[i] * w[i];
    r = r + p;
  }
  return r;
}

/* linear window: keeps last n samples, oldest first (liquid window/wdelay).
 * Like liquid's windowcf, the buffer is longer than the window (n + slack)
 * and the live n samples are shifted back to the front only when the write
 * position reaches the end: O(1) amortised per push, same contents. */
template <typename T> struct Window {
  std::vector<T> buf;
  unsigned n = 0, rd = 0, cap = 0;
  void init(unsigned len) {
    n = len;
    cap = len + std::max(len, 256u);
    buf.assign(cap, T{});
    rd = 0;
  }
  void reset() {
    std::fill(buf.begin(), buf.end(), T{});
    rd = 0;
  }
  void push(T x) {
    if (n == 0) return;
    if (rd + n == cap) {
      std::memmove(buf.data(), buf.data() + rd + 1, (n - 1) * sizeof(T));
      rd = 0;
      buf[n - 1] = x;
      return;
    }
    rd++;
    buf[rd + n - 1] = x;
  }
  const T *data() const { return buf.data() + rd; }
};

/* firfilt_crcf: y = scale * sum_i h[i] x[t-i] */
struct FirFiltCrcf {
  std::vector<float> hrev;
  Window<cf> w;
  float scale = 1.0f;
  void create(const float *h, unsigned n) {
    hrev.resize(n);
    for (unsigned i = 0; i < n; ++i) hrev[i] = h[n - 1 - i];
    w.init(n);
    scale = 1.0f;
  }
  void reset() { w.reset(); }
  void push(cf x) { w.push(x); }
  cf execute() const {
    cf y = dot_cf(hrev.data(), w.data(), static_cast<unsigned>(hrev.size()));
    return cf(y.real() * scale, y.imag() * scale);
  }
  unsigned length() const { return static_cast<unsigned>(hrev.size()); }
};

/* firdecim_crcf: output computed after pushing sample 0 of each M-block */
struct FirDecimCrcf {
  unsigned M = 1;
  std::vector<float> hrev;
  Window<cf> w;
  float scale = 1.0f;
  void create(unsigned m, const float *h, unsigned n) {
    M = m;
    hrev.resize(n);
    for (unsigned i = 0; i < n; ++i) hrev[i] = h[n - 1 - i];
    w.init(n);
    scale = 1.0f;
  }
  void execute(const cf *x, cf *y) {
    for (unsigned i = 0; i < M; ++i) {
      w.push(x[i]);
      if (i == 0) {
        cf r = dot_cf(hrev.data(), w.data(), static_cast<unsigned>(hrev.size()));
        *y = cf(r.real() * scale, r.imag() * scale);
      }
    }
  }
};

/* iirfilt_rrrf, transfer-function form, direct form II, a[0] normalised */
struct IirFilt {
  std::vector<float> b, a, v;
  void create(const float *bb, unsigned nb, const float *aa, unsigned na) {
    unsigned n = std::max(nb, na);
    b.assign(n, 0.0f);
    a.assign(n, 0.0f);
    float a0 = aa[0];
    for (unsigned i = 0; i < nb; ++i) b[i] = bb[i] / a0;
    for (unsigned i = 0; i < na; ++i) a[i] = aa[i] / a0;
    v.assign(n, 0.0f);
  }
  // iirfilt_rrrf_create_dc_blocker: H(z) = (1 - z^-1) / (1 - (1-alpha) z^-1)
  void create_dc_blocker(float alpha) {
    float bb[2] = {1.0f, -1.0f};
    float aa[2] = {1.0f, -1.0f + alpha};
    create(bb, 2, aa, 2);
  }
  void reset() { std::fill(v.begin(), v.end(), 0.0f); }
  float execute(float x) {
    unsigned n = static_cast<unsigned>(v.size());
    for (unsigned i = n - 1; i > 0; --i) v[i] = v[i - 1];
    float s = dot_rf(a.data() + 1, v.data() + 1, n - 1);
    v[0] = x - s;
    return dot_rf(b.data(), v.data(), n);
  }
};

/* freqdem: y = arg(conj(r_prev) r) / (2 pi kf) */
struct FreqDem {
  float ref = 1.0f;
  cf prev{0.0f, 0.0f};
  void create(float kf) {
    ref = static_cast<float>(1.0 / (2.0 * kPiD * static_cast<double>(kf)));
    prev = cf(0.0f, 0.0f);
  }
  void reset() { prev = cf(0.0f, 0.0f); }
  float demodulate(cf r) {
    float a = prev.real(), b = prev.imag();
    float re = a * r.real() + b * r.imag();
    float im = a * r.imag() - b * r.real();
    prev = r;
    return std::atan2(im, re) * ref;
  }
};

/* agc_crcf */
struct Agc {
  float g = 1.0f, scale = 1.0f, alpha = 0.01f, y2p = 1.0f;
  void create() {
    alpha = 0.01f;
    g = 1.0f;
    y2p = 1.0f;
    scale = 1.0f;
  }
  void set_bandwidth(float bt) { alpha = bt; }
  void set_gain(float gain) { g = gain; }
  cf execute(cf x) {
    cf y(x.real() * g, x.imag() * g);
    float y2 = y.real() * y.real() + y.imag() * y.imag();
    y2p = static_cast<float>((1.0 - static_cast<double>(alpha)) * static_cast<double>(y2p) +
                             static_cast<double>(alpha * y2));
    if (y2p > 1e-6f) g *= std::exp(-0.5f * alpha * std::log(y2p));
    if (g > 1e6f) g = 1e6f;
    return cf(y.real() * scale, y.imag() * scale);
  }
};

/* nco_crcf with 32-bit fixed-point phase and the simple 2nd-order PLL */
static uint32_t nco_constrain(float theta) {
  float p = static_cast<float>(static_cast<double>(theta) * 0.159154943091895);
  float fpart = p - static_cast<float>(static_cast<long>(p));
  if (fpart < 0.0f) fpart = static_cast<float>(static_cast<double>(fpart) + 1.0);
  float s = fpart * 4294967296.0f;
  if (s >= 4294967296.0f) return 0u; // x86 cvttss2si64 + truncation
  return static_cast<uint32_t>(s);
}
struct Nco {
  uint32_t theta = 0, dtheta = 0;
  float alpha = 0.0f, beta = 0.0f;
  void set_frequency(float f) { dtheta = nco_constrain(f); }
  void reset() {
    theta = 0;
    dtheta = 0;
  }
  void pll_set_bandwidth(float bw) {
    alpha = bw;
    beta = std::sqrt(bw);
  }
  void pll_step(float dphi) {
    dtheta += nco_constrain(dphi * alpha);
    theta += nco_constrain(dphi * beta);
  }
  void step() { theta += dtheta; }
  float get_phase() const {
    return static_cast<float>(2.0 * kPiD * static_cast<double>(static_cast<float>(theta)) /
                              4294967296.0);
  }
};

/* firpfb: branch i taps h[i + n*npfb]; window shared by all branches */
struct FirPfb {
  unsigned npfb = 0, sub = 0;
  std::vector<float> hrev; // [npfb][sub], reversed per branch
  Window<float> wr;
  Window<cf> wc;
  void create(unsigned nf, const float *h, unsigned hlen) {
    npfb = nf;
    sub = hlen / nf;
    hrev.assign(static_cast<size_t>(npfb) * sub, 0.0f);
    for (unsigned i = 0; i < npfb; ++i)
      for (unsigned n = 0; n < sub; ++n) hrev[i * sub + (sub - n - 1)] = h[i + n * npfb];
    wr.init(sub);
    wc.init(sub);
  }
  void reset() {
    wr.reset();
    wc.reset();
  }
  float exec_r(unsigned i) const { return dot_rf(&hrev[i * sub], wr.data(), sub); }
  cf exec_c(unsigned i) const { return dot_cf(&hrev[i * sub], wc.data(), sub); }
};

/* resamp_rrrf (float timing phase, linear interpolation between branches) */
struct Resamp {
  unsigned m = 12, npfb = 32;
  float rate = 1.0f, del = 1.0f, tau = 0.0f, bf = 0.0f, mu = 0.0f;
  int b = 0;
  int state = 0; // 0 interp, 1 boundary
  float y0 = 0.0f, y1 = 0.0f;
  FirPfb f;
  std::vector<float> proto;
  void create(float r, unsigned mm, float fc, float As, unsigned nf) {
    m = mm;
    npfb = nf;
    unsigned n = 2 * m * npfb + 1;
    std::vector<float> hf(n);
    firdes_kaiser(n, fc / static_cast<float>(npfb), As, 0.0f, hf.data());
    float gain = 0.0f;
    for (unsigned i = 0; i < n; ++i) gain += hf[i];
    gain = static_cast<float>(npfb) / gain;
    proto.resize(n);
    for (unsigned i = 0; i < n; ++i) proto[i] = hf[i] * gain;
    f.create(npfb, proto.data(), n - 1);
    set_rate(r);
    reset();
  }
  void set_rate(float r) {
    rate = r;
    del = 1.0f / rate;
  }
  void reset() {
    f.reset();
    state = 0;
    tau = 0.0f;
    bf = 0.0f;
    b = 0;
    mu = 0.0f;
    y0 = 0.0f;
    y1 = 0.0f;
  }
  void update_timing() {
    tau += del;
    bf = tau * static_cast<float>(npfb);
    b = static_cast<int>(std::floor(bf));
    mu = bf - static_cast<float>(b);
  }
  unsigned execute(float x, float *y) {
    f.wr.push(x);
    unsigned n = 0;
    while (b < static_cast<int>(npfb)) {
      if (state == 1) {
        y1 = f.exec_r(0);
        y[n++] = (1.0f - mu) * y0 + mu * y1;
        update_timing();
        state = 0;
      } else {
        y0 = f.exec_r(static_cast<unsigned>(b));
        if (b == static_cast<int>(npfb) - 1) {
          state = 1;
          b = static_cast<int>(npfb);
        } else {
          y1 = f.exec_r(static_cast<unsigned>(b + 1));
          y[n++] = (1.0f - mu) * y0 + mu * y1;
          update_timing();
        }
      }
    }
    tau -= 1.0f;
    bf -= static_cast<float>(npfb);
    b -= static_cast<int>(npfb);
    return n;
  }
};

/* iirfiltsos_rrrf (direct form II) for the symsync loop filter */
struct IirSos {
  float b[3] = {0, 0, 0}, a[3] = {1, 0, 0}, v[3] = {0, 0, 0};
  void set(const float *B, const float *A) {
    float a0 = A[0];
    for (int i = 0; i < 3; ++i) {
      b[i] = B[i] / a0;
      a[i] = A[i] / a0;
    }
  }
  void reset() { v[0] = v[1] = v[2] = 0.0f; }
  float execute(float x) {
    float t1 = a[1] * v[1];
    float t2 = a[2] * v[2];
    v[0] = x - t1 - t2;
    float y = b[0] * v[0] + b[1] * v[1] + b[2] * v[2];
    v[2] = v[1];
    v[1] = v[0];
    return y;
  }
};

/* symsync_crcf (polyphase MF + dMF timing recovery) */
struct SymSync {
  unsigned k = 3, k_out = 1, npfb = 32;
  unsigned decim_counter = 0;
  bool is_locked = false;
  float rate = 3.0f, del = 3.0f, tau = 0.0f, bf = 0.0f;
  int b = 0;
  float q = 0.0f, q_hat = 0.0f, rate_adjustment = 0.0f;
  float B[3] = {0, 0, 0}, A[3] = {1, 0, 0};
  IirSos pll;
  FirPfb mf, dmf;
  std::vector<float> h, dh;
  void create_rnyquist(unsigned kk, unsigned m, float beta, unsigned nf) {
    unsigned hlen = 2 * nf * kk * m + 1;
    h.resize(hlen);
    firdes_rrcos(nf * kk, m, beta, 0.0f, h.data());
    create(kk, nf, h.data(), hlen);
  }
  void create(unsigned kk, unsigned nf, const float *hh, unsigned hlen) {
    k = kk;
    npfb = nf;
    set_output_rate(1);
    dh.resize(hlen);
    float hdh_max = 0.0f;
    for (unsigned i = 0; i < hlen; ++i) {
      if (i == 0) dh[i] = hh[i + 1] - hh[hlen - 1];
      else if (i == hlen - 1) dh[i] = hh[0] - hh[i - 1];
      else dh[i] = hh[i + 1] - hh[i - 1];
      if (std::fabs(hh[i] * dh[i]) > hdh_max || i == 0) hdh_max = std::fabs(hh[i] * dh[i]);
    }
    for (unsigned i = 0; i < hlen; ++i) dh[i] *= 0.06f / hdh_max;
    mf.create(npfb, hh, hlen);
    dmf.create(npfb, dh.data(), hlen);
    A[0] = 1.0f; B[0] = 0.0f;
    A[1] = 0.0f; B[1] = 0.0f;
    A[2] = 0.0f; B[2] = 0.0f;
    pll.set(B, A);
    reset();
    set_lf_bw(0.01f);
    is_locked = false;
  }
  void set_output_rate(unsigned ko) {
    k_out = ko;
    rate = static_cast<float>(k) / static_cast<float>(k_out);
    del = rate;
  }
  void set_lf_bw(float bt) {
    float alpha = 1.000f - bt;
    float beta = 0.220f * bt;
    float a = 0.500f;
    float bb = 0.495f;
    B[0] = beta; B[1] = 0.0f; B[2] = 0.0f;
    A[0] = 1.00f - a * alpha;
    A[1] = -bb * alpha;
    A[2] = 0.0f;
    pll.set(B, A);
    rate_adjustment = static_cast<float>(0.5 * static_cast<double>(bt));
  }
  void reset() {
    mf.reset(); // liquid resets the matched filter bank only
    rate = static_cast<float>(k) / static_cast<float>(k_out);
    del = rate;
    b = 0;
    bf = 0.0f;
    tau = 0.0f;
    q = 0.0f;
    q_hat = 0.0f;
    decim_counter = 0;
    pll.reset();
  }
  void advance_loop(cf mfo, cf dmfo) {
    q = mfo.real() * dmfo.real() + mfo.imag() * dmfo.imag(); // Re(conj(mf) dmf)
    if (q > 1.0f) q = 1.0f;
    else if (q < -1.0f) q = -1.0f;
    q_hat = pll.execute(q);
    rate += rate_adjustment * q_hat;
    del = rate + q_hat;
  }
  // one input sample -> 0..n outputs; returns count
  unsigned step(cf x, cf *y) {
    mf.wc.push(x);
    dmf.wc.push(x);
    unsigned n = 0;
    while (b < static_cast<int>(npfb)) {
      cf mfo = mf.exec_c(static_cast<unsigned>(b));
      y[n] = cf(mfo.real() / static_cast<float>(k), mfo.imag() / static_cast<float>(k));
      if (decim_counter == k_out) {
        decim_counter = 0;
        if (!is_locked) {
          cf dmfo = dmf.exec_c(static_cast<unsigned>(b));
          advance_loop(mfo, dmfo);
        }
      }
      decim_counter++;
      tau += del;
      bf = tau * static_cast<float>(npfb);
      b = static_cast<int>(std::round(bf));
      n++;
    }
    tau -= 1.0f;
    bf -= static_cast<float>(npfb);
    b -= static_cast<int>(npfb);
    return n;
  }
};

/* modem PSK2 (generic PSK demodulator) + demodulator phase error */
struct ModemPsk2 {
  cf r{0, 0}, xhat{0, 0};
  unsigned demodulate(cf x) {
    const float alpha = static_cast<float>(kPiD / 2.0);            // pi / M
    const float d_phi = static_cast<float>(kPiD * (1.0 - 1.0 / 2)); // pi (1 - 1/M)
    float theta = std::atan2(x.imag(), x.real());
    theta -= d_phi;
    if (static_cast<double>(theta) < -kPiD)
      theta = static_cast<float>(static_cast<double>(theta) + 2.0 * kPiD);
    unsigned s = (theta > 0.0f) ? 1u : 0u; // linear array demod, m = 1
    float arg = static_cast<float>(s) * 2.0f * alpha;
    xhat = cf(std::cos(arg), std::sin(arg));
    r = x;
    return s;
  }
  float phase_error() const {
    // Im(r * conj(xhat))
    return r.imag() * xhat.real() - r.real() * xhat.imag();
  }
};

} // namespace lq

/* ========================================================================= */
namespace ref {

constexpr float kPi = 3.14159265358979323846f;

/* ComplexDecimator -- src/dsp/liquid_primitives.cpp:370-499 */
struct ComplexDecimator {
  lq::FirDecimCrcf obj;
  uint32_t factor = 1, tapsPerPhase = 12;
  float As = 70.0f;
  std::vector<float> taps;
  std::vector<cf> block;
  void init(uint32_t f, uint32_t tpp, float as) {
    if (f == 0) throw std::runtime_error("complex decimator factor must be >= 1");
    factor = f;
    tapsPerPhase = std::max<uint32_t>(4, tpp);
    As = as;
    block.assign(factor, cf(0, 0));
    taps.clear();
    if (factor == 1) return;
    uint32_t hLen = factor * tapsPerPhase;
    taps.assign(hLen, 0.0f);
    float cutoff = std::clamp(0.45f / static_cast<float>(factor), 0.01f, 0.45f);
    lq::firdes_kaiser(hLen, cutoff, As, 0.0f, taps.data());
    obj.create(factor, taps.data(), hLen);
    obj.scale = 2.0f * cutoff;
  }
  void reset() {
    if (factor == 1) return;
    uint32_t hLen = factor * tapsPerPhase;
    float cutoff = std::clamp(0.45f / static_cast<float>(factor), 0.01f, 0.45f);
    obj.create(factor, taps.data(), hLen);
    obj.scale = 2.0f * cutoff;
  }
  size_t executeComplex(const uint8_t *in, size_t inSamples, cf *out, size_t cap) {
    if (!in || !out || inSamples == 0 || cap == 0) return 0;
    constexpr float kScale = 1.0f / 127.5f;
    if (factor == 1) {
      size_t n = std::min(inSamples, cap);
      for (size_t i = 0; i < n; ++i)
        out[i] = cf((static_cast<float>(in[2 * i]) - 127.5f) * kScale,
                    (static_cast<float>(in[2 * i + 1]) - 127.5f) * kScale);
      return n;
    }
    size_t blocks = std::min(inSamples / factor, cap);
    for (size_t b = 0; b < blocks; ++b) {
      for (size_t k = 0; k < factor; ++k) {
        size_t idx = (b * factor + k) * 2;
        block[k] = cf((static_cast<float>(in[idx]) - 127.5f) * kScale,
                      (static_cast<float>(in[idx + 1]) - 127.5f) * kScale);
      }
      cf y;
      obj.execute(block.data(), &y);
      out[b] = y;
    }
    return blocks;
  }
  // execute: u8 -> u8 requantised (liquid_primitives.cpp:422-459)
  size_t execute(const uint8_t *in, size_t inSamples, uint8_t *out, size_t cap) {
    if (!in || !out || inSamples == 0 || cap == 0) return 0;
    if (factor == 1) {
      size_t n = std::min(inSamples, cap);
      std::copy_n(in, n * 2, out);
      return n;
    }
    std::vector<cf> y(std::min(inSamples / factor, cap));
    const size_t blocks = executeComplex(in, inSamples, y.data(), y.size());
    for (size_t b = 0; b < blocks; ++b) {
      const float iOut = std::clamp((y[b].real() * 127.5f) + 127.5f, 0.0f, 255.0f);
      const float qOut = std::clamp((y[b].imag() * 127.5f) + 127.5f, 0.0f, 255.0f);
      out[2 * b] = static_cast<uint8_t>(iOut);
      out[2 * b + 1] = static_cast<uint8_t>(qOut);
    }
    return blocks;
  }
};

/* liquid_primitives FIRFilter::init(length, cutoff, As, center) :62-113 */
static void design_fir(std::vector<float> &taps, float &scale, uint32_t length, float cutoff,
                       float As, float center) {
  taps.assign(length, 0.0f);
  lq::firdes_kaiser(length, cutoff, As, 0.0f, taps.data());
  if (std::fabs(center) < 1e-6f) {
    scale = 2.0f * cutoff;
    return;
  }
  const int mid = static_cast<int>(length / 2);
  constexpr float kTwoPi = 6.28318530717958647692f;
  for (uint32_t n = 0; n < length; ++n) {
    const float phase = kTwoPi * center * static_cast<float>(static_cast<int>(n) - mid);
    taps[n] = 2.0f * taps[n] * std::cos(phase);
  }
  double sumAbs = 0.0;
  for (float t : taps) sumAbs += std::fabs(t);
  if (sumAbs > 1e-12) {
    const float inv = static_cast<float>(1.0 / sumAbs);
    for (float &t : taps) t *= inv;
  }
  scale = 1.0f;
}

struct FIR {
  lq::FirFiltCrcf f;
  std::vector<float> taps;
  float scale = 1.0f;
  void init(uint32_t length, float cutoff, float As = 60.0f, float center = 0.0f) {
    design_fir(taps, scale, length, cutoff, As, center);
    f.create(taps.data(), length);
    f.scale = scale;
  }
  void reset() {
    f.create(taps.data(), static_cast<unsigned>(taps.size()));
    f.scale = scale;
  }
  void push(cf x) { f.push(x); }
  cf execute() const { return f.execute(); }
};

struct IIR {
  lq::IirFilt f;
  bool ready = false, dc = false;
  float dcAlpha = 0.0f;
  std::vector<float> b, a;
  void init(const std::vector<float> &bb, const std::vector<float> &aa) {
    b = bb;
    a = aa;
    dc = false;
    f.create(b.data(), static_cast<unsigned>(b.size()), a.data(), static_cast<unsigned>(a.size()));
    ready = true;
  }
  void initDC(float alpha) {
    dc = true;
    dcAlpha = alpha;
    f.create_dc_blocker(alpha);
    ready = true;
  }
  void reset() {
    if (!ready) return;
    f.reset();
  }
  float execute(float x) { return ready ? f.execute(x) : x; }
};

struct ResamplerW { // liquid_primitives Resampler :325-362
  lq::Resamp r;
  float ratio = 1.0f;
  void init(float rr, uint32_t m = 12, float fc = 0.47f, float As = 60.0f, uint32_t nf = 32) {
    if (rr < 0.005f || rr > 8.0f) throw std::runtime_error("resampler ratio out of range");
    ratio = rr;
    r.create(rr, m, fc, As, nf);
  }
  void reset() { r.reset(); }
  uint32_t execute(float x, float *out) { return r.execute(x, out); }
};

/* FMDemod -- src/fm_demod.cpp */
static const int kXdrFmBwHz[30] = {309000, 298000, 281000, 263000, 246000, 229000, 211000, 194000,
                                   177000, 159000, 142000, 125000, 108000, 95000,  90000,  83000,
                                   73000,  63000,  55000,  48000,  42000,  36000,  32000,  27000,
                                   24000,  20000,  17000,  15000,  9000,   0};

struct FMDemod {
  enum AgcMode { Off = 0, Fast = 1, Slow = 2 };
  int inputRate, outputRate;
  double deviation = 75000.0;
  bool deemphEnabled = true;
  int bandwidthMode = 0;
  int w0 = 194000;
  int agcMode = Off;
  bool clipping = false;
  float clipRatio = 0.0f;
  FIR iqFilter;
  lq::FreqDem fd;
  IIR dcI, dcQ, monoDeemph, monoDc;
  ResamplerW monoResamp;
  lq::Agc agc;
  bool agcReady = false;
  float agcBw = 0.0f, agcG0 = 1.0f;
  std::vector<float> scratch;

  FMDemod(int in, int out) : inputRate(std::max(1, in)), outputRate(std::max(1, out)) {
    const float iqCutoffNorm = std::clamp(110000.0f / static_cast<float>(inputRate), 0.01f, 0.45f);
    iqFilter.init(81, iqCutoffNorm);
    dcI.initDC(0.0005f);
    dcQ.initDC(0.0005f);
    monoResamp.init(static_cast<float>(outputRate) / static_cast<float>(inputRate));
    monoDc.initDC(0.0008f);
    setDeviation(75000.0);
    setDeemphasis(75);
    setDspAgcMode(Off);
  }
  void setDeemphasis(int tau_us) {
    if (tau_us <= 0) {
      deemphEnabled = false;
      return;
    }
    deemphEnabled = true;
    const float tau = static_cast<float>(tau_us) * 1e-6f;
    const float dt = 1.0f / static_cast<float>(outputRate);
    const float alpha = dt / (tau + dt);
    monoDeemph.init({alpha}, {1.0f, -(1.0f - alpha)});
  }
  void setDeviation(double d) {
    deviation = d;
    fd.create(static_cast<float>(deviation / static_cast<double>(inputRate)));
  }
  void reset() {
    clipping = false;
    clipRatio = 0.0f;
    iqFilter.reset();
    fd.reset();
    dcI.reset();
    dcQ.reset();
    if (deemphEnabled) monoDeemph.reset();
    monoDc.reset();
    monoResamp.reset();
    if (agcReady) initAgc();
  }
  void setBandwidthMode(int mode) {
    static constexpr int kTef[] = {311000, 287000, 254000, 236000, 217000, 200000,
                                   184000, 168000, 151000, 133000, 114000, 97000,
                                   84000,  72000,  64000,  56000,  0};
    int c = std::clamp(mode, 0, 16);
    setBandwidthHz(kTef[c]);
  }
  void setBandwidthHz(int bwHz) {
    const int eff = (bwHz <= 0) ? w0 : bwHz;
    int selected = 29;
    if (eff > 0) {
      int minDiff = std::numeric_limits<int>::max();
      for (int i = 0; i < 29; ++i) {
        int diff = std::abs(kXdrFmBwHz[i] - eff);
        if (diff < minDiff) {
          minDiff = diff;
          selected = i;
        }
      }
    }
    if (selected == bandwidthMode) return;
    bandwidthMode = selected;
    const int sel = kXdrFmBwHz[selected];
    const double head = 0.45 * static_cast<double>(inputRate);
    const double cut = (sel > 0) ? std::clamp(static_cast<double>(sel) * 0.5, 9000.0, head) : head;
    const float cn = std::clamp(static_cast<float>(cut / static_cast<double>(inputRate)), 0.01f, 0.45f);
    const uint32_t len = (sel > 0 && sel <= 73000) ? 121U : 81U;
    const float As = (sel > 0 && sel <= 42000) ? 70.0f : 60.0f;
    iqFilter.init(len, cn, As);
  }
  void setW0(int bw) { w0 = std::clamp(bw, 0, 400000); }
  void initAgc() {
    agc.create();
    agc.set_bandwidth(agcBw);
    agc.set_gain(agcG0);
    agcReady = true;
  }
  void setDspAgcMode(int mode) {
    agcMode = mode;
    if (agcMode == Off) return;
    agcBw = (agcMode == Fast) ? 0.01f : 0.001f;
    agcG0 = 1.0f;
    initAgc();
  }
  float step(float iRaw, float qRaw) {
    const float iDc = dcI.execute(iRaw);
    const float qDc = dcQ.execute(qRaw);
    iqFilter.push(cf(iDc, qDc));
    cf x = iqFilter.execute();
    if (agcMode != Off && agcReady) x = agc.execute(x);
    return fd.demodulate(x);
  }
  void demodulate(const uint8_t *iq, float *audio, size_t len) {
    size_t clip = 0;
    for (size_t i = 0; i < len; ++i) {
      uint8_t ib = iq[2 * i], qb = iq[2 * i + 1];
      if (ib == 0 || ib == 255 || qb == 0 || qb == 255) clip++;
      const float iR = (static_cast<float>(ib) - 127.0f) / 127.5f;
      const float qR = (static_cast<float>(qb) - 127.0f) / 127.5f;
      audio[i] = step(iR, qR);
    }
    clipping = clip > 0;
    clipRatio = len ? static_cast<float>(clip) / static_cast<float>(len) : 0.0f;
  }
  void demodulateComplex(const cf *iq, float *audio, size_t len) {
    size_t clip = 0;
    for (size_t i = 0; i < len; ++i) {
      const float iR = iq[i].real(), qR = iq[i].imag();
      if (std::fabs(iR) >= 0.995f || std::fabs(qR) >= 0.995f) clip++;
      audio[i] = step(iR, qR);
    }
    clipping = clip > 0;
    clipRatio = len ? static_cast<float>(clip) / static_cast<float>(len) : 0.0f;
  }
  size_t downsampleAudio(const float *d, float *audio, size_t n) {
    size_t out = 0;
    float tmp[8];
    for (size_t i = 0; i < n; ++i) {
      uint32_t p = monoResamp.execute(d[i], tmp);
      for (uint32_t k = 0; k < p; ++k) {
        float s = tmp[k];
        if (deemphEnabled) s = monoDeemph.execute(s);
        s = monoDc.execute(s);
        audio[out++] = s;
      }
    }
    return out;
  }
  size_t processSplitComplex(const cf *iq, float *mpx, float *mono, size_t n) {
    if (scratch.size() < n) scratch.resize(n);
    demodulateComplex(iq, scratch.data(), n);
    if (mpx) std::memcpy(mpx, scratch.data(), n * sizeof(float));
    if (!mono) return 0;
    return downsampleAudio(scratch.data(), mono, n);
  }
  size_t processSplit(const uint8_t *iq, float *mpx, float *mono, size_t n) {
    if (scratch.size() < n) scratch.resize(n);
    demodulate(iq, scratch.data(), n);
    if (mpx) std::memcpy(mpx, scratch.data(), n * sizeof(float));
    if (!mono) return 0;
    return downsampleAudio(scratch.data(), mono, n);
  }
};

/* StereoDecoder -- src/stereo_decoder.cpp */
struct StereoDecoder {
  enum Blend { Soft = 0, Normal = 1, Aggressive = 2 };
  static constexpr int kPilotAcquireBlocks = 6, kPilotLossBlocks = 24;
  static constexpr float kMatrixScale = 0.5f, kPilotRatioAcquire = 0.040f,
                         kPilotRatioHold = 0.022f, kMpxMinAcquire = 0.005f,
                         kMpxMinHold = 0.0028f, kPilotCoherenceAcquire = 0.18f,
                         kPilotCoherenceHold = 0.11f, kPllLockAcquireHz = 180.0f,
                         kPllLockHoldHz = 320.0f, kEnvSmooth = 0.9995f,
                         kEnvInject = 1.0f - 0.9995f, kIqSmooth = 0.9995f,
                         kIqInject = 1.0f - 0.9995f;
  int inputRate;
  bool stereoDetected = false, forceStereo = false, forceMono = false;
  int blendMode = Normal;
  float pilotMagnitude = 0, pilotBandMagnitude = 0, mpxMagnitude = 0, stereoBlend = 0;
  int pilotLevelTenthsKHz = 0;
  float pilotI = 0, pilotQ = 0, pllPhase = 0, pllFreq, pllMinFreq, pllMaxFreq;
  int pilotCount = 0, pilotLossCount = 0;
  std::vector<float> delayLine;
  size_t delayPos = 0;
  int delaySamples = 0;
  FIR pilotBpf, leftLpf, rightLpf;
  lq::Nco pll;
  float nominalFreq;

  StereoDecoder(int in, int /*out*/)
      : inputRate(in), pllFreq(2.0f * kPi * 19000.0f / static_cast<float>(in)),
        pllMinFreq(2.0f * kPi * 18750.0f / static_cast<float>(in)),
        pllMaxFreq(2.0f * kPi * 19250.0f / static_cast<float>(in)) {
    int taps = static_cast<int>(std::ceil(3.8 * static_cast<double>(inputRate) / 3000.0));
    taps = std::clamp(taps, 63, 511);
    if ((taps % 2) == 0) taps++;
    const float centerNorm = std::clamp(19000.0f / static_cast<float>(inputRate), 0.001f, 0.49f);
    const float cutNorm = std::clamp(250.0f / static_cast<float>(inputRate), 0.0005f, 0.45f);
    pilotBpf.init(static_cast<uint32_t>(taps), cutNorm, 60.0f, centerNorm);
    const float audioCut = std::clamp(15000.0f / static_cast<float>(inputRate), 0.01f, 0.45f);
    leftLpf.init(121, audioCut);
    rightLpf.init(121, audioCut);
    delaySamples = std::max(0, (taps - 1) / 2);
    delayLine.assign(static_cast<size_t>(std::max(1, delaySamples + 1)), 0.0f);
    nominalFreq = 2.0f * kPi * 19000.0f / static_cast<float>(inputRate);
    pll.reset();
    pll.set_frequency(nominalFreq);
    pll.pll_set_bandwidth(0.01f);
  }
  void reset() {
    stereoDetected = false;
    pilotMagnitude = pilotBandMagnitude = mpxMagnitude = stereoBlend = 0.0f;
    pilotLevelTenthsKHz = 0;
    pilotI = pilotQ = 0.0f;
    pllPhase = 0.0f;
    pllFreq = 2.0f * kPi * 19000.0f / static_cast<float>(inputRate);
    pilotCount = pilotLossCount = 0;
    delayPos = 0;
    std::fill(delayLine.begin(), delayLine.end(), 0.0f);
    pilotBpf.reset();
    pll.reset();
    pll.set_frequency(nominalFreq);
    leftLpf.reset();
    rightLpf.reset();
  }
  size_t processAudio(const float *mono, float *left, float *right, size_t n,
                      float *phaseTrace = nullptr, float *blendTrace = nullptr) {
    if (!mono || !left || !right || n == 0) return 0;
    float attackTau = 0.120f, releaseTau = 0.030f, lowQualityGate = 0.85f, lockFloor = 0.0f;
    if (blendMode == Soft) {
      attackTau = 0.090f;
      releaseTau = 0.040f;
      lowQualityGate = 0.75f;
    } else if (blendMode == Aggressive) {
      attackTau = 0.180f;
      releaseTau = 0.015f;
      lowQualityGate = 0.95f;
    }
    const float blendAttack = 1.0f - std::exp(-1.0f / (attackTau * static_cast<float>(inputRate)));
    const float blendRelease = 1.0f - std::exp(-1.0f / (releaseTau * static_cast<float>(inputRate)));
    const float nominal = 2.0f * kPi * 19000.0f / static_cast<float>(inputRate);
    auto target = [&](float ratio, float coh, float errHz) -> float {
      if (forceMono) return 0.0f;
      if (forceStereo) return 1.0f;
      const float ratioQ = std::clamp((ratio - kPilotRatioHold) /
                                          std::max(kPilotRatioAcquire - kPilotRatioHold, 1e-4f),
                                      0.0f, 1.0f);
      const float cohQ = std::clamp((coh - kPilotCoherenceHold) /
                                        std::max(kPilotCoherenceAcquire - kPilotCoherenceHold, 1e-4f),
                                    0.0f, 1.0f);
      const float pllQ = std::clamp((kPllLockHoldHz - errHz) /
                                        std::max(kPllLockHoldHz - kPllLockAcquireHz, 1e-3f),
                                    0.0f, 1.0f);
      const float quality = std::min(ratioQ, std::min(cohQ, pllQ));
      float shaped = quality * quality;
      if (blendMode == Soft) shaped = std::sqrt(std::max(0.0f, quality));
      else if (blendMode == Aggressive) shaped = quality * quality * quality;
      if (ratio < (kPilotRatioHold * lowQualityGate) || coh < (kPilotCoherenceHold * lowQualityGate) ||
          errHz > (kPllLockHoldHz * 1.10f))
        return 0.0f;
      if (stereoDetected) return std::clamp(lockFloor + ((1.0f - lockFloor) * shaped), 0.0f, 1.0f);
      return 0.0f;
    };
    size_t out = 0;
    for (size_t i = 0; i < n; ++i) {
      const float mpx = mono[i];
      pilotBpf.push(cf(mpx, 0.0f));
      const float pilot = pilotBpf.execute().real();
      pilotBandMagnitude = (pilotBandMagnitude * kEnvSmooth) + (std::fabs(pilot) * kEnvInject);
      mpxMagnitude = (mpxMagnitude * kEnvSmooth) + (std::fabs(mpx) * kEnvInject);
      const float phaseNow = pll.get_phase();
      const float vcoI = std::cos(phaseNow);
      const float vcoQ = std::sin(phaseNow);
      const float error = pilot * vcoQ;
      pll.pll_step(error);
      pll.step();
      const float phaseNext = pll.get_phase();
      float dphi = phaseNext - phaseNow;
      if (dphi > kPi) dphi -= 2.0f * kPi;
      else if (dphi < -kPi) dphi += 2.0f * kPi;
      pllPhase = phaseNext;
      pllFreq = std::clamp(dphi, pllMinFreq, pllMaxFreq);
      pilotI = (pilotI * kIqSmooth) + ((pilot * vcoI) * kIqInject);
      pilotQ = (pilotQ * kIqSmooth) + ((pilot * vcoQ) * kIqInject);
      const float magNow = std::sqrt((pilotI * pilotI) + (pilotQ * pilotQ));
      const float ratioNow = pilotBandMagnitude / std::max(mpxMagnitude, 1e-3f);
      const float cohNow = magNow / std::max(pilotBandMagnitude, 1e-4f);
      const float errNow = std::fabs(pllFreq - nominal) * static_cast<float>(inputRate) / (2.0f * kPi);
      const float tgt = target(ratioNow, cohNow, errNow);
      const float delayed = delayLine[delayPos];
      delayLine[delayPos] = mpx;
      delayPos++;
      if (delayPos >= delayLine.size()) delayPos = 0;
      const float monoNorm = delayed * kMatrixScale;
      const float pllRe = std::cos(pllPhase);
      const float pllIm = std::sin(pllPhase);
      const float cos2 = (pllRe * pllRe) - (pllIm * pllIm);
      const float lr = 2.0f * delayed * cos2;
      const float sl = (delayed + lr) * kMatrixScale;
      const float sr = (delayed - lr) * kMatrixScale;
      const float a = (tgt > stereoBlend) ? blendAttack : blendRelease;
      stereoBlend += (tgt - stereoBlend) * a;
      const float lRaw = monoNorm + ((sl - monoNorm) * stereoBlend);
      const float rRaw = monoNorm + ((sr - monoNorm) * stereoBlend);
      leftLpf.push(cf(lRaw, 0.0f));
      rightLpf.push(cf(rRaw, 0.0f));
      left[out] = leftLpf.execute().real();
      right[out] = rightLpf.execute().real();
      if (phaseTrace) phaseTrace[out] = pllPhase;
      if (blendTrace) blendTrace[out] = stereoBlend;
      out++;
    }
    const float mag = std::sqrt((pilotI * pilotI) + (pilotQ * pilotQ));
    pilotMagnitude = (pilotMagnitude * 0.9f) + (mag * 0.1f);
    const float mpxThr = stereoDetected ? kMpxMinHold : kMpxMinAcquire;
    const float ratio = pilotBandMagnitude / std::max(mpxMagnitude, 1e-3f);
    const float coh = pilotMagnitude / std::max(pilotBandMagnitude, 1e-4f);
    const float ratioThr = stereoDetected ? kPilotRatioHold : kPilotRatioAcquire;
    const float cohThr = stereoDetected ? kPilotCoherenceHold : kPilotCoherenceAcquire;
    const float errHz = std::fabs(pllFreq - nominal) * static_cast<float>(inputRate) / (2.0f * kPi);
    const float pllThr = stereoDetected ? kPllLockHoldHz : kPllLockAcquireHz;
    const bool present = (mpxMagnitude > mpxThr) && (ratio > ratioThr) && (coh > cohThr) && (errHz < pllThr);
    if (!forceStereo) {
      if (!stereoDetected) {
        if (present) {
          pilotCount++;
          pilotLossCount = 0;
          if (pilotCount >= kPilotAcquireBlocks) stereoDetected = true;
        } else {
          pilotCount = 0;
        }
      } else if (present) {
        pilotLossCount = 0;
      } else if (++pilotLossCount >= kPilotLossBlocks) {
        stereoDetected = false;
        pilotCount = 0;
        pilotLossCount = 0;
      }
    }
    const float calibrated = pilotMagnitude * 8.0f;
    pilotLevelTenthsKHz = std::clamp(static_cast<int>(std::round(calibrated * 750.0f)), 0, 750);
    return out;
  }
};

/* AFPostProcessor -- src/af_post_processor.cpp */
struct AFPostProcessor {
  int inputRate, outputRate;
  bool deemphEnabled = false;
  IIR lDe, rDe, lDc, rDc;
  ResamplerW lRs, rRs;
  AFPostProcessor(int in, int out) : inputRate(std::max(1, in)), outputRate(std::max(1, out)) {
    const float ratio = static_cast<float>(outputRate) / static_cast<float>(inputRate);
    lRs.init(ratio);
    rRs.init(ratio);
    lDc.initDC(0.005f);
    rDc.initDC(0.005f);
    reset();
    setDeemphasis(75);
  }
  void reset() {
    lRs.reset();
    rRs.reset();
    lDc.reset();
    rDc.reset();
    if (deemphEnabled) {
      lDe.reset();
      rDe.reset();
    }
  }
  void setDeemphasis(int tau_us) {
    if (tau_us <= 0) {
      deemphEnabled = false;
      return;
    }
    deemphEnabled = true;
    const float tau = static_cast<float>(tau_us) * 1e-6f;
    const float T = 1.0f / static_cast<float>(outputRate);
    const float alpha = T / (tau + T);
    lDe.init({alpha}, {1.0f, -(1.0f - alpha)});
    rDe.init({alpha}, {1.0f, -(1.0f - alpha)});
  }
  size_t process(const float *inL, const float *inR, size_t n, float *oL, float *oR, size_t cap) {
    if (!inL || !inR || !oL || !oR || n == 0 || cap == 0) return 0;
    size_t out = 0;
    float tl[8], tr[8];
    for (size_t i = 0; i < n && out < cap; ++i) {
      uint32_t pl = lRs.execute(inL[i], tl);
      uint32_t pr = rRs.execute(inR[i], tr);
      uint32_t p = std::min(pl, pr);
      for (uint32_t k = 0; k < p && out < cap; ++k) {
        float l = tl[k], r = tr[k];
        if (deemphEnabled) {
          l = lDe.execute(l);
          r = rDe.execute(r);
        }
        l = lDc.execute(l);
        r = rDc.execute(r);
        oL[out] = l;
        oR[out] = r;
        out++;
      }
    }
    return out;
  }
};

/* ---------------- RDS: redsea_port ---------------- */
constexpr float kTargetRate = 171000.0f;
constexpr float kBitsPerSecond = 1187.5f;

struct BiphaseDecoder { // subcarrier.cpp:50-86
  cf prev{0, 0};
  std::array<float, 128> hist{};
  uint32_t clock = 0, polarity = 0;
  bool push(cf sym, bool &value) {
    const cf bi((sym.real() - prev.real()) * 0.5f, (sym.imag() - prev.imag()) * 0.5f);
    value = bi.real() >= 0.0f;
    bool has = (clock % 2 == polarity);
    prev = sym;
    hist[clock] = std::fabs(bi.real());
    clock++;
    if (clock == hist.size()) {
      float even = 0.0f, odd = 0.0f;
      for (size_t i = 0; i < hist.size(); i += 2) {
        even += hist[i];
        odd += hist[i + 1];
      }
      if (even > odd) polarity = 0;
      else if (odd > even) polarity = 1;
      hist.fill(0.0f);
      clock = 0;
    }
    return has;
  }
};

struct DeltaDecoder {
  bool prev = false;
  bool decode(bool in) {
    bool o = in != prev;
    prev = in;
    return o;
  }
};

static float unwrapf(float p) {
  constexpr float k2Pi = 2.f * kPi;
  if (p > kPi) return p - k2Pi;
  if (p < -kPi) return p + k2Pi;
  return p;
}

struct SubcarrierSet { // subcarrier.cpp:94-235, stream 0 only (rds_decoder.cpp:89)
  float resampleRatio;
  lq::Resamp resampler;
  lq::Agc agc;
  FIR lpf;
  lq::SymSync symsync;
  DeltaDecoder delta;
  BiphaseDecoder biphase;
  lq::Nco nco;
  float ncoInitialFreq = 0.0f, prevF0 = 0.0f, phase0 = 0.0f;
  lq::ModemPsk2 modem;
  uint32_t sampleNum = 0, sampleNumSinceReset = 0;
  std::vector<float> rs;

  explicit SubcarrierSet(float fs) : resampleRatio(kTargetRate / fs) {
    resampler.create(1.0f, 13, 0.47f, 60.0f, 32);
    agc.create();
    agc.set_bandwidth(500.0f / kTargetRate);
    agc.set_gain(0.08f);
    lpf.init(255, 2400.0f / kTargetRate);
    symsync.create_rnyquist(3, 3, 0.8f, 32);
    symsync.set_lf_bw(2200.0f / kTargetRate);
    symsync.set_output_rate(1);
    ncoInitialFreq = 57000.f * (2.f * kPi) / kTargetRate;
    nco.reset();
    nco.set_frequency(ncoInitialFreq);
    nco.pll_set_bandwidth(0.03f / kTargetRate);
    if (resampleRatio < 0.005f || resampleRatio > 2.0f)
      throw std::runtime_error("error: Can't support this sample rate");
    resampler.set_rate(resampleRatio);
  }
  void reset() {
    symsync.reset();
    nco.reset();
    nco.set_frequency(ncoInitialFreq);
    sampleNumSinceReset = 0;
  }
  void ncoStep() { // liquid_wrappers.cpp:125-139 (stream 0 phase only)
    nco.step();
    const float now = nco.get_phase();
    const float delta = unwrapf(now - prevF0);
    prevF0 = now;
    const float scaled = delta * 57000.f / 57000.f;
    phase0 = unwrapf(phase0 + scaled);
  }
  template <typename BitFn> void processSample(float x, BitFn &&onBit) {
    const cf ph(std::cos(-phase0), std::sin(-phase0)); // std::polar(1, -phase)
    const cf bb(x * ph.real(), x * ph.imag());
    lpf.push(bb);
    if (sampleNumSinceReset % 24 == 0) {
      cf lo = agc.execute(lpf.execute());
      cf syms[8];
      unsigned ns = symsync.step(lo, syms);
      if (ns == 1) { // liquid_wrappers.cpp:347-353: Maybe{out[0], n_out == 1}
        cf sym = syms[0];
        modem.demodulate(sym);
        const float pe = std::clamp(modem.phase_error(), -kPi, kPi);
        nco.pll_step(pe * 12.0f);
        bool v;
        if (biphase.push(sym, v)) onBit(delta.decode(v));
      }
    }
    ncoStep();
    sampleNum++;
    sampleNumSinceReset++;
  }
  template <typename BitFn> void chunkToBits(const float *in, size_t n, BitFn &&onBit) {
    float tmp[4];
    for (size_t i = 0; i < n; ++i) {
      unsigned k = resampler.execute(in[i], tmp);
      for (unsigned j = 0; j < k; ++j) processSample(tmp[j], onBit);
    }
  }
};

/* ---- BlockStream -- src/redsea_port/block_sync.cpp ---- */
enum Offset { OA = 0, OB = 1, OC = 2, OCp = 3, OD = 4, OInvalid = 5 };
static int blockNumberFor(int off) {
  switch (off) {
    case OA: return 0;
    case OB: return 1;
    case OC:
    case OCp: return 2;
    case OD: return 3;
    default: return 0;
  }
}
static int nextOffsetFor(int off) {
  switch (off) {
    case OA: return OB;
    case OB: return OC;
    case OC: return OD;
    case OCp: return OD;
    case OD: return OA;
    default: return OA;
  }
}
static int offsetForSyndrome(uint32_t s) {
  switch (s) {
    case 0b1111011000: return OA;
    case 0b1111010100: return OB;
    case 0b1001011100: return OC;
    case 0b1111001100: return OCp;
    case 0b1001011000: return OD;
    default: return OInvalid;
  }
}
static uint32_t syndrome(uint32_t v) {
  static const uint32_t H[26] = {0b1000000000, 0b0100000000, 0b0010000000, 0b0001000000, 0b0000100000,
                                 0b0000010000, 0b0000001000, 0b0000000100, 0b0000000010, 0b0000000001,
                                 0b1011011100, 0b0101101110, 0b0010110111, 0b1010000111, 0b1110011111,
                                 0b1100010011, 0b1101010101, 0b1101110110, 0b0110111011, 0b1000000001,
                                 0b1111011100, 0b0111101110, 0b0011110111, 0b1010100111, 0b1110001111,
                                 0b1100011011};
  uint32_t r = 0;
  for (int k = 0; k < 26; ++k)
    if ((v >> k) & 1u) r ^= H[25 - k];
  return r;
}
struct ErrTable {
  // [offset][52] pairs (syndrome, error vector), table order of block_sync.cpp:216-245
  uint32_t syn[5][52], err[5][52];
  ErrTable() {
    const uint32_t words[5] = {0b0011111100, 0b0110011000, 0b0101101000, 0b1101010000, 0b0110110100};
    for (int o = 0; o < 5; ++o) {
      int idx = 0;
      for (uint32_t bits : {1u, 3u})
        for (uint32_t sh = 0; sh < 26; ++sh) {
          uint32_t e = (bits << sh) & ((1u << 26) - 1u);
          syn[o][idx] = syndrome(e ^ words[o]);
          err[o][idx] = e;
          idx++;
        }
    }
  }
};
static const ErrTable &errTable() {
  static const ErrTable t;
  return t;
}

struct Block {
  uint32_t raw = 0;
  uint16_t data = 0;
  bool received = false, hadErrors = false;
  int offset = OInvalid;
};
struct Group {
  Block blocks[4];
};
struct SyncPulse {
  int offset = OInvalid;
  uint32_t pos = 0;
  bool couldFollow(const SyncPulse &o) const {
    const uint32_t d = pos - o.pos;
    return d % 26 == 0 && d / 26 <= 6 && offset != OInvalid && o.offset != OInvalid &&
           (blockNumberFor(o.offset) + d / 26) % 4 == static_cast<uint32_t>(blockNumberFor(offset));
  }
};

struct BlockStream {
  uint32_t bitcount = 0, untilNext = 1, reg = 0;
  int expected = OA;
  bool inSync = false;
  int errHist[50] = {0};
  size_t errPtr = 0;
  Group current, ready;
  bool hasReady = false;
  uint32_t bitsSinceLost = 0;
  SyncPulse pulses[4];
  bool useFec = true;

  int errSum() const {
    int s = 0;
    for (int v : errHist) s += v;
    return s;
  }
  void pushPulse(int off, uint32_t pos) {
    for (int i = 0; i < 3; ++i) pulses[i] = pulses[i + 1];
    pulses[3].offset = off;
    pulses[3].pos = pos;
  }
  bool sequenceFound() const {
    const SyncPulse &third = pulses[3];
    for (int i = 0; i < 2; ++i)
      for (int j = i + 1; j < 3; ++j)
        if (third.couldFollow(pulses[j]) && pulses[j].couldFollow(pulses[i])) return true;
    return false;
  }
  void acquire(const Block &b) {
    if (inSync) return;
    bitsSinceLost++;
    if (b.offset != OInvalid) {
      pushPulse(b.offset, bitcount);
      if (sequenceFound()) {
        inSync = true;
        expected = b.offset;
        current = Group();
        bitsSinceLost = 0;
      }
    }
  }
  void pushBit(bool bit) {
    reg = (reg << 1u) + (bit ? 1u : 0u);
    untilNext--;
    bitcount++;
    if (untilNext == 0) {
      findBlock();
      untilNext = inSync ? 26 : 1;
    }
  }
  void findBlock() {
    Block b;
    b.raw = reg & ((1u << 26) - 1u);
    b.offset = offsetForSyndrome(syndrome(b.raw));
    acquire(b);
    if (!inSync) return;
    if (expected == OC && b.offset == OCp) expected = OCp;
    b.hadErrors = (b.offset != expected);
    errHist[errPtr] = b.hadErrors ? 1 : 0;
    errPtr = (errPtr + 1) % 50;
    if (errSum() > 42) {
      inSync = false;
      std::fill(std::begin(errHist), std::end(errHist), 0);
      return;
    }
    b.data = static_cast<uint16_t>(b.raw >> 10);
    if (b.hadErrors && useFec) {
      const ErrTable &t = errTable();
      const uint32_t s = syndrome(b.raw);
      for (int i = 0; i < 52; ++i)
        if (t.syn[expected][i] == s) {
          b.data = static_cast<uint16_t>((b.raw ^ t.err[expected][i]) >> 10);
          b.offset = expected;
          break;
        }
    }
    if (b.offset == expected) {
      b.received = true;
      current.blocks[blockNumberFor(expected)] = b;
    }
    const int next = nextOffsetFor(expected);
    if (next == OA) {
      ready = current;
      hasReady = true;
      current = Group();
    }
    expected = next;
  }
};

static oracle_group packGroup(const Group &g, uint32_t blockIndex) {
  auto e = [&](int i) -> uint8_t {
    if (!g.blocks[i].received) return 3;
    return g.blocks[i].hadErrors ? 1 : 0;
  };
  oracle_group o{};
  o.a = g.blocks[0].received ? g.blocks[0].data : 0;
  o.b = g.blocks[1].received ? g.blocks[1].data : 0;
  o.c = g.blocks[2].received ? g.blocks[2].data : 0;
  o.d = g.blocks[3].received ? g.blocks[3].data : 0;
  o.errors = static_cast<uint8_t>((e(0) << 6) | (e(1) << 4) | (e(2) << 2) | e(3));
  o.block_index = blockIndex;
  return o;
}

struct RDSDecoder { // rds_decoder.cpp
  SubcarrierSet sub;
  BlockStream bs;
  explicit RDSDecoder(int fs) : sub(static_cast<float>(std::max(1, fs))) {}
  void reset() {
    sub.reset();
    bs = BlockStream();
  }
  template <typename GroupFn, typename BitFn>
  void process(const float *mpx, size_t n, GroupFn &&onGroup, BitFn &&onBit) {
    if (!mpx || n == 0) return;
    size_t off = 0;
    while (off < n) { // rds_decoder.cpp:80-92, 8192-sample chunks
      size_t chunk = std::min<size_t>(8192, n - off);
      sub.chunkToBits(mpx + off, chunk, [&](bool bit) {
        onBit(bit);
        bs.pushBit(bit);
        if (bs.hasReady) {
          bs.hasReady = false;
          onGroup(bs.ready);
        }
      });
      off += chunk;
    }
  }
};

/* ---- per-block pipeline harness: main.cpp:1232-1308 ---- */
struct Pipeline {
  oracle_cfg cfg;
  int M;
  ComplexDecimator decim;
  FMDemod demod;
  StereoDecoder stereo;
  AFPostProcessor af;
  std::unique_ptr<RDSDecoder> rds;
  std::vector<cf> bb;
  std::vector<float> mpx, l, r, ol, orr;
  uint32_t blockIndex = 0;
  // retuneMuteSamplesRemaining / retuneMuteTotalSamples (main.cpp:1034-1035)
  size_t muteRemaining = 0, muteTotal = 0;

  explicit Pipeline(const oracle_cfg &c)
      : cfg(c), M(c.iq_rate / c.dsp_rate), demod(c.dsp_rate, c.out_rate),
        stereo(c.dsp_rate, c.out_rate), af(c.dsp_rate, c.out_rate) {
    if (M < 1 || c.iq_rate % c.dsp_rate != 0) throw std::runtime_error("iq_rate must be k*dsp_rate");
    demod.setW0(c.w0_bandwidth_hz);
    demod.setDspAgcMode(c.dsp_agc);
    stereo.blendMode = c.blend;
    const uint32_t tpp = (M >= 8) ? 28u : ((M >= 4) ? 20u : 12u);
    decim.init(static_cast<uint32_t>(M), tpp, 80.0f);
    if (c.deemphasis == 0) {
      af.setDeemphasis(50);
      demod.setDeemphasis(50);
    } else if (c.deemphasis == 1) {
      af.setDeemphasis(75);
      demod.setDeemphasis(75);
    } else {
      af.setDeemphasis(0);
      demod.setDeemphasis(0);
    }
    stereo.forceMono = c.force_mono != 0;
    stereo.forceStereo = c.force_stereo != 0;
    demod.setBandwidthHz(c.bandwidth_hz);
    if (c.rds) rds = std::make_unique<RDSDecoder>(c.dsp_rate);
    bb.resize(c.block);
    mpx.resize(c.block);
    l.resize(c.block);
    r.resize(c.block);
    ol.resize(c.block);
    orr.resize(c.block);
  }
  void reset() {
    demod.reset();
    stereo.reset();
    af.reset();
    decim.reset();
    if (rds) rds->reset();
  }
  void retune(int muteSamples) {
    reset();
    const size_t k = (muteSamples < 0) ? static_cast<size_t>(cfg.out_rate / 25) : static_cast<size_t>(muteSamples);
    muteRemaining = k;
    muteTotal = k;
  }
  int block(const uint8_t *iq, int iqSamples, float *mpxOut, float *pl, float *pr, int cap,
            oracle_group *groups, int gcap, oracle_blockinfo *info) {
    size_t n;
    size_t nOut = 0;
    const size_t B = static_cast<size_t>(cfg.block);
    if (M > 1) {
      n = decim.executeComplex(iq, static_cast<size_t>(iqSamples), bb.data(), B);
    } else {
      n = std::min(static_cast<size_t>(iqSamples), B);
    }
    if (!cfg.stereo) {
      nOut = (M > 1) ? demod.processSplitComplex(bb.data(), mpx.data(), ol.data(), n)
                     : demod.processSplit(iq, mpx.data(), ol.data(), n);
      for (size_t i = 0; i < nOut; ++i) {
        const float m = ol[i] * 0.5f;
        ol[i] = m;
        orr[i] = m;
      }
    } else {
      if (M > 1) demod.processSplitComplex(bb.data(), mpx.data(), nullptr, n);
      else demod.processSplit(iq, mpx.data(), nullptr, n);
    }
    int ng = 0;
    if (rds) {
      rds->process(mpx.data(), n,
                   [&](const Group &g) {
                     if (groups && ng < gcap) groups[ng] = packGroup(g, blockIndex);
                     ng++;
                   },
                   [](bool) {});
    }
    int sd = 0, pt = 0;
    if (cfg.stereo) {
      size_t ns = stereo.processAudio(mpx.data(), l.data(), r.data(), n);
      nOut = af.process(l.data(), r.data(), ns, ol.data(), orr.data(), B);
      sd = stereo.stereoDetected ? 1 : 0;
      pt = stereo.pilotLevelTenthsKHz;
    }
    // XDR stereo indicator (main.cpp:1298-1300)
    const int indicator = (sd != 0 || (stereo.forceMono && cfg.stereo && pt >= 20)) ? 1 : 0;
    for (size_t i = 0; i < nOut; ++i) {
      ol[i] = std::clamp(ol[i], -1.0f, 1.0f);
      orr[i] = std::clamp(orr[i], -1.0f, 1.0f);
    }
    // retune fade-out / mute / fade-in (main.cpp:1310-1337)
    if (muteRemaining > 0 && nOut > 0) {
      const size_t muteCount = std::min(nOut, muteRemaining);
      const size_t alreadyMuted = (muteTotal > muteRemaining) ? (muteTotal - muteRemaining) : 0;
      const size_t fadeSamples =
          std::max<size_t>(1, std::min(static_cast<size_t>(cfg.out_rate / 200), muteTotal / 2));
      for (size_t i = 0; i < muteCount; ++i) {
        const size_t idx = alreadyMuted + i;
        float gain = 0.0f;
        if (idx < fadeSamples) {
          gain = 1.0f - (static_cast<float>(idx) / static_cast<float>(fadeSamples));
        } else if (idx >= (muteTotal - fadeSamples)) {
          const size_t tail = muteTotal - idx;
          gain = static_cast<float>(tail) / static_cast<float>(fadeSamples);
        }
        gain = std::clamp(gain, 0.0f, 1.0f);
        ol[i] *= gain;
        orr[i] *= gain;
      }
      muteRemaining -= muteCount;
      if (muteRemaining == 0) muteTotal = 0;
    }
    if (mpxOut) std::memcpy(mpxOut, mpx.data(), n * sizeof(float));
    size_t nc = std::min(nOut, static_cast<size_t>(std::max(cap, 0)));
    if (pl) std::memcpy(pl, ol.data(), nc * sizeof(float));
    if (pr) std::memcpy(pr, orr.data(), nc * sizeof(float));
    if (info) {
      info->n_mpx = static_cast<int>(n);
      info->n_pcm = static_cast<int>(nOut);
      info->stereo_detected = sd;
      info->pilot_tenths_khz = pt;
      info->clip_ratio = demod.clipRatio;
      info->n_groups = ng;
      info->stereo_indicator = indicator;
    }
    blockIndex++;
    return static_cast<int>(nOut);
  }
};

} // namespace ref

/* ========================================================================= */
extern "C" {

void *oracle_pipeline_create(const oracle_cfg *cfg) {
  try {
    return new ref::Pipeline(*cfg);
  } catch (...) {
    return nullptr;
  }
}
void oracle_pipeline_destroy(void *p) { delete static_cast<ref::Pipeline *>(p); }
void oracle_pipeline_reset(void *p) { static_cast<ref::Pipeline *>(p)->reset(); }
void oracle_pipeline_retune(void *p, int mute_samples) { static_cast<ref::Pipeline *>(p)->retune(mute_samples); }
int oracle_pipeline_block(void *p, const uint8_t *iq, int iq_samples, float *mpx_out, float *pcm_l,
                          float *pcm_r, int pcm_cap, oracle_group *groups, int groups_cap,
                          oracle_blockinfo *info) {
  return static_cast<ref::Pipeline *>(p)->block(iq, iq_samples, mpx_out, pcm_l, pcm_r, pcm_cap, groups,
                                                groups_cap, info);
}
/* main.cpp's runtime setter paths (XDR callbacks applied between blocks):
 * keys as include/fmx.h FMX_PARAM_*: 1 bandwidth Hz (main.cpp:1052-1062),
 * 2 W0, 3 deemphasis 0/1/2 (main.cpp:1123-1136), 4 dsp_agc, 5 blend,
 * 6 force mono, 7 force stereo, 8 bandwidth mode. */
void oracle_pipeline_set(void *pp, int key, int v) {
  auto *p = static_cast<ref::Pipeline *>(pp);
  switch (key) {
    case 1: p->demod.setBandwidthHz(v); break;
    case 2: p->demod.setW0(v); break;
    case 3:
      if (v == 0) {
        p->af.setDeemphasis(50);
        p->demod.setDeemphasis(50);
      } else if (v == 1) {
        p->af.setDeemphasis(75);
        p->demod.setDeemphasis(75);
      } else {
        p->af.setDeemphasis(0);
        p->demod.setDeemphasis(0);
      }
      break;
    case 4: p->demod.setDspAgcMode(v); break;
    case 5: p->stereo.blendMode = v; break;
    case 6: p->stereo.forceMono = v != 0; break;
    case 7: p->stereo.forceStereo = v != 0; break;
    case 8: p->demod.setBandwidthMode(v); break;
    case 9:  // setDeemphasis(tau_us) on both objects
      p->af.setDeemphasis(v);
      p->demod.setDeemphasis(v);
      break;
    case 10: p->demod.setDeviation(static_cast<double>(v)); break;
    default: break;
  }
}

int oracle_pipeline_taps(void *pp, int which, float *out, int cap) {
  auto *p = static_cast<ref::Pipeline *>(pp);
  std::vector<float> v;
  switch (which) {
    case 0: v = p->decim.taps; break;
    case 1: v = p->demod.iqFilter.taps; break;
    case 2: v = p->stereo.pilotBpf.taps; break;
    case 3: v = p->stereo.leftLpf.taps; break;
    case 4: v = p->af.lRs.r.proto; break;
    case 5:
      if (p->rds) v = p->rds->sub.resampler.proto;
      break;
    case 6:
      if (p->rds) v = p->rds->sub.lpf.taps;
      break;
    case 7:
      if (p->rds) v = p->rds->sub.symsync.h;
      break;
    case 8:
      if (p->rds) v = p->rds->sub.symsync.dh;
      break;
    default: return -1;
  }
  int n = static_cast<int>(v.size());
  if (out) std::memcpy(out, v.data(), static_cast<size_t>(std::min(n, cap)) * sizeof(float));
  return n;
}

void *oracle_decim_create(uint32_t factor, uint32_t tpp, float as) {
  auto *d = new ref::ComplexDecimator();
  d->init(factor, tpp, as);
  return d;
}
void oracle_decim_destroy(void *p) { delete static_cast<ref::ComplexDecimator *>(p); }
void oracle_decim_reset(void *p) { static_cast<ref::ComplexDecimator *>(p)->reset(); }
size_t oracle_decim_execute_complex(void *p, const uint8_t *iq, size_t n, float *out, size_t cap) {
  return static_cast<ref::ComplexDecimator *>(p)->executeComplex(iq, n, reinterpret_cast<cf *>(out), cap);
}
size_t oracle_decim_execute(void *p, const uint8_t *iq, size_t n, uint8_t *out, size_t cap) {
  return static_cast<ref::ComplexDecimator *>(p)->execute(iq, n, out, cap);
}

void *oracle_demod_create(int in, int out) { return new ref::FMDemod(in, out); }
void oracle_demod_destroy(void *p) { delete static_cast<ref::FMDemod *>(p); }
void oracle_demod_reset(void *p) { static_cast<ref::FMDemod *>(p)->reset(); }
/* keys: 1 deemphasis us, 2 W0 Hz, 3 bandwidth Hz, 4 agc mode, 5 deviation Hz,
 * 6 bandwidth mode (TEF table) */
void oracle_demod_set(void *pp, int key, int v) {
  auto *p = static_cast<ref::FMDemod *>(pp);
  switch (key) {
    case 1: p->setDeemphasis(v); break;
    case 2: p->setW0(v); break;
    case 3: p->setBandwidthHz(v); break;
    case 4: p->setDspAgcMode(v); break;
    case 5: p->setDeviation(static_cast<double>(v)); break;
    case 6: p->setBandwidthMode(v); break;
    default: break;
  }
}
size_t oracle_demod_process_split_complex(void *p, const float *iq, float *mpx, float *mono, size_t n) {
  return static_cast<ref::FMDemod *>(p)->processSplitComplex(reinterpret_cast<const cf *>(iq), mpx, mono, n);
}
size_t oracle_demod_process_split(void *p, const uint8_t *iq, float *mpx, float *mono, size_t n) {
  return static_cast<ref::FMDemod *>(p)->processSplit(iq, mpx, mono, n);
}
float oracle_demod_clip_ratio(void *p) { return static_cast<ref::FMDemod *>(p)->clipRatio; }

void *oracle_stereo_create(int in, int out) { return new ref::StereoDecoder(in, out); }
void oracle_stereo_destroy(void *p) { delete static_cast<ref::StereoDecoder *>(p); }
void oracle_stereo_reset(void *p) { static_cast<ref::StereoDecoder *>(p)->reset(); }
/* keys: 1 blend mode, 2 force mono, 3 force stereo */
void oracle_stereo_set(void *pp, int key, int v) {
  auto *p = static_cast<ref::StereoDecoder *>(pp);
  if (key == 1) p->blendMode = v;
  else if (key == 2) p->forceMono = v != 0;
  else if (key == 3) p->forceStereo = v != 0;
}
size_t oracle_stereo_process(void *pp, const float *mpx, float *l, float *r, size_t n, int *st, int *pt) {
  auto *p = static_cast<ref::StereoDecoder *>(pp);
  size_t k = p->processAudio(mpx, l, r, n);
  if (st) *st = p->stereoDetected ? 1 : 0;
  if (pt) *pt = p->pilotLevelTenthsKHz;
  return k;
}
size_t oracle_stereo_process_trace(void *pp, const float *mpx, float *l, float *r, size_t n, float *ph,
                                   float *bl) {
  return static_cast<ref::StereoDecoder *>(pp)->processAudio(mpx, l, r, n, ph, bl);
}

void *oracle_afpost_create(int in, int out) { return new ref::AFPostProcessor(in, out); }
void oracle_afpost_destroy(void *p) { delete static_cast<ref::AFPostProcessor *>(p); }
void oracle_afpost_reset(void *p) { static_cast<ref::AFPostProcessor *>(p)->reset(); }
void oracle_afpost_set_deemphasis(void *p, int tau) { static_cast<ref::AFPostProcessor *>(p)->setDeemphasis(tau); }
size_t oracle_afpost_process(void *p, const float *l, const float *r, size_t n, float *ol, float *or_,
                             size_t cap) {
  return static_cast<ref::AFPostProcessor *>(p)->process(l, r, n, ol, or_, cap);
}

void *oracle_rds_create(int fs) { return new ref::RDSDecoder(fs); }
void oracle_rds_destroy(void *p) { delete static_cast<ref::RDSDecoder *>(p); }
void oracle_rds_reset(void *p) { static_cast<ref::RDSDecoder *>(p)->reset(); }
int oracle_rds_process(void *pp, const float *mpx, size_t n, oracle_group *groups, int cap, uint8_t *bits,
                       int bits_cap, int *n_bits) {
  auto *p = static_cast<ref::RDSDecoder *>(pp);
  int ng = 0, nb = 0;
  p->process(
      mpx, n,
      [&](const ref::Group &g) {
        if (groups && ng < cap) groups[ng] = ref::packGroup(g, 0);
        ng++;
      },
      [&](bool b) {
        if (bits && nb < bits_cap) bits[nb] = b ? 1 : 0;
        nb++;
      });
  if (n_bits) *n_bits = nb;
  return ng;
}

void *oracle_blocksync_create(void) { return new ref::BlockStream(); }
void oracle_blocksync_destroy(void *p) { delete static_cast<ref::BlockStream *>(p); }
int oracle_blocksync_push(void *pp, const uint8_t *bits, int n, oracle_group *groups, int cap) {
  auto *p = static_cast<ref::BlockStream *>(pp);
  int ng = 0;
  for (int i = 0; i < n; ++i) {
    p->pushBit(bits[i] != 0);
    if (p->hasReady) {
      p->hasReady = false;
      if (groups && ng < cap) groups[ng] = ref::packGroup(p->ready, static_cast<uint32_t>(i));
      ng++;
    }
  }
  return ng;
}

double oracle_run_many(const oracle_cfg *cfg, int n_channels, const uint8_t *iq, int n_blocks, int threads,
                       double *checksum) {
  if (threads < 1) threads = 1;
  const int M = cfg->iq_rate / cfg->dsp_rate;
  const size_t blockBytes = static_cast<size_t>(2) * static_cast<size_t>(cfg->block) * static_cast<size_t>(M);
  std::vector<std::unique_ptr<ref::Pipeline>> pipes(static_cast<size_t>(n_channels));
  for (int c = 0; c < n_channels; ++c) pipes[static_cast<size_t>(c)] = std::make_unique<ref::Pipeline>(*cfg);
  std::vector<double> sums(static_cast<size_t>(n_channels), 0.0);
  std::atomic<int> next{0};
  auto t0 = std::chrono::steady_clock::now();
  auto worker = [&]() {
    std::vector<float> pl(static_cast<size_t>(cfg->block)), pr(static_cast<size_t>(cfg->block));
    std::vector<oracle_group> g(64);
    for (;;) {
      int c = next.fetch_add(1);
      if (c >= n_channels) break;
      double s = 0.0;
      for (int b = 0; b < n_blocks; ++b) {
        const uint8_t *src = iq + (static_cast<size_t>(c) * n_blocks + b) * blockBytes;
        oracle_blockinfo info{};
        int n = pipes[static_cast<size_t>(c)]->block(src, cfg->block * M, nullptr, pl.data(), pr.data(),
                                                     cfg->block, g.data(), 64, &info);
        for (int i = 0; i < n; ++i) s += pl[static_cast<size_t>(i)] + 0.5 * pr[static_cast<size_t>(i)];
        s += info.n_groups;
      }
      sums[static_cast<size_t>(c)] = s;
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t) th.emplace_back(worker);
  for (auto &t : th) t.join();
  auto t1 = std::chrono::steady_clock::now();
  double tot = 0.0;
  for (double v : sums) tot += v;
  if (checksum) *checksum = tot;
  return std::chrono::duration<double>(t1 - t0).count();
}

} // extern "C"

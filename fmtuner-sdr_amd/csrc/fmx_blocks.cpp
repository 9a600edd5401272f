// fmx_blocks.cpp -- the C++ facades of include/fmx_blocks.hpp over the C ABI.
//
// A facade object owns a one-channel handle (fmx_create with C = 1) whose
// configuration reproduces the reference object's constructor defaults:
// FMDemod ctor IQ filter (bandwidth_hz = -1 keeps it, fm_demod.cpp:29-46),
// 75 us de-emphasis (fm_demod.cpp:44, af_post_processor.h:25), AGC off,
// blend Normal (stereo_decoder.cpp:27).  Calls longer than the handle's block
// are split into block-sized pieces; state carries across pieces exactly as
// across calls.
#include "fmx_blocks.hpp"

#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <string>

namespace fmx {
namespace detail {

static constexpr int kSlotBlock = 8192;  // processing.dsp_block_samples default (config.h:49)

class Slot {
public:
  Slot(int iq_rate, int dsp_rate, int out_rate) {
    if (fmx_device_count() <= 0) throw std::runtime_error("fmx: no MI355X (HIP) device");
    fmx_config c{};
    c.iq_rate = iq_rate;
    c.dsp_rate = dsp_rate;
    c.out_rate = out_rate;
    c.block = kSlotBlock;
    c.w0_bandwidth_hz = 194000;
    c.bandwidth_hz = -1;  // keep the constructor's IQ filter
    c.dsp_agc = FMX_AGC_OFF;
    c.stereo = 1;
    c.blend = FMX_BLEND_NORMAL;
    c.deemphasis = FMX_DEEMPH_75US;
    c.rds = 1;
    const int rc = fmx_create(&c, 1, 0, &h);
    if (rc != FMX_OK) {
      std::string msg = h ? fmx_last_error(h) : "";
      if (h) fmx_destroy(h);
      h = nullptr;
      throw std::runtime_error("fmx_create failed: " + msg);
    }
    for (auto &b : buf) b = nullptr;
  }
  ~Slot() {
    for (auto &b : buf)
      if (b) fmx_free(h, b);
    if (h) fmx_destroy(h);
  }
  Slot(const Slot &) = delete;
  Slot &operator=(const Slot &) = delete;

  void check(int rc, const char *what) const {
    if (rc != FMX_OK) throw std::runtime_error(std::string(what) + ": " + fmx_last_error(h));
  }
  // device scratch i (0..5) of at least `bytes`
  void *dev(int i, size_t bytes) {
    if (cap[i] < bytes) {
      if (buf[i]) fmx_free(h, buf[i]);
      buf[i] = nullptr;
      check(fmx_malloc(h, &buf[i], bytes), "fmx_malloc");
      cap[i] = bytes;
    }
    return buf[i];
  }
  void up(void *d, const void *hs, size_t bytes) { check(fmx_memcpy_h2d(h, d, hs, bytes), "fmx_memcpy_h2d"); }
  void down(void *hd, const void *d, size_t bytes) { check(fmx_memcpy_d2h(h, hd, d, bytes), "fmx_memcpy_d2h"); }
  int down_int(const void *d) {
    int v = 0;
    down(&v, d, sizeof(int));
    return v;
  }
  void set(int key, int value) { check(fmx_set_param(h, 0, key, value), "fmx_set_param"); }
  void reset() { check(fmx_reset(h, 0), "fmx_reset"); }

  void *h = nullptr;
  void *buf[6];
  size_t cap[6] = {0, 0, 0, 0, 0, 0};
};


}  // namespace detail

using detail::kSlotBlock;
using detail::Slot;

/* ---------------- ComplexDecimator ---------------- */
ComplexDecimator::ComplexDecimator() = default;
ComplexDecimator::~ComplexDecimator() = default;

void ComplexDecimator::init(std::uint32_t factor, std::uint32_t tapsPerPhase, float stopBandAtten) {
  if (factor == 0) throw std::runtime_error("complex decimator factor must be >= 1");
  const std::uint32_t tpp = std::max<std::uint32_t>(4, tapsPerPhase);
  const std::uint32_t want = (factor >= 8U) ? 28U : ((factor >= 4U) ? 20U : 12U);
  const bool ok = (factor == 2 || factor == 4 || factor == 8 || factor == 10) && tpp == want &&
                  stopBandAtten == 80.0f;
  if (!ok)
    throw std::invalid_argument("fmx: ComplexDecimator supports the main.cpp designs "
                                "(factor 2/4/8/10, taps/phase 12/20/28/28, As 80)");
  factor_ = factor;
  slot_ = std::make_unique<Slot>(240000 * static_cast<int>(factor), 240000, 32000);
}

void ComplexDecimator::reset() {
  if (slot_) slot_->reset();
}

std::size_t ComplexDecimator::executeComplex(const uint8_t *iqIn, std::size_t inSamples, std::complex<float> *iqOut,
                                             std::size_t outCapacity) const {
  if (!iqIn || !iqOut || inSamples == 0 || outCapacity == 0 || !slot_) return 0;
  const std::size_t blocks = std::min(inSamples / factor_, outCapacity);
  std::size_t done = 0;
  while (done < blocks) {
    const int n = static_cast<int>(std::min<std::size_t>(blocks - done, kSlotBlock));
    const size_t in_bytes = 2 * static_cast<size_t>(n) * factor_;
    void *d_in = slot_->dev(0, in_bytes);
    void *d_out = slot_->dev(1, 8 * static_cast<size_t>(n));
    slot_->up(d_in, iqIn + 2 * done * factor_, in_bytes);
    slot_->check(fmx_decimate(slot_->h, static_cast<const uint8_t *>(d_in), in_bytes, n, static_cast<float *>(d_out),
                              2 * n),
                 "fmx_decimate");
    slot_->down(iqOut + done, d_out, 8 * static_cast<size_t>(n));
    done += static_cast<std::size_t>(n);
  }
  return blocks;
}

std::size_t ComplexDecimator::execute(const uint8_t *iqIn, std::size_t inSamples, uint8_t *iqOut,
                                      std::size_t outCapacity) const {
  if (!iqIn || !iqOut || inSamples == 0 || outCapacity == 0 || !slot_) return 0;
  const std::size_t blocks = std::min(inSamples / factor_, outCapacity);
  std::size_t done = 0;
  while (done < blocks) {
    const int n = static_cast<int>(std::min<std::size_t>(blocks - done, kSlotBlock));
    const size_t in_bytes = 2 * static_cast<size_t>(n) * factor_;
    void *d_in = slot_->dev(0, in_bytes);
    void *d_out = slot_->dev(1, 2 * static_cast<size_t>(n));
    slot_->up(d_in, iqIn + 2 * done * factor_, in_bytes);
    slot_->check(fmx_decimate_u8(slot_->h, static_cast<const uint8_t *>(d_in), in_bytes, n,
                                 static_cast<uint8_t *>(d_out), 2 * static_cast<size_t>(n)),
                 "fmx_decimate_u8");
    slot_->down(iqOut + 2 * done, d_out, 2 * static_cast<size_t>(n));
    done += static_cast<std::size_t>(n);
  }
  return blocks;
}

/* ---------------- FMDemod ---------------- */
FMDemod::FMDemod(int inputRate, int outputRate)
    : inputRate_(std::max(1, inputRate)), outputRate_(std::max(1, outputRate)) {
  slot_ = std::make_unique<Slot>(inputRate_, inputRate_, outputRate_);
}
FMDemod::~FMDemod() = default;

std::size_t FMDemod::processSplit(const uint8_t *iq, float *mpxOut, float *monoOut, std::size_t n) {
  if (!iq || !mpxOut || n == 0) return 0;
  std::size_t done = 0, mono = 0;
  int clipped = 0;
  while (done < n) {
    const int m = static_cast<int>(std::min<std::size_t>(n - done, kSlotBlock));
    void *d_in = slot_->dev(0, 2 * static_cast<size_t>(m));
    float *d_mpx = static_cast<float *>(slot_->dev(1, 4 * static_cast<size_t>(m)));
    float *d_mono = monoOut ? static_cast<float *>(slot_->dev(2, 4 * static_cast<size_t>(m))) : nullptr;
    int *d_cnt = static_cast<int *>(slot_->dev(3, sizeof(int)));
    float *d_clip = static_cast<float *>(slot_->dev(4, sizeof(float)));
    slot_->up(d_in, iq + 2 * done, 2 * static_cast<size_t>(m));
    slot_->check(fmx_demod_u8(slot_->h, static_cast<const uint8_t *>(d_in), 2 * static_cast<size_t>(m), m, d_mpx, m,
                              d_mono, m, d_cnt, d_clip),
                 "fmx_demod_u8");
    slot_->down(mpxOut + done, d_mpx, 4 * static_cast<size_t>(m));
    float ratio = 0.0f;
    slot_->down(&ratio, d_clip, sizeof(float));
    clipped += static_cast<int>(ratio * static_cast<float>(m) + 0.5f);
    if (monoOut) {
      const int k = slot_->down_int(d_cnt);
      slot_->down(monoOut + mono, d_mono, 4 * static_cast<size_t>(k));
      mono += static_cast<std::size_t>(k);
    }
    done += static_cast<std::size_t>(m);
  }
  clipRatio_ = static_cast<float>(clipped) / static_cast<float>(n);
  clipping_ = clipped > 0;
  return mono;
}

std::size_t FMDemod::processSplitComplex(const std::complex<float> *iq, float *mpxOut, float *monoOut, std::size_t n) {
  if (!iq || !mpxOut || n == 0) return 0;
  std::size_t done = 0, mono = 0;
  while (done < n) {
    const int m = static_cast<int>(std::min<std::size_t>(n - done, kSlotBlock));
    float *d_in = static_cast<float *>(slot_->dev(0, 8 * static_cast<size_t>(m)));
    float *d_mpx = static_cast<float *>(slot_->dev(1, 4 * static_cast<size_t>(m)));
    float *d_mono = monoOut ? static_cast<float *>(slot_->dev(2, 4 * static_cast<size_t>(m))) : nullptr;
    int *d_cnt = static_cast<int *>(slot_->dev(3, sizeof(int)));
    slot_->up(d_in, iq + done, 8 * static_cast<size_t>(m));
    slot_->check(fmx_demod(slot_->h, d_in, 2 * m, m, d_mpx, m, d_mono, m, d_cnt), "fmx_demod");
    slot_->down(mpxOut + done, d_mpx, 4 * static_cast<size_t>(m));
    if (monoOut) {
      const int k = slot_->down_int(d_cnt);
      slot_->down(monoOut + mono, d_mono, 4 * static_cast<size_t>(k));
      mono += static_cast<std::size_t>(k);
    }
    done += static_cast<std::size_t>(m);
  }
  return mono;
}

std::size_t FMDemod::downsampleAudio(const float *demod, float *audio, std::size_t numSamples) {
  if (!demod || !audio || numSamples == 0) return 0;
  std::size_t done = 0, out = 0;
  while (done < numSamples) {
    const int m = static_cast<int>(std::min<std::size_t>(numSamples - done, kSlotBlock));
    float *d_in = static_cast<float *>(slot_->dev(0, 4 * static_cast<size_t>(m)));
    float *d_out = static_cast<float *>(slot_->dev(1, 4 * static_cast<size_t>(m)));
    int *d_cnt = static_cast<int *>(slot_->dev(3, sizeof(int)));
    slot_->up(d_in, demod + done, 4 * static_cast<size_t>(m));
    slot_->check(fmx_downsample(slot_->h, d_in, m, m, d_out, m, d_cnt), "fmx_downsample");
    const int k = slot_->down_int(d_cnt);
    slot_->down(audio + out, d_out, 4 * static_cast<size_t>(k));
    out += static_cast<std::size_t>(k);
    done += static_cast<std::size_t>(m);
  }
  return out;
}

void FMDemod::process(const uint8_t *iq, float *audio, std::size_t numSamples) {
  // demodulate + downsampleAudio: the MPX goes to a scratch, the audio out
  if (!iq || !audio || numSamples == 0) return;
  scratch_.resize(numSamples);
  lastAudio_ = processSplit(iq, scratch_.data(), audio, numSamples);
}
void FMDemod::processComplex(const std::complex<float> *iq, float *audio, std::size_t numSamples) {
  if (!iq || !audio || numSamples == 0) return;
  scratch_.resize(numSamples);
  lastAudio_ = processSplitComplex(iq, scratch_.data(), audio, numSamples);
}
void FMDemod::processNoDownsample(const uint8_t *iq, float *audio, std::size_t numSamples) {
  if (!iq || !audio || numSamples == 0) return;
  processSplit(iq, audio, nullptr, numSamples);
}
void FMDemod::reset() { slot_->reset(); }
void FMDemod::setDeemphasis(int tau_us) { slot_->set(FMX_PARAM_DEEMPH_US, tau_us); }
void FMDemod::setDeviation(double deviation) {
  const double hz = std::floor(deviation + 0.5);
  if (!(hz >= 1.0 && hz <= 1e9)) throw std::invalid_argument("fmx: FMDemod deviation must be 1 Hz .. 1 GHz");
  slot_->set(FMX_PARAM_DEVIATION_HZ, static_cast<int>(hz));
}
void FMDemod::setBandwidthMode(int mode) { slot_->set(FMX_PARAM_BANDWIDTH_MODE, mode); }
void FMDemod::setBandwidthHz(int bwHz) { slot_->set(FMX_PARAM_BANDWIDTH_HZ, bwHz); }
void FMDemod::setW0BandwidthHz(int bwHz) { slot_->set(FMX_PARAM_W0_HZ, bwHz); }
void FMDemod::setDspAgcMode(DspAgcMode mode) { slot_->set(FMX_PARAM_DSP_AGC, static_cast<int>(mode)); }

/* ---------------- StereoDecoder ---------------- */
StereoDecoder::StereoDecoder(int inputRate, int outputRate) {
  slot_ = std::make_unique<Slot>(std::max(1, inputRate), std::max(1, inputRate), std::max(1, outputRate));
}
StereoDecoder::~StereoDecoder() = default;

std::size_t StereoDecoder::processAudio(const float *mono, float *left, float *right, std::size_t numSamples) {
  if (!mono || !left || !right || numSamples == 0) return 0;
  std::size_t done = 0;
  while (done < numSamples) {
    const int m = static_cast<int>(std::min<std::size_t>(numSamples - done, kSlotBlock));
    float *d_in = static_cast<float *>(slot_->dev(0, 4 * static_cast<size_t>(m)));
    float *d_l = static_cast<float *>(slot_->dev(1, 4 * static_cast<size_t>(m)));
    float *d_r = static_cast<float *>(slot_->dev(2, 4 * static_cast<size_t>(m)));
    int *d_st = static_cast<int *>(slot_->dev(3, 2 * sizeof(int)));
    slot_->up(d_in, mono + done, 4 * static_cast<size_t>(m));
    slot_->check(fmx_stereo(slot_->h, d_in, m, m, d_l, d_r, m, d_st, d_st + 1), "fmx_stereo");
    slot_->down(left + done, d_l, 4 * static_cast<size_t>(m));
    slot_->down(right + done, d_r, 4 * static_cast<size_t>(m));
    int flags[2] = {0, 0};
    slot_->down(flags, d_st, sizeof(flags));
    stereo_ = flags[0] != 0;
    pilotTenths_ = flags[1];
    done += static_cast<std::size_t>(m);
  }
  return numSamples;
}
void StereoDecoder::reset() { slot_->reset(); }
void StereoDecoder::setForceStereo(bool force) { slot_->set(FMX_PARAM_FORCE_STEREO, force ? 1 : 0); }
void StereoDecoder::setForceMono(bool force) { slot_->set(FMX_PARAM_FORCE_MONO, force ? 1 : 0); }
void StereoDecoder::setBlendMode(BlendMode mode) { slot_->set(FMX_PARAM_BLEND, static_cast<int>(mode)); }

/* ---------------- AFPostProcessor ---------------- */
AFPostProcessor::AFPostProcessor(int inputRate, int outputRate)
    : inputRate_(std::max(1, inputRate)), outputRate_(std::max(1, outputRate)) {
  slot_ = std::make_unique<Slot>(inputRate_, inputRate_, outputRate_);
}
AFPostProcessor::~AFPostProcessor() = default;
void AFPostProcessor::reset() { slot_->reset(); }
void AFPostProcessor::setDeemphasis(int tau_us) { slot_->set(FMX_PARAM_DEEMPH_US, tau_us); }

std::size_t AFPostProcessor::process(const float *inL, const float *inR, std::size_t inSamples, float *outL,
                                     float *outR, std::size_t outCapacity) {
  if (!inL || !inR || !outL || !outR || inSamples == 0 || outCapacity == 0) return 0;
  std::size_t done = 0, out = 0;
  while (done < inSamples && out < outCapacity) {
    const int m = static_cast<int>(std::min<std::size_t>(inSamples - done, kSlotBlock));
    const int cap = static_cast<int>(std::min<std::size_t>(outCapacity - out, kSlotBlock));
    float *d_l = static_cast<float *>(slot_->dev(0, 4 * static_cast<size_t>(m)));
    float *d_r = static_cast<float *>(slot_->dev(1, 4 * static_cast<size_t>(m)));
    float *d_ol = static_cast<float *>(slot_->dev(2, 4 * static_cast<size_t>(kSlotBlock)));
    float *d_or = static_cast<float *>(slot_->dev(4, 4 * static_cast<size_t>(kSlotBlock)));
    int *d_cnt = static_cast<int *>(slot_->dev(3, sizeof(int)));
    slot_->up(d_l, inL + done, 4 * static_cast<size_t>(m));
    slot_->up(d_r, inR + done, 4 * static_cast<size_t>(m));
    slot_->check(fmx_afpost(slot_->h, d_l, d_r, m, m, d_ol, d_or, kSlotBlock, cap, d_cnt), "fmx_afpost");
    const int k = slot_->down_int(d_cnt);
    slot_->down(outL + out, d_ol, 4 * static_cast<size_t>(k));
    slot_->down(outR + out, d_or, 4 * static_cast<size_t>(k));
    out += static_cast<std::size_t>(k);
    done += static_cast<std::size_t>(m);
  }
  return out;
}

/* ---------------- RDSDecoder ---------------- */
RDSDecoder::RDSDecoder(int inputRate) {
  const int fs = std::max(1, inputRate);
  slot_ = std::make_unique<Slot>(fs, fs, 32000);
}
RDSDecoder::~RDSDecoder() = default;
void RDSDecoder::reset() { slot_->reset(); }

void RDSDecoder::process(const float *mpx, std::size_t numSamples, const std::function<void(const RDSGroup &)> &onGroup) {
  if (!mpx || numSamples == 0) return;
  constexpr int kCap = 64;
  std::size_t done = 0;
  while (done < numSamples) {
    const int m = static_cast<int>(std::min<std::size_t>(numSamples - done, kSlotBlock));
    float *d_in = static_cast<float *>(slot_->dev(0, 4 * static_cast<size_t>(m)));
    auto *d_g = static_cast<fmx_rds_group *>(slot_->dev(1, sizeof(fmx_rds_group) * kCap));
    int *d_cnt = static_cast<int *>(slot_->dev(3, sizeof(int)));
    slot_->up(d_in, mpx + done, 4 * static_cast<size_t>(m));
    slot_->check(fmx_rds(slot_->h, d_in, m, m, d_g, kCap, d_cnt), "fmx_rds");
    const int k = std::min(kCap, slot_->down_int(d_cnt));
    fmx_rds_group g[kCap];
    if (k > 0) slot_->down(g, d_g, sizeof(fmx_rds_group) * static_cast<size_t>(k));
    for (int i = 0; i < k; ++i) {
      if (onGroup) onGroup(RDSGroup{g[i].a, g[i].b, g[i].c, g[i].d, g[i].errors});
    }
    done += static_cast<std::size_t>(m);
  }
}

/* ---------------- Receiver ---------------- */
Receiver::Receiver(const fmx_config &cfg, int channels, int device) : channels_(channels) {
  const int rc = fmx_create(&cfg, channels, device, &h_);
  if (rc != FMX_OK) {
    std::string msg = h_ ? fmx_last_error(h_) : "";
    if (h_) fmx_destroy(h_);
    h_ = nullptr;
    throw std::runtime_error("fmx_create failed: " + msg);
  }
}
Receiver::~Receiver() {
  if (h_) fmx_destroy(h_);
}
void Receiver::processBlock(const uint8_t *d_iq, std::size_t iq_stride, int n, const fmx_block_out &out) {
  if (fmx_process_block(h_, d_iq, iq_stride, n, &out) != FMX_OK)
    throw std::runtime_error(std::string("fmx_process_block: ") + fmx_last_error(h_));
}
void Receiver::reset(int channel) {
  if (fmx_reset(h_, channel) != FMX_OK) throw std::runtime_error(std::string("fmx_reset: ") + fmx_last_error(h_));
}
void Receiver::setParam(int channel, int key, int value) {
  if (fmx_set_param(h_, channel, key, value) != FMX_OK)
    throw std::runtime_error(std::string("fmx_set_param: ") + fmx_last_error(h_));
}
void Receiver::sync() {
  if (fmx_sync(h_) != FMX_OK) throw std::runtime_error(std::string("fmx_sync: ") + fmx_last_error(h_));
}

}  // namespace fmx

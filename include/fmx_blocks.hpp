// fmx_blocks.hpp -- C++17 facades with the reference's block-process API,
// running on MI355X through the C ABI of include/fmx.h.
//
// Each class keeps the method names, argument meaning and return values of
// the reference class it replaces, so a maintainer can swap the include and
// the type name and leave main.cpp, the XDR server and the audio sinks as
// they are:
//
//   fmx::ComplexDecimator  <- fm_tuner::dsp::liquid::ComplexDecimator
//                             (include/dsp/liquid_primitives.h:161-188)
//   fmx::FMDemod           <- FMDemod          (include/fm_demod.h:11-67)
//   fmx::StereoDecoder     <- StereoDecoder    (include/stereo_decoder.h:10-55)
//   fmx::AFPostProcessor   <- AFPostProcessor  (include/af_post_processor.h:9-37)
//   fmx::RDSDecoder        <- RDSDecoder       (include/rds_decoder.h:17-29)
//
// One facade object = one channel slot of its own GPU handle; buffers are
// host pointers (copied through HBM per call).  The many-channel entry point
// for new code is fmx::Receiver (a thin owner of fmx_process_block).
//
// Error behaviour follows the reference: construction / design failures
// throw std::runtime_error and null or empty inputs return 0.  Settings the
// GPU build does not implement (ComplexDecimator designs other than the ones
// main.cpp creates) throw std::invalid_argument instead of silently
// differing.  There is no CPU fallback: without a GPU the constructors throw.
#ifndef FMX_BLOCKS_HPP
#define FMX_BLOCKS_HPP

#include <complex>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <memory>
#include <vector>

#include "fmx.h"

namespace fmx {

namespace detail {
class Slot;  // one-channel handle + device staging buffers (fmx_blocks.cpp)
}

class ComplexDecimator {
public:
  ComplexDecimator();
  ~ComplexDecimator();
  ComplexDecimator(const ComplexDecimator &) = delete;
  ComplexDecimator &operator=(const ComplexDecimator &) = delete;

  // Supported: the designs main.cpp:670-674 creates (factor 2/4/8/10 with
  // taps-per-phase 12/20/28/28, As 80).
  void init(std::uint32_t factor, std::uint32_t tapsPerPhase = 12, float stopBandAtten = 70.0f);
  void reset();
  // Like the reference: min(inSamples / factor, outCapacity) outputs; a
  // remainder of inSamples % factor samples is dropped, not buffered.  const
  // as in the reference (the filter state lives in the device handle).
  std::size_t executeComplex(const uint8_t *iqIn, std::size_t inSamples, std::complex<float> *iqOut,
                             std::size_t outCapacity) const;
  // u8 -> u8: the same decimation requantised to interleaved bytes
  // (liquid_primitives.cpp:422-459)
  std::size_t execute(const uint8_t *iqIn, std::size_t inSamples, uint8_t *iqOut, std::size_t outCapacity) const;
  bool ready() const { return slot_ != nullptr; }
  std::uint32_t factor() const { return factor_; }

private:
  std::unique_ptr<detail::Slot> slot_;
  std::uint32_t factor_ = 1;
};

class FMDemod {
public:
  enum class DspAgcMode { Off = 0, Fast = 1, Slow = 2 };
  FMDemod(int inputRate, int outputRate);
  ~FMDemod();

  // demodulate + downsampleAudio into audio (fm_demod.cpp:228-243); the
  // reference returns nothing, the 32 kHz count is getLastAudioCount()
  void process(const uint8_t *iq, float *audio, std::size_t numSamples);
  void processComplex(const std::complex<float> *iq, float *audio, std::size_t numSamples);
  // discriminator MPX only (fm_demod.cpp:276-279)
  void processNoDownsample(const uint8_t *iq, float *audio, std::size_t numSamples);
  std::size_t getLastAudioCount() const { return lastAudio_; }
  // mpxOut: n discriminator samples; monoOut (may be null): 32 kHz audio
  // (downsampleAudio of the MPX); returns the mono sample count.
  std::size_t processSplit(const uint8_t *iq, float *mpxOut, float *monoOut, std::size_t n);
  std::size_t processSplitComplex(const std::complex<float> *iq, float *mpxOut, float *monoOut, std::size_t n);
  std::size_t downsampleAudio(const float *demod, float *audio, std::size_t numSamples);
  void reset();

  void setDeemphasis(int tau_us);       // any tau, <= 0 = off (fm_demod.cpp:50-62)
  void setDeviation(double deviation);  // Hz, rounded to an integer (fm_demod.cpp:64-71)
  void setBandwidthMode(int mode);
  void setBandwidthHz(int bwHz);
  void setW0BandwidthHz(int bwHz);
  void setDspAgcMode(DspAgcMode mode);
  bool isClipping() const { return clipping_; }
  float getClippingRatio() const { return clipRatio_; }

private:
  std::unique_ptr<detail::Slot> slot_;
  int inputRate_, outputRate_;
  bool clipping_ = false;
  float clipRatio_ = 0.0f;
  std::size_t lastAudio_ = 0;
  std::vector<float> scratch_;
};

class StereoDecoder {
public:
  enum class BlendMode { Soft = 0, Normal = 1, Aggressive = 2 };
  StereoDecoder(int inputRate, int outputRate);
  ~StereoDecoder();

  std::size_t processAudio(const float *mono, float *left, float *right, std::size_t numSamples);
  void reset();
  void setForceStereo(bool force);
  void setForceMono(bool force);
  void setBlendMode(BlendMode mode);
  int getPilotLevelTenthsKHz() const { return pilotTenths_; }
  bool isStereo() const { return stereo_; }

private:
  std::unique_ptr<detail::Slot> slot_;
  int pilotTenths_ = 0;
  bool stereo_ = false;
};

class AFPostProcessor {
public:
  AFPostProcessor(int inputRate, int outputRate);
  ~AFPostProcessor();

  void reset();
  void setDeemphasis(int tau_us);  // any tau, <= 0 = off (af_post_processor.cpp:31-45)
  std::size_t process(const float *inL, const float *inR, std::size_t inSamples, float *outL, float *outR,
                      std::size_t outCapacity);

private:
  std::unique_ptr<detail::Slot> slot_;
  int inputRate_, outputRate_;
};

struct RDSGroup {  // rds_decoder.h:9-15
  uint16_t blockA, blockB, blockC, blockD;
  uint8_t errors;
};

class RDSDecoder {
public:
  explicit RDSDecoder(int inputRate);
  ~RDSDecoder();
  void reset();
  void process(const float *mpx, std::size_t numSamples, const std::function<void(const RDSGroup &)> &onGroup);

private:
  std::unique_ptr<detail::Slot> slot_;
};

// Many channels at once: one fmx_process_block per reference block.
class Receiver {
public:
  Receiver(const fmx_config &cfg, int channels, int device = 0);
  ~Receiver();
  Receiver(const Receiver &) = delete;
  Receiver &operator=(const Receiver &) = delete;
  void *handle() const { return h_; }
  int channels() const { return channels_; }
  // d_iq: device [channels][iq_stride] u8; out: device buffers (fmx.h)
  void processBlock(const uint8_t *d_iq, std::size_t iq_stride, int n, const fmx_block_out &out);
  void reset(int channel = -1);
  void setParam(int channel, int key, int value);
  void sync();

private:
  void *h_ = nullptr;
  int channels_ = 0;
};

}  // namespace fmx

#endif

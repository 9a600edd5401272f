/*
 * fmx.h -- C ABI of the MI355X many-channel FM demodulator (libfmx.so).
 *
 * This is the drop-in boundary for bkram/fmtuner-sdr's per-block DSP hot path
 * (SURVEY.md 8b).  One handle holds N independent channels, each with the
 * exact state of one set of reference objects:
 *
 *   ComplexDecimator   include/dsp/liquid_primitives.h:161-188
 *   FMDemod            include/fm_demod.h:11-67
 *   StereoDecoder      include/stereo_decoder.h:10-55
 *   AFPostProcessor    include/af_post_processor.h:9-37
 *   RDSDecoder         include/rds_decoder.h:17-29
 *
 * and one call of fmx_process_block() replaces one iteration of the
 * reference's per-block body (src/main.cpp:1239-1308) for every channel.
 * The C++ facades in include/fmx_blocks.hpp map one reference object onto one
 * channel slot and keep the reference's method signatures.
 *
 * Conventions (reference-compatible):
 *   - sizes are SAMPLES, not bytes; IQ buffers are 2*n bytes, I then Q;
 *   - the caller owns every buffer; outputs are written from index 0;
 *   - functions return 0 (FMX_OK) or a negative FMX_E* code; the message is
 *     available from fmx_last_error(); nothing throws across the ABI;
 *   - pointers named d_* are DEVICE pointers (hipMalloc'd memory on the
 *     handle's device), pointers named h_* are host pointers;
 *   - a handle is not thread-safe (like the reference objects); all work is
 *     queued on the handle's own HIP stream, fmx_sync() waits for it.
 *
 * No HIP or torch types appear in this header.
 */
#ifndef FMX_H
#define FMX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI history: 9 (round 6) adds fmx_diag_set / fmx_diag_rds_ring and fmx_build_info; 8 (round 5) adds FMX_K_BITS (FMX_K_COUNT 8); 7 (round 5) adds fmx_host_stats and FMX_K_FRONTEND_GENERIC (FMX_K_COUNT 7); 6 (round 4) adds FMX_K_PILOT (FMX_K_COUNT 6); 5 (round 4) added FMX_K_RS (FMX_K_COUNT 5; fmx_kernel_times
 * fills at most n entries); 4 (round 3) added fmx_synth_config.level_spread_db,
 * which changed that struct's size: callers must be rebuilt against this
 * header. */
#define FMX_ABI_VERSION 9

enum {
  FMX_OK = 0,
  FMX_E_INVALID = -1,   /* bad argument / unsupported configuration        */
  FMX_E_HIP = -2,       /* HIP runtime failure                             */
  FMX_E_NOMEM = -3,     /* device allocation failed                        */
  FMX_E_CAPACITY = -4,  /* n exceeds the block size the handle was made for */
  FMX_E_NODEVICE = -5   /* no HIP device / kernels not loadable            */
};

/* dsp_agc (config.h:51) */
enum { FMX_AGC_OFF = 0, FMX_AGC_FAST = 1, FMX_AGC_SLOW = 2 };
/* stereo_blend (config.h:52) */
enum { FMX_BLEND_SOFT = 0, FMX_BLEND_NORMAL = 1, FMX_BLEND_AGGRESSIVE = 2 };
/* tuner.deemphasis (main.cpp:699-708) */
enum { FMX_DEEMPH_50US = 0, FMX_DEEMPH_75US = 1, FMX_DEEMPH_OFF = 2 };

typedef struct {
  int iq_rate;         /* SDR rate, integer multiple of dsp_rate             */
  int dsp_rate;        /* 240000 (2.4 MS/s / 10) or 256000 (reference)       */
  int out_rate;        /* 32000                                              */
  int block;           /* max DSP samples per call (dsp_block_samples)       */
  int w0_bandwidth_hz; /* processing.w0_bandwidth_hz                         */
  int bandwidth_hz;    /* XDR W value (0 = W0)                               */
  int dsp_agc;         /* FMX_AGC_*                                          */
  int stereo;          /* processing.stereo                                  */
  int blend;           /* FMX_BLEND_*                                        */
  int deemphasis;      /* FMX_DEEMPH_*                                       */
  int force_mono;
  int force_stereo;
  int rds;             /* decode RDS                                          */
} fmx_config;

/* One RDS group as the reference's RDSGroup (rds_decoder.h:9-15). */
typedef struct {
  uint16_t a, b, c, d;
  uint8_t errors; /* (eA<<6)|(eB<<4)|(eC<<2)|eD, e: 0 ok, 1 corrected, 3 missing */
  uint8_t pad;
  uint32_t block_index; /* fmx_process_block call that emitted it */
} fmx_rds_group;

/* RF-domain level of the raw u8 IQ of one call, as computeSignalLevel
 * (src/signal_level.cpp:145-204) + smoothSignalLevel (:206-214) of the
 * reference's per-read path (main.cpp:1166-1174). */
typedef struct {
  float level120;          /* SignalLevelResult::level120                     */
  float level120_smoothed; /* smoothSignalLevel(level120, per-channel state)  */
  double dbfs;
  double compensated_dbfs;
  double hard_clip_ratio;
  double near_clip_ratio;
} fmx_signal_level;

/* Device output buffers of fmx_process_block (all optional except where
 * noted; pass NULL to skip).  Strides are in elements. */
typedef struct {
  float *d_mpx;            /* [C][mpx_stride] discriminator MPX at dsp_rate   */
  int mpx_stride;
  float *d_pcm_l;          /* [C][pcm_stride] clamped 32 kHz audio (required) */
  float *d_pcm_r;          /* [C][pcm_stride]                                 */
  int pcm_stride;
  int *d_pcm_count;        /* [C] samples written per channel (required)      */
  int *d_stereo;           /* [C] StereoDecoder::isStereo()                   */
  int *d_pilot_tenths;     /* [C] getPilotLevelTenthsKHz()                    */
  float *d_clip_ratio;     /* [C] FMDemod::getClippingRatio()                 */
  fmx_rds_group *d_groups; /* [C][groups_stride]                              */
  int groups_stride;
  int *d_group_count;      /* [C]                                             */
  fmx_signal_level *d_signal; /* [C] RF level of this call's IQ (u8 input)    */
  int *d_stereo_indicator; /* [C] XDR stereo flag: isStereo() || (forceMono &&
                              stereo && pilot >= 2.0 kHz), main.cpp:1298-1300 */
} fmx_block_out;

/* ---- build record ----
 * "src=<16 hex> defs=<A/B defines>": the first 16 hex digits of the SHA-256
 * of the sources this library was compiled from (fmtuner-sdr_amd/Makefile
 * FMX_SRC_SHA: csrc/, include/fmx.h, include/fmx_blocks.hpp and the Makefile,
 * concatenated in sorted path order) and the variant defines (empty for the
 * shipped library).  __graft_entry__.smoke() checks it against the tree. */
const char *fmx_build_info(void);

/* ---- lifetime ---- */
int fmx_device_count(void);
int fmx_create(const fmx_config *cfg, int n_channels, int device, void **handle);
int fmx_destroy(void *handle);
const char *fmx_last_error(void *handle);
int fmx_sync(void *handle);
int fmx_num_channels(void *handle);

/* Runtime::reset fan-out (main.cpp:686-691: demod, stereo, afPost,
 * decimator) plus the RDS worker reset (main.cpp:909-916).  channel = -1
 * resets every channel. */
int fmx_reset(void *handle, int channel);
/* The retune path of main.cpp:1028-1042: the same reset fan-out, then the
 * PCM of the next mute_samples 32 kHz outputs (per channel, across calls) is
 * faded out over OUTPUT_RATE/200 samples, muted, and faded back in, as
 * main.cpp:1310-1337 does after the clamp.  mute_samples < 0 takes the
 * reference's kRetuneMuteSamples = OUTPUT_RATE/25 (main.cpp:696-697); 0
 * cancels a running mute.  At most 65535. */
int fmx_retune(void *handle, int channel, int mute_samples);

/* Per-channel settings mirroring the reference setters; channel = -1 = all. */
enum {
  FMX_PARAM_BANDWIDTH_HZ = 1,  /* FMDemod::setBandwidthHz (fm_demod.cpp:168)   */
  FMX_PARAM_W0_HZ = 2,         /* FMDemod::setW0BandwidthHz (:206)             */
  FMX_PARAM_DEEMPHASIS = 3,    /* tuner.deemphasis 0/1/2 -> both demod + AF   */
  FMX_PARAM_DSP_AGC = 4,       /* FMDemod::setDspAgcMode (:210)                */
  FMX_PARAM_BLEND = 5,         /* StereoDecoder::setBlendMode                  */
  FMX_PARAM_FORCE_MONO = 6,    /* StereoDecoder::setForceMono                  */
  FMX_PARAM_FORCE_STEREO = 7,  /* StereoDecoder::setForceStereo                */
  FMX_PARAM_BANDWIDTH_MODE = 8, /* FMDemod::setBandwidthMode (TEF table)       */
  FMX_PARAM_DEEMPH_US = 9,     /* setDeemphasis(tau_us) of FMDemod + AFPostProcessor,
                                  any tau; <= 0 switches it off (fm_demod.cpp:50-62) */
  FMX_PARAM_DEVIATION_HZ = 10  /* FMDemod::setDeviation(Hz) (fm_demod.cpp:64-71)  */
};
int fmx_set_param(void *handle, int channel, int key, int value);
/* computeSignalLevel's arguments (main.cpp:1166-1170): applied tuner gain
 * (dB), gain compensation factor (kSignalGainCompFactor 0.5, main.cpp:513),
 * config sdr.signal_bias_db / signal_floor_dbfs / signal_ceil_dbfs
 * (config.h:27-29; defaults -4 / -55 / -19).  channel = -1 = all. */
int fmx_set_signal_params(void *handle, int channel, int applied_gain_db, double gain_comp_factor,
                          double bias_db, double floor_dbfs, double ceil_dbfs);

/* One reference block for every channel.  d_iq: [C][iq_stride] bytes, each
 * row holding 2*n*M interleaved u8 I/Q (M = iq_rate / dsp_rate); n <= block.
 * Queued on the handle's stream; results are valid after fmx_sync(). */
int fmx_process_block(void *handle, const uint8_t *d_iq, size_t iq_stride, int n,
                      const fmx_block_out *out);

/* ---- per-object stages (same state as fmx_process_block) ----
 * Each mirrors one reference method, batched over all C channels. */
/* ComplexDecimator::executeComplex: d_out [C][out_stride] complex float */
int fmx_decimate(void *handle, const uint8_t *d_iq, size_t iq_stride, int n_out, float *d_out,
                 int out_stride);
/* ComplexDecimator::execute (liquid_primitives.cpp:422-459): the same
 * decimation, requantised to interleaved u8 (clamp(y*127.5 + 127.5) -> u8);
 * d_out [C][out_stride] bytes, 2 per output sample */
int fmx_decimate_u8(void *handle, const uint8_t *d_iq, size_t iq_stride, int n_out, uint8_t *d_out,
                    size_t out_stride);
/* FMDemod::processSplitComplex(iq, mpx, mono, n): d_iq_cf complex float
 * [C][in_stride]; d_mono may be NULL (stereo mode: returns 0 samples). */
int fmx_demod(void *handle, const float *d_iq_cf, int in_stride, int n, float *d_mpx, int mpx_stride,
              float *d_mono, int mono_stride, int *d_mono_count);
/* FMDemod::processSplit(iq, mpx, mono, n) on u8 IQ at dsp_rate (iq_rate ==
 * dsp_rate; byte LUT (v-127)/127.5, clip = byte 0/255, fm_demod.cpp:219-249) */
int fmx_demod_u8(void *handle, const uint8_t *d_iq, size_t iq_stride, int n, float *d_mpx, int mpx_stride,
                 float *d_mono, int mono_stride, int *d_mono_count, float *d_clip_ratio);
/* FMDemod::downsampleAudio(demod, audio, n): mono resampler + de-emphasis +
 * DC block on MPX (fm_demod.cpp:279-295) */
int fmx_downsample(void *handle, const float *d_mpx, int mpx_stride, int n, float *d_out, int out_stride,
                   int *d_count);
/* StereoDecoder::processAudio */
int fmx_stereo(void *handle, const float *d_mpx, int mpx_stride, int n, float *d_left, float *d_right,
               int lr_stride, int *d_stereo, int *d_pilot_tenths);
/* AFPostProcessor::process (outCapacity = cap) */
int fmx_afpost(void *handle, const float *d_left, const float *d_right, int in_stride, int n,
               float *d_out_l, float *d_out_r, int out_stride, int cap, int *d_count);
/* RDSDecoder::process: groups of this call per channel */
int fmx_rds(void *handle, const float *d_mpx, int mpx_stride, int n, fmx_rds_group *d_groups,
            int groups_stride, int *d_group_count);

/* ---- device memory helpers (so C/FFI callers need no HIP headers) ---- */
int fmx_malloc(void *handle, void **d_ptr, size_t bytes);
int fmx_free(void *handle, void *d_ptr);
int fmx_memcpy_h2d(void *handle, void *d_dst, const void *h_src, size_t bytes);
int fmx_memcpy_d2h(void *handle, void *h_dst, const void *d_src, size_t bytes);
int fmx_memset(void *handle, void *d_ptr, int value, size_t bytes);

/* ---- HIP-event timing of the hot kernels (bench roofline support) ----
 * When enabled, every launch of each kernel is bracketed by events on the
 * stream it runs on; fmx_kernel_times returns the summed milliseconds and
 * launch counts per kernel id since the last reset. */
enum {
  FMX_K_FRONTEND = 0, /* decimate + DC + IQ FIR + AGC + discriminator (+ pilot BPF, + RDS
                         resample when process_block does not run them as kernels of their own) */
  FMX_K_STEREO = 1,   /* pilot PLL + blend + L-R matrix (one lane per channel)                 */
  FMX_K_AUDIO = 2,    /* L/R 15 kHz FIRs + 32 kHz resampler + de-emphasis + DC + clamp         */
  FMX_K_RDS = 3,      /* 57 kHz BPSK demod + symsync (+ biphase + block sync in fmx_rds)        */
  FMX_K_RS = 4,       /* the 240k -> 171k RDS resampler when process_block runs it as its own
                         kernel (k_rs, on the RDS stream ahead of k_rds)                        */
  FMX_K_PILOT = 5,    /* the 19 kHz pilot BPF when process_block runs it as its own kernel
                         (k_pilot, on the front-end stream after k_fe8)                         */
  FMX_K_FRONTEND_GENERIC = 6, /* process_block's front end when it runs as the generic k_frontend
                         (calls of n < 1024 samples, unaligned IQ rows) instead of k_fe8;
                         FMX_K_FRONTEND then counts k_fe8 launches only                           */
  FMX_K_BITS = 7,     /* process_block's RDS bit decoders (biphase, delta, block sync, groups:
                         k_bits, on the audio stream ahead of k_audio)                          */
  FMX_K_COUNT = 8
};
/* enable: 0 off, 1 every step's launches, N > 1 the launches of every N-th
 * step only (a sample: fewer event packets on the streams in the timed region) */
int fmx_timing_enable(void *handle, int enable);
/* diagnostic: frontend per-stage clocks, 8 values (diagnostics library
 * libfmx_diag.so, handle created with FMX_STAMPS=1 in the environment;
 * FMX_E_INVALID otherwise -- the product libfmx.so reads no environment) */
int fmx_debug_stamps(void *handle, unsigned long long *out, int n);
int fmx_kernel_times(void *handle, double *ms, int *launches, int n);
/* host-side waits of fmx_process_block since the last call (then reset):
 * out[0] waits on a pinned schedule image's last reader, out[1] those that
 * found it still pending (the host blocked), out[2] milliseconds blocked.
 * Fills at most n (<= 3) entries. */
int fmx_host_stats(void *handle, double *out, int n);
/* diagnostics (round 6).  A call of >= 256 RDS-rate samples leaves the RDS
 * FIR's 256-sample ring (the mixed samples a reset's decimation-phase
 * rebuild reads) to per-round NCO checkpoints instead of writing it; it is
 * refilled, bit-identically, when needed.  fmx_diag_set(FMX_DIAG_RDS_RING_ALWAYS,
 * 1) makes k_rds write it every call (round 5's behaviour; the test arm);
 * fmx_diag_rds_ring copies the channel's ring, oldest sample first, as 256
 * (re, im) float pairs to host memory (synchronous; refills it first). */
enum { FMX_DIAG_RDS_RING_ALWAYS = 1 };
int fmx_diag_set(void *handle, int what, int value);
int fmx_diag_rds_ring(void *handle, int channel, float *out);

/* ---- synthetic IQ (bench / tests input; see fmx_synth.h) ---- */
typedef struct {
  int iq_rate;
  int kind;        /* 0 mono two-tone, 1 stereo, 2 stereo + RDS             */
  float amplitude; /* 0.8                                                   */
  float noise_std; /* AWGN per component (0 = none)                         */
  uint32_t seed_base;
  int max_offset_hz;
  float rds_level; /* 0.05                                                  */
  int n_bits;      /* RDS bit-table length per channel                      */
  float level_spread_db; /* per-channel carrier level: amplitude * 10^(-u d / 20),
                            u in (0, 1] from the channel seed, d this value
                            (0 = every channel at `amplitude`)              */
} fmx_synth_config;
/* RDS test pattern: encoded (differential) bits [n_ch][n_bits] and, if
 * h_groups != NULL, the transmitted groups [n_ch][n_bits/104][4]. */
int fmx_synth_rds_bits(const fmx_synth_config *cfg, uint32_t ch0, int n_ch, uint8_t *h_bits,
                       uint16_t *h_groups);
/* host generation: h_out [n_ch][2*n_samples]; h_bits [n_ch][n_bits] or NULL */
int fmx_synth_host(const fmx_synth_config *cfg, uint32_t ch0, int n_ch, int64_t sample0, int n_samples,
                   const uint8_t *h_bits, uint8_t *h_out, size_t out_stride, int threads);
/* device generation on the handle's stream: d_out [n_ch][out_stride] */
int fmx_synth_device(void *handle, const fmx_synth_config *cfg, uint32_t ch0, int n_ch, int64_t sample0,
                     int n_samples, const uint8_t *d_bits, uint8_t *d_out, size_t out_stride);

/* ---- diagnostics (host only, no GPU needed) ---- */
/* Filter taps the handle would use: which = 0 decimator, 1 IQ FIR,
 * 2 pilot BPF, 3 L/R LPF, 4 audio resampler prototype, 5 RDS resampler
 * prototype, 6 RDS 2.4 kHz LPF, 7 symsync RRC, 8 symsync derivative;
 * the MFMA tables read back as float taps:
 * 10 pilot BPF fragments, 11 IQ FIR fragments, 12 L/R LPF fragments (k_audio),
 * 13 decimator A fragments (row 0), 9 the same fragments' rows 0..15.
 * Returns the tap count (negative on error). */
int fmx_design_taps(const fmx_config *cfg, int which, float *out, int cap);
/* liquid resamp_rrrf output schedule for rate 1/del over n_in inputs from
 * the reset state: packed = i | (branch << 16) | (boundary << 24). */
int fmx_resamp_schedule(float del, int n_in, int *packed, float *mu, int cap);

/* ---- host-side consumers of the GPU outputs ----
 * The reference's wire and file formats, fed from fmx_process_block's
 * outputs (copied to the host).  No GPU needed. */
/* Per-channel PI debounce state of the XDR server (xdr_server.h:151-156). */
typedef struct {
  uint16_t pi_buf[64];
  uint8_t pi_err[8];
  uint8_t fill, pos, last_state, pad;
  uint16_t last_value, pad2;
} fmx_xdr_pi_state;
/* XDRServer ctor / setFrequencyState reset (xdr_server.cpp:261-266, 465-470). */
void fmx_xdr_pi_reset(fmx_xdr_pi_state *s);
/* XDRServer::updateRDS for n groups of one channel (xdr_server.cpp:189-213,
 * 403-457): writes the queued lines ("P%04X" + '?' per block-A error level,
 * "R%04X%04X%04X%02X"), each ending in '\n', NUL-terminated.  Returns the bytes
 * written, or -(bytes needed + 1) when cap is too small (then nothing is
 * written and the state is unchanged). */
int fmx_xdr_rds_lines(fmx_xdr_pi_state *s, const fmx_rds_group *groups, int n, char *out, int cap);
/* Scan line of main.cpp:1069-1113 as XDRServer::pushScanLine queues it
 * ("U" + "f=level,..." with level = (float)(level_sum / reads) at one
 * decimal; points with reads == 0 skipped; empty when no point).  level_sum
 * holds summed fmx_signal_level.level120 values.  Same return convention. */
int fmx_xdr_scan_line(const int *freq_khz, const double *level_sum, const int *reads, int n, char *out, int cap);
/* AudioOutput::writeWAVHeader (audio_output.cpp:1346-1377): 44 bytes for
 * data_bytes of S16LE 32 kHz stereo.  Returns 44. */
int fmx_wav_header(uint32_t data_bytes, uint8_t *out44);
/* AudioOutput::write volume ramp (:1432-1467) + writeWAVData (:1379-1398):
 * n stereo frames -> 2n interleaved int16; *volume_scale carries the sink's
 * m_currentVolumeScale (initially 0.85).  Returns n. */
int fmx_pcm_to_s16(const float *left, const float *right, int n, int volume_percent, float *volume_scale,
                   int16_t *out);
/* writeIqCapture (main.cpp:742-747): n raw I/Q byte pairs to path
 * (append != 0 appends).  fmx_iq_replay reads n pairs at a sample offset
 * back (returns the pairs read). */
int fmx_iq_capture(const char *path, const uint8_t *iq, int n_samples, int append);
int fmx_iq_replay(const char *path, long long sample_offset, int n_samples, uint8_t *out);

#ifdef __cplusplus
}
#endif
#endif

// fmx_internal.h -- host-side internals of libfmx (not part of the ABI).
#ifndef FMX_INTERNAL_H
#define FMX_INTERNAL_H

#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/fmx.h"
#include "fmx_design.h"

namespace fmx {

// ---- design (fmx_design.cpp) ----
struct DesignExtras {
  std::vector<float> proto_af, proto_rds, rrc, rrc_d;
};
void firdes_kaiser(unsigned n, float fc, float As, float mu, float *h);
uint32_t nco_constrain(float theta);
int design_build(const fmx_config &cfg, FmxDesign *d, DesignExtras *ex, std::string *err);
int bandwidth_select(int bw_hz, int w0);
int tef_bandwidth_hz(int mode);

// liquid resamp_rrrf timing state (float tau, interp/boundary), simulated on
// the host because it does not depend on the signal.
struct ResampTiming {
  float tau = 0.0f, bf = 0.0f, mu = 0.0f, del = 1.0f;
  int b = 0, state = 0;
};
void timing_reset(ResampTiming &t);
int timing_run(ResampTiming &t, int n_in, FmxSched *out, int cap);
bool timing_equal(const ResampTiming &a, const ResampTiming &b);

// ---- kernel argument blocks (fmx_kernels.hip) ----
enum FeInMode { FE_IN_U8_DECIM = 0, FE_IN_CF = 1, FE_IN_U8_DIRECT = 2, FE_IN_MPX = 3 };

// process_block runs the 19 kHz pilot BPF of a k_fe8 step as its own kernel
// (k_pilot, after k_fe8 on the front-end stream); k_fe8 then writes only the
// MPX and its history rows (FeArgs::st_hist_out)
struct FeArgs {
  const FmxDesign *des;
  int des_fs;        // DSP rate (host copy of des->fs, for the launcher)
  const FmxChanParam *par;
  int C, n, in_mode;
  // inputs
  const uint8_t *iq;
  size_t iq_stride;
  const float *in_f; // complex (FE_IN_CF) or mpx (FE_IN_MPX)
  int in_stride;
  // outputs
  float *bb_out;     // complex decimator output (fmx_decimate), may be null
  int bb_stride;
  float *mpx_out;
  int mpx_stride;
  float *pilot_out;  // null = no pilot BPF
  int pilot_stride;
  int st_hist_out;   // write the stereo history rows (st_hist_wr) even without the pilot BPF
  float *rds_out;    // null = no RDS resampling
  int rds_stride;
  int *rds_count;    // [C]
  float *clip_out;   // [C]
  unsigned long long *sig_sums; // [C][6] RF-level byte sums (u8 inputs; k_audio evaluates them), may be null
  unsigned long long *dbg;    // [8] stage clocks (diagnostics build, FMX_STAMPS), may be null
  // stages
  int do_demod;      // run DC + IQ FIR + AGC + discriminator
  // state
  uint8_t *dec_hist;
  int *dec_valid;
  float *dc_v;       // [C][2]
  float2_t *iq_hist; // [C][FMX_IQ_MAXLEN-1]
  float *agc;        // [C][2]
  float *fd_prev;    // [C][2]
  const float *st_hist_rd; // [C][FMX_HIST] stereo MPX history before this call
  float *st_hist_wr;       // [C][FMX_HIST] history after this call (another buffer)
  float *rds_hist;   // [C][32]
  // schedules
  const FmxSched *rds_sched; // [groups][rds_sched_stride]
  const int *rds_sched_n;    // [groups]
  const int *rds_group;      // [C]
  int rds_sched_stride;
  // k_fe8 leaves the RDS resampler to k_rs: it writes the previous call's
  // last 32 MPX samples here ([C][32]) instead of resampling (may be null)
  float *rds_win_out;
  // the NEXT step's RDS schedule slot, copied by the first workgroups of this
  // launch from the mapped pinned image (fmx_capi.cpp process_block): no copy
  // kernel on the front end's stream between two front ends; n16 = 0: none
  const void *next_sched_src;
  void *next_sched_dst;
  unsigned next_sched_n16;
};

struct PllArgs {
  const FmxDesign *des;
  const FmxChanParam *par;
  int C, n;
  const float *pilot;
  int pilot_stride;
  const float *mpx;
  int mpx_stride;
  const float *st_hist_rd; // [C][FMX_HIST] history the frontend of this call read
  float *lraw, *rraw;
  int lr_stride;
  int lr_tiled;            // raw L/R in pair tiles (lr_tile_idx, fmx_kernels.hip), else [C][lr_stride]
  FmxStereoState *st;
  int *stereo_out, *pilot_tenths_out;
  int *indicator_out;      // [C] XDR stereo indicator (main.cpp:1298-1300), may be null
  unsigned long long *dbg; // [16] per-wave work / barrier clocks (diagnostic, FMX_STAMPS=1), may be null
  int n_cu;                // CUs of the handle's device (launch_pll's workgroup shape)
};

struct AudioArgs {
  const FmxDesign *des;
  const FmxChanParam *par;
  int C, n, mode; // mode 0 stereo (LR FIR + AF), 1 AF only, 2 mono (FMDemod), 3 mono pipeline
  int cap;
  const float *in_l, *in_r;
  int in_stride;
  int in_tiled;    // in_l / in_r in pair tiles (raw L/R from k_pll), else [C][in_stride]
  float *out_l, *out_r;
  int out_stride;
  int *out_count;
  float *lr_hist;  // [C][2][FMX_LR_LEN-1]
  float *af_win;   // [C][2][32]
  float *af_iir;   // [C][4]
  float *mono_win; // [C][32]
  float *mono_iir; // [C][2]
  float *lr_out_l, *lr_out_r; // optional filtered L/R at dsp rate (fmx_stereo)
  int lr_out_stride;
  const FmxSched *sched; // [groups][sched_stride]
  const int *sched_n;
  const int *group; // [C]
  int sched_stride;
  int clamp;
  int *mute;       // [C][2] retune fade/mute {remaining, total} (main.cpp:1310-1337), may be null
  int mute_fade;   // OUTPUT_RATE / 200
  // RF level of the step (computeSignalLevel / smoothSignalLevel) from the
  // front end's byte sums, when sig_out is set
  fmx_signal_level *sig_out;          // [C]
  const unsigned long long *sig_sums; // [C][6]
  long sig_samples;                   // IQ samples behind the sums
  const double *sig_par;              // [C][4] gain*factor, bias, floor, ceil
  float *sig_smooth;                  // [C][2] smoother value, initialized flag
};

struct RdsArgs {
  const FmxDesign *des;
  int C;
  const float *in; // 171 kHz samples
  int in_stride;
  const int *in_count; // [C]
  FmxRdsState *st;
  float *ring; // [C][FMX_RDS_RING][2]
  // the previous RDS call's input rows (its slot; same stride), for the ring
  // refill of a short call after a long one (FmxRdsState::ring_ok)
  const float *in_prev;
  int ring_always; // write the ring every call (FMX_RDS_RING_ALWAYS=1: the round-5 behaviour, the A/B and test arm)
  fmx_rds_group *groups;
  int groups_stride;
  int *group_count;
  uint32_t block_index;
  unsigned long long *dbg; // [8] stage clocks (diagnostic, FMX_STAMPS=1), may be null
  // the call's PSK2 symbols, k_rds -> k_bits (the bit decoders)
  float *sym;         // [C][sym_stride] real parts
  int sym_stride;
  int *sym_count;     // [C]
  float *sym_last_im; // [C] the last symbol's imaginary part (BiphaseDecoder's prev)
  // fused (round 6, FMX_RDS_FUSED A/B builds only -- measured slower and not
  // shipped: +20 % step at 4096 channels, +61 % at 2048, profiles/r06l_*):
  // k_rds resamples the MPX to 171 kHz itself
  // (k_rs's MFMA tiles, produced as the rounds need them) instead of reading
  // `in`; as RsArgs
  int fused;
  int n;                  // MPX samples of the call
  const float *mpx;
  int mpx_stride;
  const float *win;       // [C][32] the previous call's last 32 MPX samples
  const FmxSched *sched;  // [groups][sched_stride]
  const int *sched_n;     // [groups]
  const int *group;       // [C]
  int sched_stride;
};

// k_pilot: the 19 kHz pilot BPF of a process_block step (after k_fe8)
struct PilotArgs {
  const FmxDesign *des;
  int des_pilot_len;        // host copy of des->pilot_len (launcher check)
  int C, n;
  const float *mpx;         // this step's MPX rows (the front end's output)
  int mpx_stride;
  const float *st_hist_rd;  // [C][FMX_HIST] the previous call's last MPX samples
  float *out;               // pilot rows (k_pll's input)
  int out_stride;
  int vec;                  // set by the launcher: 16-B rows
};

// k_rs: the 240k -> 171k RDS resampler of a process_block step (liquid
// resamp_rrrf, host timing schedule), 16 channels per workgroup on FP32 MFMA
struct RsArgs {
  const FmxDesign *des;
  int C, n;
  const float *mpx;     // this step's MPX rows (the front end's output)
  int mpx_stride;
  const float *win;     // [C][32] the previous call's last 32 MPX samples
  const FmxSched *sched; // [groups][sched_stride]
  const int *sched_n;   // [groups]
  const int *group;     // [C]
  int sched_stride;
  float *out;           // RDS-rate rows
  int out_stride;
  int parts;            // workgroups per 16 channels (each a contiguous run of output tiles)
};

// launchers (fmx_kernels.hip); stream is a hipStream_t
// vec: the caller guarantees every channel's decimator history is full
// (dec_valid == L-1) -- only k_frontend's VEC form needs it; k_fe8 takes cold
// and warm channels alike; 16-B row alignment is checked here.
// Events bound to the NEXT main-kernel launch of this thread (k_fe8 /
// k_frontend, k_pll, k_audio, k_rs, k_rds) through hipExtLaunchKernel: `stop`
// completes with the kernel and `start` (timing) takes its start time -- no
// marker packets between two kernels of a stream.  Consumed by that launch.
void set_launch_events(void *start, void *stop);
int launch_frontend_m(const FeArgs &a, int M, int tpp, void *stream, bool vec = false);
// whether launch_frontend_m would run k_fe8 for these arguments
bool frontend_is_fe8(const FeArgs &a, int M, int tpp);
int launch_pll(const PllArgs &a, void *stream);
int launch_pilot(const PilotArgs &a, void *stream);
int launch_audio(const AudioArgs &a, void *stream);
int launch_rds(const RdsArgs &a, void *stream);      // k_rds then k_bits (one timer over both)
struct ResetArgs;
int launch_rds_sym(const RdsArgs &a, void *stream);  // k_rds alone: the call's symbols
int launch_ring_fill(const ResetArgs &a, void *stream); // every channel's RDS ring refilled where ring_ok = 0
int launch_bits(const RdsArgs &a, void *stream);     // k_bits alone: the bit decoders
#ifndef FMX_RDS_FUSED
#define FMX_RDS_FUSED 0 // A/B: the RDS resampler inside k_rds (RdsArgs::fused)
#endif
#ifndef FMX_RS_TMAX
#define FMX_RS_TMAX 12 // k_rs: output tiles (of 16) per workgroup at most from 2048 channels (46 from 4096 on, 6 below 2048: fmx_capi.cpp)
#endif
int launch_rs(const RsArgs &a, void *stream);
int launch_synth(const fmx_synth_config &cfg, uint32_t ch0, int n_ch, int64_t sample0, int n_samples,
                 const uint8_t *bits, uint8_t *out, size_t out_stride, void *stream);
struct ResetArgs {
  const FmxDesign *des;
  int C;
  const int *mask; // [C] bitmask of parts to reset
  FmxStereoState *st;
  FmxRdsState *rds;
  float *ring;
  uint8_t *dec_hist;
  int *dec_valid;
  float *dc_v;
  float2_t *iq_hist;
  float *agc;
  float *fd_prev;
  float *st_hist; // [FMX_ST_BUFS][C][FMX_HIST]
  float *lr_hist, *af_win, *af_iir, *mono_win, *mono_iir;
  float *rds_hist;
  int *mute;      // [C][2]
  const float *rds_prev; // the last RDS call's input rows (the ring refill before a rebuild)
  int rds_stride;
};
// per-step intermediates (MPX, pilot, RDS-rate, raw L/R): front end k runs
// while stereo/RDS/audio of steps k-1, k-2 drain
#ifndef FMX_NBUF
#define FMX_NBUF 3
#endif
#define FMX_ST_BUFS (FMX_NBUF + 1) // rotating stereo-history buffers
enum ResetParts {
  RS_DECIM = 1,    // ComplexDecimator::reset
  RS_DEMOD = 2,    // FMDemod::reset (DC, IQ FIR, discriminator, mono chain)
  RS_AGC = 4,      // AGC re-init (FMDemod::reset when ready, setDspAgcMode)
  RS_STEREO = 8,   // StereoDecoder::reset
  RS_AF = 16,      // AFPostProcessor::reset
  RS_RDS = 32,     // RDSDecoder::reset (symsync + NCO + block stream)
  RS_IQFIR = 64,   // IQ FIR re-created (setBandwidthHz)
  RS_DEEMPH = 128, // de-emphasis IIRs re-created (setDeemphasis)
  RS_CREATE = 256, // object construction (everything, incl. RDS resampler/AGC)
  RS_MUTE = 512,   // retune fade/mute start; mute length in bits 16..31 (main.cpp:1034-1035)
  RS_FREQDEM = 1024 // discriminator re-created (FMDemod::setDeviation)
};
// the stream-local parts of a channel reset (reset_channel, fmx_kernels.hip):
// each part's state is read / written by the kernels of one process_block
// stream only
enum ResetStreamPart {
  RSP_FRONT = 1,  // sA: decimator / IQ FIR / DC / AGC / discriminator state, stereo history rows
  RSP_STEREO = 2, // sB: FmxStereoState (k_pll)
  RSP_RDS = 4,    // sC: FmxRdsState up to the bit decoders, mix-down ring (k_rds)
  RSP_AUDIO = 8,  // sD: L/R FIR history, AF / mono resampler + IIRs, retune mute (k_audio)
  RSP_BITS = 16,  // sD: FmxRdsState's bit decoders, bi_prev_re on (k_bits)
  RSP_ALL = 31
};
#define FMX_RESET_LIST 64 // channels per k_reset_list launch (a kernel argument, no upload)
struct ResetList {
  int n;
  int ch[FMX_RESET_LIST];
  int m[FMX_RESET_LIST];
};
int launch_reset(const ResetArgs &a, void *stream);
int launch_reset_list(const ResetArgs &a, const ResetList &L, int parts, int st_buf, void *stream);
int launch_iq_to_u8(const float *in, int in_stride, int C, int n, uint8_t *out, size_t out_stride, void *stream);
int launch_copy16(const void *src, void *dst, size_t n16, void *stream); // 16-B words, any memory the device maps

} // namespace fmx

#endif

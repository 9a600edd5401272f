// fmx_design.h -- filter designs, per-channel parameters and per-channel state
// layout of the MI355X FM demodulator (shared by host code and HIP kernels).
//
// Every constant here is what one reference object computes in its
// constructor / setter; the host computes them once per handle
// (fmx_design.cpp) and uploads them to HBM, where all channels share them.
#ifndef FMX_DESIGN_H
#define FMX_DESIGN_H

#include <stdint.h>

#define FMX_MAX_DEC 512      // M * taps_per_phase (liquid_primitives.cpp:388)
#define FMX_DEC_PAD 32       // zero taps each side of dec_pad (>= 3*M)
#define FMX_IQ_DESIGNS 31    // 30 XDR bandwidth filters + the FMDemod ctor filter
#define FMX_IQ_CTOR 30       // index of the ctor filter (fm_demod.cpp:103-105)
#define FMX_IQ_MAXLEN 121
#define FMX_PILOT_MAX 511    // stereo_decoder.cpp:98 clamp
#define FMX_LR_LEN 121       // stereo_decoder.cpp:110-111
#define FMX_LR_KS 5          // K steps of k_audio's MFMA L/R FIR: (121 + 15 + 31) / 32
#define FMX_NPFB 32          // resamp_rrrf / symsync filter-bank size
#define FMX_AF_SUB 24        // 2*m, m = 12 (liquid_primitives.h:145)
#define FMX_RDS_RS_SUB 26    // 2*m, m = 13 (subcarrier.cpp:45)
#define FMX_RDS_FIR 255      // subcarrier.cpp:101
#define FMX_RDS_DECIM 24     // subcarrier.hh:205-206
#define FMX_RDS_NACC 11      // ceil(255 / 24) streaming partial sums
#define FMX_SS_SUB 18        // (2*32*3*3+1 - 1) / 32
#define FMX_HIST 512         // stereo MPX history (>= pilot taps - 1 and delay line)
#define FMX_RDS_RING 256     // last mixed RDS samples kept for a decimation-phase rebuild
#define FMX_RDS_CK 12        // k_rds's per-round NCO checkpoints (24 (CK - 1) + 1 >= RING samples)
#define FMX_PAD 10           // zero taps around padded FIR tap arrays (5 each side)
#define FMX_DEC_KS_MAX 16    // K steps of the f16 MFMA decimator: ceil((15 M + L + 1) / 32)
#define FMX_DEC_QN (15 * 10 + 32 * FMX_DEC_KS_MAX) // entries of the flat decimator tap window (M <= 10)
#define FMX_PILOT_KS_MAX 17  // K steps of the MFMA pilot BPF for up to FMX_PILOT_MAX taps
#define FMX_IQ_KS_MAX 5      // K steps of the MFMA IQ FIR for up to FMX_IQ_MAXLEN taps
#define FMX_PILOT_QN (32 * FMX_PILOT_KS_MAX + 16) // entries of the flat pilot tap window
#define FMX_IQ_QN (32 * FMX_IQ_KS_MAX + 16)       // entries of a flat IQ FIR tap window
#define FMX_LR_QN (32 * FMX_LR_KS + 16)           // entries of the flat L/R FIR tap window

typedef struct {
  float x, y;
} float2_t;

typedef struct {
  // rates / geometry
  int M, fs, out_rate, block;
  // ComplexDecimator (liquid_primitives.cpp:370-403): taps already multiplied
  // by the u8 normalisation 1/127.5, plus the firdecim scale 2*fc.
  int dec_len, dec_tpp;
  float dec_scale;
  // 127.5 * sum(dec_taps): the u8 decimators run the FIR on the raw bytes
  // and subtract this once per output (instead of 127.5 from every sample)
  float dec_dc;
  float dec_taps[FMX_MAX_DEC];
  float dec_taps_raw[FMX_MAX_DEC];
  float dec_poly[FMX_MAX_DEC]; // [p][q] = dec_taps[q*M + p]  (phase-major)
  float dec_pad[FMX_MAX_DEC + 2 * FMX_DEC_PAD]; // [FMX_DEC_PAD + k] = dec_taps[k], zeros around
  // k_fe8's MFMA decimator (16 outputs x 16 blocks per v_mfma_f32_16x16x32_f16):
  // q[d] = dec_taps[L - d] * 2^16 for d in [1, L] (0 elsewhere) as f16 hi + lo
  // (22 significant bits), laid out as the per-lane A fragments
  //   dec_frag[ks][s][l][j] = q[32 ks + 8 (l >> 4) + j - M (l & 15)]
  // y = (acc - dec_dc16) * dec_scale16, dec_dc16 = -2^16 sum(taps) / 2 (the
  // 127.5 centre of the bytes entering as b - 128), dec_scale16 = dec_scale 2^-16
  uint16_t dec_frag[FMX_DEC_KS_MAX][2][64][8] __attribute__((aligned(16)));
  // the same q as one flat window (round 6): dec_q16[s][i] = q[i - 15 M] (hi,
  // lo), so that lane l's fragment at K step ks is the 8 entries from
  // 32 ks + 8 (l >> 4) + 15 M - M (l & 15) on; process_block's k_fe8 copies
  // the window (1.2 KB at M = 10) into LDS once per workgroup and reads its
  // fragments there instead of dec_frag's 2 KB per K step from L2
  uint16_t dec_q16[2][FMX_DEC_QN] __attribute__((aligned(16)));
  float dec_dc16, dec_scale16;
  // FMDemod IQ FIR designs (fm_demod.cpp:168-204) and discriminator gain
  int iq_len[FMX_IQ_DESIGNS];
  float iq_scale[FMX_IQ_DESIGNS];
  float iq_taps[FMX_IQ_DESIGNS][FMX_IQ_MAXLEN];
  float iq_pad[FMX_IQ_DESIGNS][FMX_IQ_MAXLEN + FMX_PAD]; // [k + 5] = taps[k], zeros around
  float iq_z16[FMX_IQ_DESIGNS][FMX_IQ_MAXLEN + 32]; // [k + 16] = taps[k], 16 zeros each side (k_fe8)
  // k_fe8's MFMA IQ FIR, fragments as pilot_frag (below) per design: taps *
  // 2^12 as f16 hi + lo, iq_ks[i] = ceil((P8 + 15) / 32) K steps
  int iq_ks[FMX_IQ_DESIGNS];
  uint16_t iq_frag[FMX_IQ_DESIGNS][FMX_IQ_KS_MAX][2][64][8] __attribute__((aligned(16)));
  // the same per design as a flat window for process_block's k_fe8 (round 6),
  // laid out as pilot_q16: iq_q16[i][c][s][e] = q[e + c - 15]
  uint16_t iq_q16[FMX_IQ_DESIGNS][2][2][FMX_IQ_QN] __attribute__((aligned(16)));
  float fd_ref;          // 1 / (2 pi kf), kf = 75 kHz / Fs
  float deemph_alpha[2]; // 50 us, 75 us at out_rate (fm_demod.cpp:119-131)
  // StereoDecoder (stereo_decoder.cpp:25-63)
  int pilot_len, delay_len; // delay_len = delaySamples + 1 (ring size)
  float pilot_taps[FMX_PILOT_MAX];
  float pilot_pad[FMX_PILOT_MAX + FMX_PAD];
  float pilot_z16[FMX_PILOT_MAX + 32]; // [k + 16] = taps[k], 16 zeros each side (k_fe8)
  float pilot_pair[FMX_PILOT_MAX + FMX_PAD][2] __attribute__((aligned(8))); // {pad[k], pad[k+1]}: packed-FMA tap pairs
  // k_fe8's MFMA pilot BPF (16 outputs x 16 blocks per v_mfma_f32_16x16x32_f16):
  // lane l's A fragment of K step ks, split s (hi, lo of tap * 2^12):
  // pilot_frag[ks][s][l][j] = q[32 ks + 8 (l >> 4) + j - (l & 15)], q[d] =
  // h[P8 - 1 - d] (P8 = fir8 length, 8k + 1, leading zero taps)
  int pilot_ks; // K steps: ceil((P8 + 15) / 32)
  uint16_t pilot_frag[FMX_PILOT_KS_MAX][2][64][8] __attribute__((aligned(16)));
  // the same q as a flat window for k_pilot's LDS (round 6): pilot_q16[c][s][i]
  // = q[i + c - 15] (copy c = 1 shifted by one entry, so that every lane's 8
  // entries, from 32 ks + 8 (l >> 4) + 15 - (l & 15), start on a dword)
  uint16_t pilot_q16[2][2][FMX_PILOT_QN] __attribute__((aligned(16)));
  float lr_scale;
  float lr_taps[FMX_LR_LEN];
  // k_audio's MFMA L/R FIR fragments, as pilot_frag: taps * 2^12 as f16 hi +
  // lo, lr_frag[ks][s][l][j] = q[32 ks + 8 (l >> 4) + j - (l & 15)]
  uint16_t lr_frag[FMX_LR_KS][2][64][8] __attribute__((aligned(16)));
  // the same q as a flat window for k_audio's LDS (round 6), as pilot_q16:
  // lr_q16[c][s][e] = q[e + c - 15]
  uint16_t lr_q16[2][2][FMX_LR_QN] __attribute__((aligned(16)));
  float lr_pad[FMX_LR_LEN + FMX_PAD];
  float lr_pair[FMX_LR_LEN + FMX_PAD][2] __attribute__((aligned(8)));
  float nominal, pll_min, pll_max, pll_alpha, pll_beta;
  uint32_t pll_dtheta0;
  float blend_attack[3], blend_release[3], gate[3];
  // resamplers: branch-major taps h[b][n] = proto[b + n*32]
  float af_h[FMX_NPFB * FMX_AF_SUB];
  float rds_rs_h[FMX_NPFB * FMX_RDS_RS_SUB];
  float af_del, rds_del;
  // RDS subcarrier (subcarrier.cpp:94-106, liquid_wrappers.cpp)
  float rds_fir[FMX_RDS_NACC * FMX_RDS_DECIM]; // 255 taps + zeros to 264 (k_rds reads rows jp + 24 i)
  float rds_fir_scale;
  // k_rds tap rows for the wave-uniform decimation phase jp: row jp holds
  // h[jp + 24 i], i = 0..10, and a zero (48-B rows, read into SGPRs)
  float rds_rows[FMX_RDS_DECIM][12] __attribute__((aligned(16)));
  float agc_bw, agc_g0;
  uint32_t rds_dtheta0;
  float rds_alpha, rds_beta;
  float ss_mf[FMX_NPFB * FMX_SS_SUB];  // [b][n] = h[b + n*32]
  float ss_dmf[FMX_NPFB * FMX_SS_SUB];
  float ss_b0, ss_a1, ss_a2; // loop filter (normalised by a0; b1 = b2 = 0)
  float ss_rate_adj;
  float psk_xr1, psk_xi1; // cexpjf(pi) of the PSK2 modem
} FmxDesign;

// Per-channel settable parameters (reference setters), uploaded on change.
typedef struct {
  int iqsel;       // index into iq_* designs
  int agc;         // 0 off, 1 fast, 2 slow
  int blend;       // 0 soft, 1 normal, 2 aggressive
  int force_mono;
  int force_stereo;
  int deemph;      // 0 -> 50us, 1 -> 75us, 2 -> off, 3 -> deemph_alpha (setDeemphasis(tau_us))
  float deemph_alpha; // dt / (tau + dt) of a custom tau (fm_demod.cpp:50-62, af_post_processor.cpp:31-45)
  float fd_ref;       // 1 / (2 pi kf) of a custom deviation (fm_demod.cpp:64-71); 0 = the design's 75 kHz
} FmxChanParam;

// StereoDecoder scalars (stereo_decoder.h:27-50)
typedef struct {
  uint32_t theta, dtheta; // liquid NCO (fixed point)
  float pilot_band_mag, mpx_mag, pilot_i, pilot_q, pilot_magnitude, blend;
  float pll_freq, pll_phase;
  int pilot_count, loss_count, detected, level;
} FmxStereoState;

// RDS per-channel state (SubcarrierSet + BlockStream), one lane per channel.
typedef struct {
  // NCO + quad-phase wrapper (liquid_wrappers.cpp:271-312), stream 0
  uint32_t theta, dtheta;
  float prev_f0, phase0;
  uint32_t sample_since_reset;
  uint32_t ring_pos;       // total mixed samples written to the ring
  int rebuild;             // decimation phase changed by a reset
  // streaming FIR partial sums for the next 11 decimation instants
  float acc_re[FMX_RDS_NACC], acc_im[FMX_RDS_NACC];
  // AGC (agc_crcf)
  float agc_g, agc_y2p;
  // symsync
  float ss_win_re[FMX_SS_SUB], ss_win_im[FMX_SS_SUB];
  int ss_mf_valid;         // pushes since the matched-filter bank was reset
  float ss_rate, ss_del, ss_tau, ss_q_hat, ss_v1, ss_v2;
  int ss_b, ss_decim;
  // round 6: the ring as checkpoints.  A call of >= FMX_RDS_RING samples
  // writes no ring; it records the NCO words its last FMX_RDS_CK rounds
  // mixed with (round r: sample t = base_r + j mixed at ck_thp + j ck_dth)
  // and its o0 / rounds / count, and ring_ok = 0.  Whoever needs the ring
  // (a reset's rebuild, a short call after a long one, fmx_diag_rds_ring)
  // refills it from those words and the call's RDS-rate input, which stays
  // in its intermediate slot until the next RDS call after it
  // (rds_ring_fill: the same mix, bit-identical).  ring_ok = 1: the ring
  // holds the last FMX_RDS_RING mixed samples
  uint32_t ck_thp[FMX_RDS_CK], ck_dth[FMX_RDS_CK];
  int ck_o0, ck_rounds, ck_count, ring_ok;
  // biphase / delta decoders
  float bi_prev_re, bi_prev_im, bi_even, bi_odd;
  uint32_t bi_clock, bi_polarity;
  int delta_prev;
  // BlockStream
  uint32_t bs_bitcount, bs_until_next, bs_reg, bs_err_mask_lo, bs_err_mask_hi;
  int bs_expected, bs_in_sync, bs_err_ptr;
  uint32_t bs_pulse_pos[4];
  int bs_pulse_off[4];
  uint32_t bs_blk_raw[4];
  uint16_t bs_blk_data[4];
  uint8_t bs_blk_flags[4]; // bit0 received, bit1 had_errors
  uint32_t bs_bits_since_lost;
  uint32_t pad;
} FmxRdsState;

// Resampler output schedule entry (host-simulated liquid resamp timing):
// y = (1-mu) * y0 + mu * y1 with
//   interp  : y0 = branch b of window(i),   y1 = branch b+1 of window(i)
//   boundary: y0 = branch 31 of window(i-1), y1 = branch 0 of window(i)
typedef struct {
  int packed; // i | (b << 16) | (boundary << 24)
  float mu;
} FmxSched;

#endif

/*
 * fmx_oracle.h -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * C API of the CPU restatement of bkram/fmtuner-sdr's per-channel FM demod hot
 * path (oracle/fmx_oracle.cpp).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library; the product path
 * (fmtuner-sdr_amd/) never links or calls it.
 *
 * Parity status: the reference delegates all DSP arithmetic to liquid-dsp
 * (jgaeddert/liquid-dsp, MIT; version UNPINNED by the reference's CI -- distro
 * libliquid-dev / brew / git HEAD).  liquid-dsp is
 * absent from this image, so every liquid object is restated here from its
 * published algorithm (choices listed in DESIGN.md section 3).  MPX / PCM parity
 * against a real liquid build is therefore UNPINNED; the RDS block-sync layer
 * is pinned against the reference's own block_sync.cpp/group.cpp compiled into
 * oracle/_ref (see oracle/Makefile), and known-answer tests pin the rest.
 */
#ifndef FMX_ORACLE_H
#define FMX_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One channel's configuration, mirroring the reference keys that
 * parameterise the hot path (config.h:46-54, main.cpp:640-710). */
typedef struct {
  int iq_rate;         /* SDR rate, e.g. 2400000 / 2048000 / 256000          */
  int dsp_rate;        /* DSP rate after /M (main.cpp:72, 240000 for 2.4M)   */
  int out_rate;        /* 32000 (main.cpp:73)                                */
  int block;           /* processing.dsp_block_samples                       */
  int w0_bandwidth_hz; /* processing.w0_bandwidth_hz (default 194000)        */
  int bandwidth_hz;    /* XDR W value, 0 = use W0 (main.cpp:416,710)         */
  int dsp_agc;         /* 0 off, 1 fast, 2 slow                              */
  int stereo;          /* processing.stereo                                  */
  int blend;           /* 0 soft, 1 normal, 2 aggressive                     */
  int deemphasis;      /* tuner.deemphasis: 0 -> 50us, 1 -> 75us, 2 -> off   */
  int force_mono;
  int force_stereo;
  int rds;             /* run the RDS decoder                                 */
} oracle_cfg;

typedef struct {
  uint16_t a, b, c, d;
  uint8_t errors;      /* rds_decoder.cpp:29-41 packing                      */
  uint8_t pad;
  uint32_t block_index;/* pipeline block in which the group was emitted     */
} oracle_group;

typedef struct {
  int n_mpx;
  int n_pcm;
  int stereo_detected;
  int pilot_tenths_khz;
  float clip_ratio;
  int n_groups;
  int stereo_indicator; /* main.cpp:1298-1300 */
} oracle_blockinfo;

/* ---- full per-channel pipeline (restates main.cpp:1232-1308) ---- */
void *oracle_pipeline_create(const oracle_cfg *cfg);
void oracle_pipeline_destroy(void *p);
void oracle_pipeline_reset(void *p); /* Runtime::reset fan-out main.cpp:686-691 + RDS reset */
/* retune (main.cpp:1028-1042): reset + fade/mute of mute_samples outputs
 * (< 0: kRetuneMuteSamples = OUTPUT_RATE/25, main.cpp:696-697) */
void oracle_pipeline_retune(void *p, int mute_samples);
/* iq: 2*iq_samples bytes (iq_samples = block*M).  Outputs may be NULL. */
int oracle_pipeline_block(void *p, const uint8_t *iq, int iq_samples,
                          float *mpx_out, float *pcm_l, float *pcm_r,
                          int pcm_cap, oracle_group *groups, int groups_cap,
                          oracle_blockinfo *info);
/* runtime setters as main.cpp applies them (keys = FMX_PARAM_* of fmx.h) */
void oracle_pipeline_set(void *p, int key, int value);
/* debug taps: which = 0 decim, 1 iqfir, 2 pilot, 3 lr, 4 af_resamp proto,
 * 5 rds_resamp proto, 6 rds_fir, 7 symsync mf, 8 symsync dmf */
int oracle_pipeline_taps(void *p, int which, float *out, int cap);

/* ---- individual reference objects (for stage-level parity) ---- */
void *oracle_decim_create(uint32_t factor, uint32_t taps_per_phase, float as);
void oracle_decim_destroy(void *p);
void oracle_decim_reset(void *p);
size_t oracle_decim_execute_complex(void *p, const uint8_t *iq, size_t in_samples,
                                    float *out_cf, size_t out_cap);
size_t oracle_decim_execute(void *p, const uint8_t *iq, size_t in_samples, uint8_t *out_u8,
                            size_t out_cap);

void *oracle_demod_create(int input_rate, int output_rate);
void oracle_demod_destroy(void *p);
void oracle_demod_reset(void *p);
void oracle_demod_set(void *p, int key, int value);
size_t oracle_demod_process_split_complex(void *p, const float *iq_cf, float *mpx,
                                          float *mono, size_t n);
size_t oracle_demod_process_split(void *p, const uint8_t *iq, float *mpx,
                                  float *mono, size_t n);
float oracle_demod_clip_ratio(void *p);

void *oracle_stereo_create(int input_rate, int output_rate);
void oracle_stereo_destroy(void *p);
void oracle_stereo_reset(void *p);
void oracle_stereo_set(void *p, int key, int value);
size_t oracle_stereo_process(void *p, const float *mpx, float *left, float *right,
                             size_t n, int *stereo, int *pilot_tenths);
/* per-sample trace of the PLL phase (float, after step) for debugging */
size_t oracle_stereo_process_trace(void *p, const float *mpx, float *left,
                                   float *right, size_t n, float *phase_trace,
                                   float *blend_trace);

void *oracle_afpost_create(int input_rate, int output_rate);
void oracle_afpost_destroy(void *p);
void oracle_afpost_reset(void *p);
void oracle_afpost_set_deemphasis(void *p, int tau_us);
size_t oracle_afpost_process(void *p, const float *l, const float *r, size_t n,
                             float *ol, float *or_, size_t cap);

void *oracle_rds_create(int input_rate);
void oracle_rds_destroy(void *p);
void oracle_rds_reset(void *p);
/* returns number of groups written; bits (optional) receives the raw
 * post-delta-decoder bit stream of this call (n_bits written). */
int oracle_rds_process(void *p, const float *mpx, size_t n, oracle_group *groups,
                       int cap, uint8_t *bits, int bits_cap, int *n_bits);

/* RDS block sync alone: push bits, collect groups (redsea BlockStream). */
void *oracle_blocksync_create(void);
void oracle_blocksync_destroy(void *p);
int oracle_blocksync_push(void *p, const uint8_t *bits, int n, oracle_group *groups,
                          int cap);

/* ---- multi-channel CPU baseline: one channel per thread ---- */
/* iq layout: [n_channels][n_blocks][2*block*M]; outputs ignored except a
 * checksum.  Returns wall seconds spent inside the DSP (excludes setup). */
double oracle_run_many(const oracle_cfg *cfg, int n_channels, const uint8_t *iq,
                       int n_blocks, int threads, double *checksum);

#ifdef __cplusplus
}
#endif
#endif

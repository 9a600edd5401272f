// fmx_synth.h -- seeded synthetic broadcast-FM IQ generator (host + device).
//
// Produces interleaved u8 IQ exactly as an RTL-SDR would deliver it
// (rtl_sdr_device.h:27 readIQ), for many independent channels.  Every
// component of the FM phase is a closed form of the integer sample index, so
// any sample of any channel can be generated independently (one GPU thread
// per sample) and the host and device produce the same stream up to the last
// ulp of the transcendental functions.  Parity tests never depend on that: the
// HIP path and the oracle always consume the same bytes.
//
// MPX (75 kHz peak deviation):
//   stereo: 0.45(L+R) + 0.45(L-R) sin(2 th_p) + 0.09 sin(th_p) + a_rds s(t) sin(3 th_p)
//   mono:   0.45 sin(2 pi f1 t) + 0.45 sin(2 pi f2 t)             (config 1)
// with th_p = 2 pi 19 kHz t, L/R single tones.  The RDS term uses rectangular
// biphase symbols; every half-bit spans exactly 24 cycles of 57 kHz, so its
// integral over complete half-bits vanishes and the phase stays closed-form.
#ifndef FMX_SYNTH_H
#define FMX_SYNTH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define FMX_HD __host__ __device__ __forceinline__
#else
#define FMX_HD inline
#endif

#include "../../include/fmx.h"

/* kind */
enum { FMX_SYNTH_MONO = 0, FMX_SYNTH_STEREO = 1, FMX_SYNTH_STEREO_RDS = 2 };

typedef fmx_synth_config fmx_synth_cfg;

#ifdef __cplusplus
extern "C" {
#endif

/* Per-channel parameters, derived from the seed only. */
typedef struct {
  int f_off;    /* carrier offset, Hz */
  int f_l, f_r; /* L/R tone frequencies, Hz (mono: f1, f2) */
  float a_l, a_r;
  float ph_l, ph_r; /* initial tone phases, rad */
  int64_t rds_off;  /* RDS bit-clock offset in samples (stations are not synchronised) */
  float amp;        /* carrier amplitude (cfg amplitude, spread over level_spread_db) */
} fmx_synth_chan;

#ifdef __cplusplus
}
#endif

FMX_HD uint64_t fmx_splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
FMX_HD float fmx_u01(uint64_t h) { /* (0,1] */
  return (float)((h >> 40) + 1) * (1.0f / 16777216.0f);
}

FMX_HD fmx_synth_chan fmx_synth_channel(const fmx_synth_cfg *cfg, uint32_t ch) {
  fmx_synth_chan c;
  uint64_t s = fmx_splitmix64((uint64_t)(cfg->seed_base + ch));
  uint64_t h1 = fmx_splitmix64(s ^ 1), h2 = fmx_splitmix64(s ^ 2), h3 = fmx_splitmix64(s ^ 3);
  int span = 2 * cfg->max_offset_hz + 1;
  c.f_off = (span > 1) ? (int)(h1 % (uint64_t)span) - cfg->max_offset_hz : 0;
  if (cfg->kind == FMX_SYNTH_MONO) {
    c.f_l = 1000;
    c.f_r = 3000;
    c.a_l = 0.45f;
    c.a_r = 0.45f;
    c.ph_l = 0.0f;
    c.ph_r = 0.0f;
  } else {
    c.f_l = 300 + (int)(h2 % 9700u);
    c.f_r = 300 + (int)((h2 >> 20) % 9700u);
    if (c.f_r == c.f_l) c.f_r += 37;
    c.a_l = 0.5f + 0.4f * fmx_u01(h3);
    c.a_r = 0.5f + 0.4f * fmx_u01(h3 >> 13);
    c.ph_l = 6.2831853f * fmx_u01(h2 >> 7);
    c.ph_r = 6.2831853f * fmx_u01(h3 >> 29);
  }
  c.rds_off = (int64_t)(fmx_splitmix64(s ^ 4) % (uint64_t)(2 * cfg->iq_rate));
  c.amp = cfg->amplitude;
  if (cfg->level_spread_db > 0.0f)
    c.amp = cfg->amplitude * powf(10.0f, -0.05f * cfg->level_spread_db * fmx_u01(fmx_splitmix64(s ^ 5)));
  return c;
}

/* angle 2 pi ((f n) mod fs) / fs for integer f (may be negative) */
FMX_HD float fmx_angle(int64_t f, int64_t n, int64_t fs) {
  int64_t r = (f * n) % fs;
  if (r < 0) r += fs;
  return (float)(6.283185307179586 * (double)r / (double)fs);
}

/* Integral of a sin(2 pi f t + ph) from 0 to t, times 2 pi * 75 kHz. */
FMX_HD float fmx_int_sin(float a, int64_t f, int64_t n, int64_t fs, float ph) {
  float k = 75000.0f * a / (float)f;
  float ang = fmx_angle(f, n, fs) + ph;
  return k * (cosf(ph) - cosf(ang));
}
/* Integral of a cos(2 pi f t + ph) from 0 to t, times 2 pi * 75 kHz. */
FMX_HD float fmx_int_cos(float a, int64_t f, int64_t n, int64_t fs, float ph) {
  float k = 75000.0f * a / (float)f;
  float ang = fmx_angle(f, n, fs) + ph;
  return k * (sinf(ang) - sinf(ph));
}

/* FM phase (rad, excluding the carrier offset) at sample n. bits: encoded
 * (differential) RDS bit table of this channel, n_bits long, may be NULL. */
FMX_HD float fmx_synth_fm_phase(const fmx_synth_cfg *cfg, const fmx_synth_chan *c, int64_t n,
                                const uint8_t *bits) {
  const int64_t fs = cfg->iq_rate;
  float ph = 0.0f;
  if (cfg->kind == FMX_SYNTH_MONO) {
    ph += fmx_int_sin(c->a_l, c->f_l, n, fs, c->ph_l);
    ph += fmx_int_sin(c->a_r, c->f_r, n, fs, c->ph_r);
    return ph;
  }
  /* 0.45 (L + R) */
  ph += fmx_int_sin(0.45f * c->a_l, c->f_l, n, fs, c->ph_l);
  ph += fmx_int_sin(0.45f * c->a_r, c->f_r, n, fs, c->ph_r);
  /* 0.45 (L - R) sin(2 th_p): a sin(wx t + p) sin(ws t) =
   *   a/2 [cos((wx - ws) t + p) - cos((wx + ws) t + p)] */
  const int64_t fs38 = 38000;
  ph += fmx_int_cos(0.225f * c->a_l, (int64_t)c->f_l - fs38, n, fs, c->ph_l);
  ph -= fmx_int_cos(0.225f * c->a_l, (int64_t)c->f_l + fs38, n, fs, c->ph_l);
  ph -= fmx_int_cos(0.225f * c->a_r, (int64_t)c->f_r - fs38, n, fs, c->ph_r);
  ph += fmx_int_cos(0.225f * c->a_r, (int64_t)c->f_r + fs38, n, fs, c->ph_r);
  /* pilot 0.09 sin(th_p) */
  ph += fmx_int_sin(0.09f, 19000, n, fs, 0.0f);
  if (cfg->kind == FMX_SYNTH_STEREO_RDS && bits && cfg->n_bits > 0) {
    /* half-bit index and symbol sign; the RDS waveform is shifted by the
     * channel's bit-clock offset (a constant phase term is dropped) */
    const int64_t nr = n + c->rds_off;
    int64_t h = (nr * 2375) / fs;
    int64_t k = h >> 1;
    int bit = bits[k % cfg->n_bits];
    float s = (bit ? 1.0f : -1.0f) * ((h & 1) ? -1.0f : 1.0f);
    float a57 = fmx_angle(57000, nr, fs);
    ph += s * (75000.0f * cfg->rds_level / 57000.0f) * (1.0f - cosf(a57));
  }
  return ph;
}

FMX_HD float fmx_gauss(uint64_t key) {
  uint64_t h1 = fmx_splitmix64(key), h2 = fmx_splitmix64(key ^ 0xA5A5A5A5ull);
  float u1 = fmx_u01(h1), u2 = fmx_u01(h2);
  return sqrtf(-2.0f * logf(u1)) * cosf(6.2831853f * u2);
}

FMX_HD uint8_t fmx_quant(float x) {
  float v = rintf(x * 127.5f + 127.5f);
  v = v < 0.0f ? 0.0f : (v > 255.0f ? 255.0f : v);
  return (uint8_t)v;
}

/* one IQ sample of channel ch at absolute sample index n */
FMX_HD void fmx_synth_sample(const fmx_synth_cfg *cfg, uint32_t ch, const fmx_synth_chan *c, int64_t n,
                             const uint8_t *bits, uint8_t *iq2) {
  const int64_t fs = cfg->iq_rate;
  float phi = fmx_angle(c->f_off, n, fs) + fmx_synth_fm_phase(cfg, c, n, bits);
  float si, co;
  si = sinf(phi);
  co = cosf(phi);
  float i = c->amp * co, q = c->amp * si;
  if (cfg->noise_std > 0.0f) {
    uint64_t key = ((uint64_t)(cfg->seed_base + ch) << 40) ^ ((uint64_t)n << 1);
    i += cfg->noise_std * fmx_gauss(key);
    q += cfg->noise_std * fmx_gauss(key | 1ull);
  }
  iq2[0] = fmx_quant(i);
  iq2[1] = fmx_quant(q);
}

#endif

// fmx_host.cpp -- host-side consumers of the GPU outputs, with the
// reference's wire and file formats.  Plain C++17, no
// HIP: the XDR server, the WAV sink and the IQ capture of fm-sdr-tuner keep
// their formats when they are fed from libfmx instead of the CPU objects.
//
//   fmx_xdr_rds_lines   XDRServer::updateRDS + evaluatePiState
//                       (src/xdr_server.cpp:189-213, 403-457): PI debounce,
//                       "P" / "R" lines, one state per channel
//   fmx_xdr_scan_line   the scan line of main.cpp:1069-1113 as pushed by
//                       XDRServer::pushScanLine (xdr_server.cpp:492-501); on
//                       the GPU every channel is a scan point measured in the
//                       same block (fmx_signal_level.level120), so a sweep is
//                       one gather instead of a retune loop
//   fmx_wav_header      AudioOutput::writeWAVHeader (audio_output.cpp:1346-1377)
//   fmx_pcm_to_s16      AudioOutput::write's volume ramp (:1432-1467) and
//                       writeWAVData's clamp + int16 conversion (:1379-1398)
//   fmx_iq_capture      writeIqCapture (main.cpp:742-747): raw u8 I/Q appended
//   fmx_iq_replay       the inverse: a capture read back as input blocks
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/fmx.h"

#ifndef FMX_SRC_SHA
#define FMX_SRC_SHA "unknown"
#endif
#ifndef FMX_KDEFS
#define FMX_KDEFS ""
#endif
extern "C" const char *fmx_build_info(void) { return "src=" FMX_SRC_SHA " defs=" FMX_KDEFS; }

namespace {

// PI confidence of `value` over the debounce buffer (the rule of
// evaluatePiState, xdr_server.cpp:189-213): `seen` = buffered copies of the
// value, `clean` = those received without block errors.  The XDR level is the
// first rule that holds, best first:
//   0  two clean copies            1  two copies, one of them clean
//   2  three copies (any errors)   3  two copies, or one clean copy
//   4  otherwise
uint8_t pi_state(const fmx_xdr_pi_state *s, uint16_t value) {
  int seen = 0, clean = 0;
  for (int i = 0; i < s->fill; i++) {
    if (s->pi_buf[i] != value) continue;
    seen++;
    clean += ((s->pi_err[i >> 3] >> (i & 7)) & 1) ? 0 : 1;
  }
  const bool rule[4] = {clean >= 2, seen >= 2 && clean > 0, seen >= 3, seen == 2 || clean > 0};
  for (uint8_t level = 0; level < 4; ++level)
    if (rule[level]) return level;
  return 4;
}

int emit(std::string &acc, const char *line) {
  acc += line;
  acc += '\n';
  return 0;
}

int copy_out(const std::string &s, char *out, int cap) {
  const int n = static_cast<int>(s.size());
  if (!out || cap < n + 1) return -(n + 1);
  std::memcpy(out, s.data(), static_cast<size_t>(n));
  out[n] = '\0';
  return n;
}

}  // namespace

extern "C" {

void fmx_xdr_pi_reset(fmx_xdr_pi_state *s) {
  if (!s) return;
  std::memset(s, 0, sizeof(*s));
  s->pos = 63; // XDRServer ctor / setFrequencyState (xdr_server.cpp:261-266, 465-470)
  s->last_state = 4;
  s->last_value = 0xFFFF;
}

int fmx_xdr_rds_lines(fmx_xdr_pi_state *s, const fmx_rds_group *g, int n, char *out, int cap) {
  if (!s || (n > 0 && !g) || n < 0) return FMX_E_INVALID;
  fmx_xdr_pi_state work = *s;
  std::string acc;
  for (int k = 0; k < n; ++k) {
    const uint16_t blockA = g[k].a;
    const uint8_t errors = g[k].errors;
    const uint8_t aErr = static_cast<uint8_t>((errors >> 6) & 0x03u);
    const uint8_t bErr = static_cast<uint8_t>((errors >> 4) & 0x03u);
    work.pos = static_cast<uint8_t>((work.pos + 1) % 64);
    work.pi_buf[work.pos] = blockA;
    const uint8_t errPos = work.pos / 8, errBit = work.pos % 8;
    if (aErr != 0) work.pi_err[errPos] |= static_cast<uint8_t>(1 << errBit);
    else work.pi_err[errPos] &= static_cast<uint8_t>(~(1 << errBit));
    if (work.fill < 64) work.fill++;
    const uint8_t st = pi_state(&work, blockA);
    if (aErr != 3 && st <= 1) {
      char line[16];
      std::snprintf(line, sizeof(line), "P%04X%.*s", blockA, static_cast<int>(std::min<uint8_t>(aErr, 3)), "???");
      emit(acc, line);
      work.last_value = blockA;
    }
    if (bErr == 0) {
      char line[32];
      std::snprintf(line, sizeof(line), "R%04X%04X%04X%02X", g[k].b, g[k].c, g[k].d, errors);
      emit(acc, line);
    }
    work.last_state = st;
  }
  const int rc = copy_out(acc, out, cap);
  if (rc >= 0) *s = work; // state advances only when the lines were delivered
  return rc;
}

int fmx_xdr_scan_line(const int *freq_khz, const double *level_sum, const int *reads, int n, char *out, int cap) {
  if (n < 0 || (n > 0 && (!freq_khz || !level_sum || !reads))) return FMX_E_INVALID;
  std::string line;
  bool first = true;
  for (int k = 0; k < n; ++k) {
    if (reads[k] <= 0) continue; // main.cpp:1099-1101
    const float rf = static_cast<float>(level_sum[k] / static_cast<double>(reads[k]));
    char pt[48];
    std::snprintf(pt, sizeof(pt), "%s%d=%.1f", first ? "" : ",", freq_khz[k], static_cast<double>(rf));
    line += pt;
    first = false;
  }
  if (!line.empty()) line = "U" + line; // XDRServer::pushScanLine
  return copy_out(line, out, cap);
}

int fmx_wav_header(uint32_t data_bytes, uint8_t *h) {
  if (!h) return FMX_E_INVALID;
  auto u32 = [&](int off, uint32_t v) {
    for (int i = 0; i < 4; ++i) h[off + i] = static_cast<uint8_t>(v >> (8 * i));
  };
  auto u16 = [&](int off, uint16_t v) {
    h[off] = static_cast<uint8_t>(v);
    h[off + 1] = static_cast<uint8_t>(v >> 8);
  };
  const uint32_t rate = 32000, channels = 2, bits = 16;
  std::memcpy(h, "RIFF", 4);
  u32(4, 36 + data_bytes);
  std::memcpy(h + 8, "WAVE", 4);
  std::memcpy(h + 12, "fmt ", 4);
  u32(16, 16);
  u16(20, 1);
  u16(22, static_cast<uint16_t>(channels));
  u32(24, rate);
  u32(28, rate * channels * bits / 8);
  u16(32, static_cast<uint16_t>(channels * bits / 8));
  u16(34, static_cast<uint16_t>(bits));
  std::memcpy(h + 36, "data", 4);
  u32(40, data_bytes);
  return 44;
}

int fmx_pcm_to_s16(const float *left, const float *right, int n, int volume_percent, float *volume_scale,
                   int16_t *out) {
  if (n < 0 || (n > 0 && (!left || !right || !out)) || !volume_scale) return FMX_E_INVALID;
  constexpr int kMaxVolumePercent = 100;
  constexpr float kDefaultVolumeScale = 0.85f, kInt16Max = 32767.0f, kVolumeEpsilon = 1e-6f;
  const int vol = std::clamp(volume_percent, 0, kMaxVolumePercent);
  const float target = (static_cast<float>(vol) / static_cast<float>(kMaxVolumePercent)) * kDefaultVolumeScale;
  const float ramp = static_cast<float>(32000) * 0.01f;
  float cur = *volume_scale;
  const float step = (target - cur) / std::max(1.0f, ramp);
  for (int i = 0; i < n; ++i) {
    if (std::abs(target - cur) > kVolumeEpsilon) {
      cur += step;
      if ((step > 0.0f && cur > target) || (step < 0.0f && cur < target)) cur = target;
    }
    const float sl = left[i] * cur, sr = right[i] * cur;
    const float l = std::max(-1.0f, std::min(1.0f, sl));
    const float r = std::max(-1.0f, std::min(1.0f, sr));
    out[2 * i] = static_cast<int16_t>(l * kInt16Max);
    out[2 * i + 1] = static_cast<int16_t>(r * kInt16Max);
  }
  *volume_scale = cur;
  return n;
}

int fmx_iq_capture(const char *path, const uint8_t *iq, int n_samples, int append) {
  if (!path || n_samples < 0 || (n_samples > 0 && !iq)) return FMX_E_INVALID;
  FILE *f = std::fopen(path, append ? "ab" : "wb");
  if (!f) return FMX_E_INVALID;
  const size_t want = static_cast<size_t>(n_samples) * 2;
  const size_t got = want ? std::fwrite(iq, 1, want, f) : 0;
  std::fclose(f);
  return got == want ? n_samples : FMX_E_INVALID;
}

int fmx_iq_replay(const char *path, long long sample_offset, int n_samples, uint8_t *out) {
  if (!path || sample_offset < 0 || n_samples < 0 || (n_samples > 0 && !out)) return FMX_E_INVALID;
  FILE *f = std::fopen(path, "rb");
  if (!f) return FMX_E_INVALID;
  if (std::fseek(f, static_cast<long>(sample_offset * 2), SEEK_SET) != 0) {
    std::fclose(f);
    return FMX_E_INVALID;
  }
  const size_t got = std::fread(out, 1, static_cast<size_t>(n_samples) * 2, f);
  std::fclose(f);
  return static_cast<int>(got / 2); // whole I/Q pairs read
}

}  // extern "C"

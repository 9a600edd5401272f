// sanitize_main.cpp -- host code under AddressSanitizer + UndefinedBehavior-
// Sanitizer (tests/test_sanitizers.py builds it with -fsanitize=address,undefined
// -fno-sanitize-recover=all and runs it on the CPU).  Links the CPU oracle
// (oracle/fmx_oracle.cpp), the product's host-side design code
// (fmx_design.cpp) and its host formats (fmx_host.cpp) from source.
//
//   sanitize_main design                  every design the product builds
//   sanitize_main host TMPDIR             XDR / scan / WAV / PCM / IQ capture
//   sanitize_main oracle IQFILE NBLK ST   oracle pipeline over u8 IQ blocks -> JSON
//   sanitize_main stages IQFILE           the oracle's per-object entry points
//   sanitize_main blocksync BITSFILE      the oracle's RDS block sync on raw bits
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "fmx_internal.h"
#include "fmx_oracle.h"

static std::vector<uint8_t> read_file(const char *path) {
  std::vector<uint8_t> v;
  FILE *f = std::fopen(path, "rb");
  if (!f) return v;
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  v.resize(static_cast<size_t>(n));
  if (n > 0 && std::fread(v.data(), 1, v.size(), f) != v.size()) v.clear();
  std::fclose(f);
  return v;
}

static fmx_config config(int iq, int dsp, int w0, int bw) {
  fmx_config c{};
  c.iq_rate = iq;
  c.dsp_rate = dsp;
  c.out_rate = 32000;
  c.block = 4096;
  c.w0_bandwidth_hz = w0;
  c.bandwidth_hz = bw;
  c.stereo = 1;
  c.blend = 1;
  c.rds = 1;
  return c;
}

static int run_design() {
  const int rates[4][2] = {{2400000, 240000}, {2048000, 256000}, {1024000, 256000}, {256000, 256000}};
  const int w0s[] = {309000, 194000, 114000, 42000, 9000};
  const int bws[] = {0, 56000, 110000, 311000};
  int built = 0;
  double sum = 0.0;
  for (auto &r : rates)
    for (int w0 : w0s)
      for (int bw : bws) {
        fmx_config c = config(r[0], r[1], w0, bw);
        auto *d = new FmxDesign();
        fmx::DesignExtras ex;
        std::string err;
        if (fmx::design_build(c, d, &ex, &err) != 0) {
          std::fprintf(stderr, "design_build failed: %s\n", err.c_str());
          return 1;
        }
        for (int i = 0; i < d->dec_len; ++i) sum += d->dec_taps[i];
        for (float v : ex.proto_rds) sum += v;
        ++built;
        delete d;
      }
  // resampler timing schedules (the host simulation k_fe8 / k_audio read)
  long outs = 0;
  for (float del : {0.7125f, 0.1333333f, 0.125f, 0.9f, 1.0f}) {
    fmx::ResampTiming t;
    fmx::timing_reset(t);
    t.del = del;
    std::vector<FmxSched> s(8192);
    for (int call = 0; call < 16; ++call) outs += fmx::timing_run(t, 4096, s.data(), static_cast<int>(s.size()));
  }
  std::printf("{\"designs\": %d, \"tap_sum\": %.9g, \"schedule_outputs\": %ld}\n", built, sum, outs);
  return 0;
}

static int run_host(const char *tmpdir) {
  // XDR P/R lines over a run of groups with PI changes and errors
  fmx_xdr_pi_state st;
  fmx_xdr_pi_reset(&st);
  std::vector<fmx_rds_group> g;
  for (int i = 0; i < 400; ++i) {
    fmx_rds_group x{};
    x.a = static_cast<uint16_t>(i < 200 ? 0x1234 : 0x5678);
    x.b = static_cast<uint16_t>(i * 2654435761u >> 16);
    x.c = static_cast<uint16_t>(i * 40503u);
    x.d = static_cast<uint16_t>(~i);
    x.errors = static_cast<uint8_t>((i * 7) & 0xFF);
    g.push_back(x);
  }
  std::vector<char> out(1 << 16);
  const int n1 = fmx_xdr_rds_lines(&st, g.data(), static_cast<int>(g.size()), out.data(), static_cast<int>(out.size()));
  const int n0 = fmx_xdr_rds_lines(&st, g.data(), static_cast<int>(g.size()), out.data(), 7); // too small: error, no overrun
  // scan line
  std::vector<int> f(300), reads(300, 3);
  std::vector<double> lv(300);
  for (int i = 0; i < 300; ++i) {
    f[static_cast<size_t>(i)] = 87500 + 100 * i;
    lv[static_cast<size_t>(i)] = 1.5 * i;
  }
  const int ns = fmx_xdr_scan_line(f.data(), lv.data(), reads.data(), 300, out.data(), static_cast<int>(out.size()));
  // WAV header + s16 PCM
  uint8_t hdr[44];
  const int nh = fmx_wav_header(123456u, hdr);
  std::vector<float> l(4096), r(4096);
  for (int i = 0; i < 4096; ++i) {
    l[static_cast<size_t>(i)] = std::sin(0.01f * i) * 1.2f;
    r[static_cast<size_t>(i)] = std::cos(0.02f * i);
  }
  float vs = 1.0f;
  std::vector<int16_t> pcm(2 * 4096);
  const int np = fmx_pcm_to_s16(l.data(), r.data(), 4096, 80, &vs, pcm.data());
  // IQ capture / replay
  const std::string path = std::string(tmpdir) + "/iq.u8";
  std::vector<uint8_t> iq(2 * 10000), back(2 * 10000);
  for (size_t i = 0; i < iq.size(); ++i) iq[i] = static_cast<uint8_t>(i * 131u);
  int rc = fmx_iq_capture(path.c_str(), iq.data(), 10000, 0);
  rc |= fmx_iq_capture(path.c_str(), iq.data(), 10000, 1);
  const int nr = fmx_iq_replay(path.c_str(), 10000, 10000, back.data());
  const bool same = std::memcmp(iq.data(), back.data(), iq.size()) == 0;
  std::printf("{\"xdr_bytes\": %d, \"xdr_small\": %d, \"scan_bytes\": %d, \"wav\": %d, \"pcm\": %d, \"capture_rc\": %d, "
              "\"replay\": %d, \"replay_equal\": %s}\n",
              n1, n0, ns, nh, np, rc, nr, same ? "true" : "false");
  return 0;
}

static int run_oracle(const char *iqfile, int nblk, int stereo) {
  const std::vector<uint8_t> iq = read_file(iqfile);
  const int B = 4096, M = 10;
  const size_t per = static_cast<size_t>(2 * B * M);
  if (iq.size() < per * static_cast<size_t>(nblk)) return 2;
  oracle_cfg c{2400000, 240000, 32000, B, 194000, 0, 0, stereo, 1, 0, 0, 0, 1};
  void *p = oracle_pipeline_create(&c);
  std::vector<float> mpx(static_cast<size_t>(B)), pl(2 * static_cast<size_t>(B)), pr(2 * static_cast<size_t>(B));
  std::vector<oracle_group> grp(64);
  std::printf("[");
  for (int b = 0; b < nblk; ++b) {
    oracle_blockinfo info{};
    oracle_pipeline_block(p, iq.data() + per * static_cast<size_t>(b), B * M, mpx.data(), pl.data(), pr.data(),
                          static_cast<int>(pl.size()), grp.data(), static_cast<int>(grp.size()), &info);
    std::printf("%s{\"stereo\": %d, \"pilot\": %d, \"n_pcm\": %d, \"groups\": [", b ? ", " : "", info.stereo_detected,
                info.pilot_tenths_khz, info.n_pcm);
    for (int k = 0; k < info.n_groups; ++k)
      std::printf("%s[%d, %d, %d, %d, %d]", k ? ", " : "", grp[static_cast<size_t>(k)].a, grp[static_cast<size_t>(k)].b,
                  grp[static_cast<size_t>(k)].c, grp[static_cast<size_t>(k)].d, grp[static_cast<size_t>(k)].errors);
    std::printf("], \"pcm_l_head\": [%.9g, %.9g, %.9g, %.9g], \"mpx_head\": [%.9g, %.9g, %.9g, %.9g]}", pl[0], pl[1],
                pl[2], pl[3], mpx[0], mpx[1], mpx[2], mpx[3]);
  }
  std::printf("]\n");
  oracle_pipeline_retune(p, -1);
  oracle_pipeline_reset(p);
  oracle_pipeline_destroy(p);
  return 0;
}

static int run_stages(const char *iqfile) {
  const std::vector<uint8_t> iq = read_file(iqfile);
  const size_t n_iq = 40960;
  if (iq.size() < 2 * n_iq) return 2;
  void *dec = oracle_decim_create(10, 28, 80.0f);
  std::vector<float> cf(2 * 4096 + 16);
  const size_t nd = oracle_decim_execute_complex(dec, iq.data(), n_iq, cf.data(), 4096);
  void *dm = oracle_demod_create(240000, 32000);
  std::vector<float> mpx(4096), mono(4096);
  const size_t nm = oracle_demod_process_split_complex(dm, cf.data(), mpx.data(), mono.data(), nd);
  void *sd = oracle_stereo_create(240000, 32000);
  std::vector<float> l(4096), r(4096);
  int st = 0, pil = 0;
  const size_t ns = oracle_stereo_process(sd, mpx.data(), l.data(), r.data(), nd, &st, &pil); // nm: mono outputs at 32 kHz
  void *af = oracle_afpost_create(240000, 32000);
  std::vector<float> ol(1024), orr(1024);
  const size_t na = oracle_afpost_process(af, l.data(), r.data(), ns, ol.data(), orr.data(), ol.size());
  void *rd = oracle_rds_create(240000);
  std::vector<oracle_group> g(16);
  std::vector<uint8_t> bits(512);
  int nb = 0;
  const int ng = oracle_rds_process(rd, mpx.data(), nd, g.data(), 16, bits.data(), 512, &nb);
  oracle_decim_destroy(dec);
  oracle_demod_destroy(dm);
  oracle_stereo_destroy(sd);
  oracle_afpost_destroy(af);
  oracle_rds_destroy(rd);
  std::printf("{\"decim\": %zu, \"demod\": %zu, \"stereo\": %zu, \"afpost\": %zu, \"rds_groups\": %d, \"rds_bits\": %d}\n",
              nd, nm, ns, na, ng, nb);
  return 0;
}

static int run_blocksync(const char *bitsfile) {
  const std::vector<uint8_t> bits = read_file(bitsfile);
  void *b = oracle_blocksync_create();
  std::vector<oracle_group> g(4096);
  int total = 0;
  for (size_t off = 0; off < bits.size(); off += 997) {
    const int n = static_cast<int>(std::min<size_t>(997, bits.size() - off));
    total += oracle_blocksync_push(b, bits.data() + off, n, g.data(), static_cast<int>(g.size()));
  }
  oracle_blocksync_destroy(b);
  std::printf("{\"groups\": %d}\n", total);
  return 0;
}

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  const std::string mode = argv[1];
  if (mode == "design") return run_design();
  if (mode == "host" && argc >= 3) return run_host(argv[2]);
  if (mode == "oracle" && argc >= 5) return run_oracle(argv[2], std::atoi(argv[3]), std::atoi(argv[4]));
  if (mode == "stages" && argc >= 3) return run_stages(argv[2]);
  if (mode == "blocksync" && argc >= 3) return run_blocksync(argv[2]);
  return 2;
}

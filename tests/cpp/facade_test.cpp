// facade_test.cpp -- parity of the C++ facades (include/fmx_blocks.hpp)
// against the oracle's reference objects on the same synthetic IQ.
// Run on a GPU by tests/test_facades.py; prints one line per check and
// exits non-zero on failure.  Tolerances as tests/test_gpu_parity.py.
#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "fmx_blocks.hpp"
#include "fmx_oracle.h"

static int g_fail = 0;
static void expect(bool ok, const char *what, double v) {
  std::printf("%-44s %-4s %.3g\n", what, ok ? "ok" : "FAIL", v);
  if (!ok) g_fail = 1;
}
static double rms(const float *a, const float *b, size_t n) {
  double s = 0.0;
  for (size_t i = 0; i < n; ++i) s += (double)(a[i] - b[i]) * (a[i] - b[i]);
  return n ? std::sqrt(s / n) : 0.0;
}
static double maxd(const float *a, const float *b, size_t n) {
  double m = 0.0;
  for (size_t i = 0; i < n; ++i) m = std::max(m, (double)std::fabs(a[i] - b[i]));
  return m;
}

int main() {
  const int M = 10, nblk = 30;
  const size_t B = 4096, NS = B * nblk;  // DSP samples
  fmx_synth_config sc{};
  sc.iq_rate = 2400000;
  sc.kind = 2;
  sc.amplitude = 0.8f;
  sc.seed_base = 0xF00D;
  sc.max_offset_hz = 5000;
  sc.rds_level = 0.05f;
  sc.n_bits = 8192;
  std::vector<uint8_t> bits(sc.n_bits);
  fmx_synth_rds_bits(&sc, 7, 1, bits.data(), nullptr);
  std::vector<uint8_t> iq(2 * NS * M);
  fmx_synth_host(&sc, 7, 1, 0, (int)(NS * M), bits.data(), iq.data(), iq.size(), 4);

  // ---- ComplexDecimator (odd call sizes; remainders dropped as in the reference) ----
  std::vector<std::complex<float>> bb_f(NS), bb_o(NS);
  {
    fmx::ComplexDecimator dec;
    dec.init(M, 28, 80.0f);
    void *od = oracle_decim_create(M, 28, 80.0f);
    const size_t calls[] = {40960, 12345, 90000, 3, 40960 * 3};
    size_t off = 0, of = 0, oo = 0;
    for (size_t c : calls) {
      if (off + c > NS * M) break;
      of += dec.executeComplex(iq.data() + 2 * off, c, bb_f.data() + of, NS - of);
      oo += oracle_decim_execute_complex(od, iq.data() + 2 * off, c, reinterpret_cast<float *>(bb_o.data() + oo),
                                         NS - oo);
      off += c;
    }
    expect(of == oo, "decimator output count", (double)of);
    expect(maxd(reinterpret_cast<float *>(bb_f.data()), reinterpret_cast<float *>(bb_o.data()), 2 * of) < 1e-5,
           "decimator max |d|", maxd(reinterpret_cast<float *>(bb_f.data()), reinterpret_cast<float *>(bb_o.data()),
                                     2 * of));
    oracle_decim_destroy(od);
  }
  // reference baseband for the rest: the oracle decimator over whole blocks
  {
    void *od = oracle_decim_create(M, 28, 80.0f);
    oracle_decim_execute_complex(od, iq.data(), NS * M, reinterpret_cast<float *>(bb_o.data()), NS);
    oracle_decim_destroy(od);
  }
  // ---- FMDemod mono path (processSplitComplex with monoOut) ----
  std::vector<float> mpx_o(NS), mono_o(NS), mpx_f(NS), mono_f(NS);
  size_t km_o = 0, km_f = 0;
  {
    fmx::FMDemod dm(240000, 32000);
    void *od = oracle_demod_create(240000, 32000);
    const size_t calls[] = {4096, 3000, 9000, 4096, 20000};
    size_t off = 0;
    while (off < NS) {
      for (size_t c : calls) {
        c = std::min(c, NS - off);
        if (!c) break;
        km_f += dm.processSplitComplex(bb_o.data() + off, mpx_f.data() + off, mono_f.data() + km_f, c);
        km_o += oracle_demod_process_split_complex(od, reinterpret_cast<const float *>(bb_o.data() + off),
                                                   mpx_o.data() + off, mono_o.data() + km_o, c);
        off += c;
      }
    }
    expect(km_f == km_o, "FMDemod mono count", (double)km_f);
    expect(maxd(mpx_f.data(), mpx_o.data(), NS) < 1e-4, "FMDemod MPX max |d|", maxd(mpx_f.data(), mpx_o.data(), NS));
    expect(rms(mono_f.data(), mono_o.data(), km_o) < 1e-4, "FMDemod mono RMS", rms(mono_f.data(), mono_o.data(), km_o));
    oracle_demod_destroy(od);
  }
  // ---- StereoDecoder ----
  std::vector<float> l_o(NS), r_o(NS), l_f(NS), r_f(NS);
  {
    fmx::StereoDecoder st(240000, 32000);
    void *os = oracle_stereo_create(240000, 32000);
    int st_o = 0, pil_o = 0, mism = 0;
    for (size_t b = 0; b < nblk; ++b) {
      st.processAudio(mpx_o.data() + b * B, l_f.data() + b * B, r_f.data() + b * B, B);
      oracle_stereo_process(os, mpx_o.data() + b * B, l_o.data() + b * B, r_o.data() + b * B, B, &st_o, &pil_o);
      mism += (st.isStereo() != (st_o != 0)) + (st.getPilotLevelTenthsKHz() != pil_o);
    }
    expect(mism == 0, "StereoDecoder flag/pilot mismatches", mism);
    expect(st_o != 0, "StereoDecoder acquired stereo", st_o);
    const double e = std::max(rms(l_f.data(), l_o.data(), NS), rms(r_f.data(), r_o.data(), NS));
    expect(e < 1e-4, "StereoDecoder L/R RMS", e);
    oracle_stereo_destroy(os);
  }
  // ---- AFPostProcessor ----
  {
    fmx::AFPostProcessor af(240000, 32000);
    void *oa = oracle_afpost_create(240000, 32000);
    std::vector<float> al_f(NS), ar_f(NS), al_o(NS), ar_o(NS);
    size_t kf = 0, ko = 0;
    for (size_t b = 0; b < nblk; ++b) {
      kf += af.process(l_o.data() + b * B, r_o.data() + b * B, B, al_f.data() + kf, ar_f.data() + kf, B);
      ko += oracle_afpost_process(oa, l_o.data() + b * B, r_o.data() + b * B, B, al_o.data() + ko, ar_o.data() + ko, B);
    }
    expect(kf == ko, "AFPostProcessor count", (double)kf);
    const double e = std::max(rms(al_f.data(), al_o.data(), ko), rms(ar_f.data(), ar_o.data(), ko));
    expect(e < 1e-4, "AFPostProcessor RMS", e);
    oracle_afpost_destroy(oa);
  }
  // ---- RDSDecoder ----
  {
    fmx::RDSDecoder rd(240000);
    void *orr = oracle_rds_create(240000);
    std::vector<oracle_group> go;
    std::vector<fmx::RDSGroup> gf;
    for (size_t b = 0; b < nblk; ++b) {
      rd.process(mpx_o.data() + b * B, B, [&](const fmx::RDSGroup &g) { gf.push_back(g); });
      oracle_group tmp[16];
      const int k = oracle_rds_process(orr, mpx_o.data() + b * B, B, tmp, 16, nullptr, 0, nullptr);
      for (int i = 0; i < k; ++i) go.push_back(tmp[i]);
    }
    bool same = gf.size() == go.size();
    for (size_t i = 0; same && i < gf.size(); ++i)
      same = gf[i].blockA == go[i].a && gf[i].blockB == go[i].b && gf[i].blockC == go[i].c &&
             gf[i].blockD == go[i].d && gf[i].errors == go[i].errors;
    expect(same, "RDSDecoder groups identical", (double)gf.size());
    expect(go.size() >= 2, "RDSDecoder decoded groups", (double)go.size());
    oracle_rds_destroy(orr);
  }
  // ---- ComplexDecimator::execute: u8 -> u8 requantised (liquid_primitives.cpp:422-459) ----
  {
    fmx::ComplexDecimator dec;
    dec.init(M, 28, 80.0f);
    void *od = oracle_decim_create(M, 28, 80.0f);
    std::vector<uint8_t> of(2 * NS), oo(2 * NS);
    const size_t nf = dec.execute(iq.data(), NS * M, of.data(), NS);
    const size_t no = oracle_decim_execute(od, iq.data(), NS * M, oo.data(), NS);
    int maxdiff = 0;
    size_t differ = 0;
    for (size_t i = 0; i < 2 * no; ++i) {
      const int d = std::abs((int)of[i] - (int)oo[i]);
      maxdiff = std::max(maxdiff, d);
      differ += d != 0;
    }
    expect(nf == no, "ComplexDecimator::execute count", (double)nf);
    // float parity (< 1e-5) leaves truncation at .999 / .000 boundaries: one LSB
    expect(maxdiff <= 1, "ComplexDecimator::execute max |d| (LSB)", maxdiff);
    expect(differ * 1000 <= 2 * no, "ComplexDecimator::execute bytes differing", (double)differ / (2.0 * no));
    oracle_decim_destroy(od);
  }
  // ---- FMDemod::process / processComplex / processNoDownsample (fm_demod.cpp:228-279) ----
  {
    // u8 IQ at the DSP rate (256 kHz, FMDemod's own byte path)
    fmx_synth_config s2 = sc;
    s2.iq_rate = 256000;
    const size_t N2 = 4096 * 12;
    std::vector<uint8_t> bits2(sc.n_bits);
    fmx_synth_rds_bits(&s2, 9, 1, bits2.data(), nullptr);
    std::vector<uint8_t> iq2(2 * N2);
    fmx_synth_host(&s2, 9, 1, 0, (int)N2, bits2.data(), iq2.data(), iq2.size(), 4);
    fmx::FMDemod dm(256000, 32000), dn(256000, 32000), dc(240000, 32000);
    void *om = oracle_demod_create(256000, 32000), *on = oracle_demod_create(256000, 32000);
    void *oc = oracle_demod_create(240000, 32000);
    std::vector<float> af(N2), ao(N2), mf(N2), mo(N2), scratch(N2), cf_(NS), co(NS);
    size_t kf = 0, ko = 0, kcf = 0, kco = 0;
    for (size_t off = 0; off < N2; off += 4096) {
      dm.process(iq2.data() + 2 * off, af.data() + kf, 4096);
      kf += dm.getLastAudioCount();
      ko += oracle_demod_process_split(om, iq2.data() + 2 * off, scratch.data(), ao.data() + ko, 4096);
      dn.processNoDownsample(iq2.data() + 2 * off, mf.data() + off, 4096);
      oracle_demod_process_split(on, iq2.data() + 2 * off, mo.data() + off, nullptr, 4096);
    }
    for (size_t off = 0; off < 4096 * 12; off += 4096) {
      dc.processComplex(bb_o.data() + off, cf_.data() + kcf, 4096);
      kcf += dc.getLastAudioCount();
      kco += oracle_demod_process_split_complex(oc, reinterpret_cast<const float *>(bb_o.data() + off),
                                                scratch.data(), co.data() + kco, 4096);
    }
    expect(kf == ko && ko > 0, "FMDemod::process audio count", (double)kf);
    expect(rms(af.data(), ao.data(), ko) < 1e-5, "FMDemod::process audio RMS", rms(af.data(), ao.data(), ko));
    expect(maxd(mf.data(), mo.data(), N2) < 3e-4, "FMDemod::processNoDownsample MPX max |d|",
           maxd(mf.data(), mo.data(), N2));
    expect(kcf == kco && kco > 0, "FMDemod::processComplex audio count", (double)kcf);
    expect(rms(cf_.data(), co.data(), kco) < 1e-5, "FMDemod::processComplex audio RMS",
           rms(cf_.data(), co.data(), kco));
    oracle_demod_destroy(om);
    oracle_demod_destroy(on);
    oracle_demod_destroy(oc);
  }
  // ---- any de-emphasis constant and deviation (fm_demod.cpp:50-71, af_post_processor.cpp:31-45) ----
  {
    fmx::FMDemod dm(240000, 32000);
    void *od = oracle_demod_create(240000, 32000);
    fmx::AFPostProcessor af(240000, 32000);
    void *oa = oracle_afpost_create(240000, 32000);
    std::vector<float> mf(NS), mo(NS), aof(NS), aoo(NS), alf(NS), arf(NS), alo(NS), aro(NS);
    size_t kf = 0, ko = 0, kaf = 0, kao = 0;
    for (size_t b = 0; b < 12; ++b) {
      if (b == 0) {
        dm.setDeemphasis(60);
        oracle_demod_set(od, 1, 60);
        dm.setDeviation(50000.0);
        oracle_demod_set(od, 5, 50000);
        af.setDeemphasis(100);
        oracle_afpost_set_deemphasis(oa, 100);
      }
      if (b == 6) {  // a second change mid-stream: the IIR / discriminator re-created
        dm.setDeemphasis(120);
        oracle_demod_set(od, 1, 120);
        dm.setDeviation(67500.0);
        oracle_demod_set(od, 5, 67500);
        af.setDeemphasis(0);
        oracle_afpost_set_deemphasis(oa, 0);
      }
      kf += dm.processSplitComplex(bb_o.data() + b * B, mf.data() + b * B, aof.data() + kf, B);
      ko += oracle_demod_process_split_complex(od, reinterpret_cast<const float *>(bb_o.data() + b * B),
                                               mo.data() + b * B, aoo.data() + ko, B);
      kaf += af.process(l_o.data() + b * B, r_o.data() + b * B, B, alf.data() + kaf, arf.data() + kaf, B);
      kao += oracle_afpost_process(oa, l_o.data() + b * B, r_o.data() + b * B, B, alo.data() + kao,
                                   aro.data() + kao, B);
    }
    expect(kf == ko, "FMDemod tau 60/120 us, 50/67.5 kHz: count", (double)kf);
    expect(maxd(mf.data(), mo.data(), 12 * B) < 3e-4, "FMDemod custom deviation MPX max |d|",
           maxd(mf.data(), mo.data(), 12 * B));
    expect(rms(aof.data(), aoo.data(), ko) < 1e-5, "FMDemod custom de-emphasis mono RMS",
           rms(aof.data(), aoo.data(), ko));
    expect(kaf == kao, "AFPostProcessor tau 100 us / off: count", (double)kaf);
    expect(std::max(rms(alf.data(), alo.data(), kao), rms(arf.data(), aro.data(), kao)) < 1e-5,
           "AFPostProcessor custom de-emphasis RMS",
           std::max(rms(alf.data(), alo.data(), kao), rms(arf.data(), aro.data(), kao)));
    oracle_demod_destroy(od);
    oracle_afpost_destroy(oa);
  }
  // ---- settings outside the GPU build fail loudly ----
  {
    bool threw = false;
    try {
      fmx::ComplexDecimator dec;
      dec.init(3, 12, 80.0f);
    } catch (const std::invalid_argument &) {
      threw = true;
    }
    expect(threw, "unsupported decimator design throws", threw);
  }
  std::printf(g_fail ? "FACADES FAIL\n" : "FACADES OK\n");
  return g_fail;
}

// ref_driver.cpp -- TEST INFRASTRUCTURE ONLY.
//
// C entry points over the reference's OWN compilable sources, linked into
// oracle/_ref/libfmx_ref.so by oracle/Makefile (sources are compiled where they
// lie under /root/reference; nothing is copied):
//   src/redsea_port/block_sync.cpp, group.cpp, util/util.cpp  (RDS block sync)
//   src/signal_level.cpp, src/cpu_features.cpp                 (RF level, 8f row 1)
// It pins the oracle's and the GPU's block-sync restatement and the RF level
// computation against the reference itself.
#include <cstdint>
#include <cstring>

#include "redsea_port/block_sync.hh"
#include "redsea_port/group.hh"
#include "redsea_port/options.hh"
#include "signal_level.h"

extern "C" {

struct ref_group {
  uint16_t a, b, c, d;
  uint8_t errors;
  uint8_t pad;
  uint32_t bit_index;
};

void *ref_blocksync_create(void) {
  auto *bs = new redsea::BlockStream();
  redsea::Options opt;
  opt.use_fec = true; // rds_decoder.cpp:17-19
  bs->init(opt);
  return bs;
}

void ref_blocksync_destroy(void *p) { delete static_cast<redsea::BlockStream *>(p); }

// Mirrors RDSDecoder::Impl::emitGroups (rds_decoder.cpp:43-59).
int ref_blocksync_push(void *p, const uint8_t *bits, int n, ref_group *out, int cap) {
  auto *bs = static_cast<redsea::BlockStream *>(p);
  int ng = 0;
  for (int i = 0; i < n; ++i) {
    bs->pushBit(bits[i] != 0);
    if (!bs->hasGroupReady()) continue;
    const redsea::Group g = bs->popGroup();
    auto e = [&](redsea::eBlockNumber b) -> uint8_t {
      if (!g.has(b)) return 3;
      return g.hadErrors(b) ? 1 : 0;
    };
    if (out && ng < cap) {
      ref_group r{};
      r.a = g.has(redsea::BLOCK1) ? g.get(redsea::BLOCK1) : 0;
      r.b = g.has(redsea::BLOCK2) ? g.get(redsea::BLOCK2) : 0;
      r.c = g.has(redsea::BLOCK3) ? g.get(redsea::BLOCK3) : 0;
      r.d = g.has(redsea::BLOCK4) ? g.get(redsea::BLOCK4) : 0;
      r.errors = static_cast<uint8_t>((e(redsea::BLOCK1) << 6) | (e(redsea::BLOCK2) << 4) |
                                      (e(redsea::BLOCK3) << 2) | e(redsea::BLOCK4));
      r.bit_index = static_cast<uint32_t>(i);
      out[ng] = r;
    }
    ng++;
  }
  return ng;
}

// computeSignalLevel (signal_level.cpp:145-203): out = {level120, dbfs,
// compensatedDbfs, hardClipRatio, nearClipRatio}
void ref_signal_level(const uint8_t *iq, size_t samples, int gain_db, double comp, double bias, double floor_db,
                      double ceil_db, double *out5) {
  const SignalLevelResult r = computeSignalLevel(iq, samples, gain_db, comp, bias, floor_db, ceil_db);
  out5[0] = r.level120;
  out5[1] = r.dbfs;
  out5[2] = r.compensatedDbfs;
  out5[3] = r.hardClipRatio;
  out5[4] = r.nearClipRatio;
}

float ref_smooth_signal_level(float input, int *initialized, float *value) {
  SignalLevelSmoother s;
  s.initialized = *initialized != 0;
  s.value = *value;
  const float r = smoothSignalLevel(input, s);
  *initialized = s.initialized ? 1 : 0;
  *value = s.value;
  return r;
}

} // extern "C"

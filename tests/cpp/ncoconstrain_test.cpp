// ncoconstrain_test.cpp -- fmx_nco_constrain (fmtuner-sdr_amd/csrc/fmx_math.h,
// the kernels' NCO phase-increment constrain: k_pll's PLL chain,
// stereo_decoder.cpp:254-256, and k_rds's PSK loop, subcarrier.cpp:205-209)
// against the reference form fmx_nco_constrain_ref (liquid nco.proto.c, as
// oracle/fmx_oracle.cpp's lq::nco_constrain) for every float bit pattern
// (NaN and Inf included; the conversion follows the device's v_cvt_u32_f32).
// Also fmx_nco_phase (the NCO phase of a word in float arithmetic) against
// the reference's double form, for every word.
// Prints JSON {"checked": N, "mismatches": M, "phase_mismatches": P, "first": [...]}.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../fmtuner-sdr_amd/csrc/fmx_math.h"

static float bits2f(uint32_t u) {
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

int main(int argc, char **argv) {
  const long long stride = (argc > 1) ? std::atoll(argv[1]) : 1;
  unsigned long long checked = 0, bad = 0, bad_phase = 0;
  uint32_t first[4] = {0, 0, 0, 0};
#pragma omp parallel for reduction(+ : checked, bad, bad_phase) schedule(static)
  for (long long i = 0; i < (1LL << 32); i += stride) {
    const float x = bits2f((uint32_t)i);
    checked++;
    const float pa = fmx_nco_phase((uint32_t)i), pb = fmx_nco_phase_ref((uint32_t)i);
    if (std::memcmp(&pa, &pb, 4) != 0) bad_phase++;
    if (fmx_nco_constrain(x) != fmx_nco_constrain_ref(x)) {
      bad++;
#pragma omp critical
      {
        for (int k = 0; k < 4; ++k)
          if (first[k] == 0) {
            first[k] = (uint32_t)i;
            break;
          }
      }
    }
  }
  std::printf("{\"stride\": %lld, \"checked\": %llu, \"mismatches\": %llu, \"phase_mismatches\": %llu, \"first\": [%u, %u, %u, %u]}\n", stride,
              checked, bad, bad_phase, first[0], first[1], first[2], first[3]);
  return 0;
}

// divconst_test.cpp -- fmx_div_const (fmtuner-sdr_amd/csrc/fmx_math.h) against
// IEEE x / c for every finite float x (all 2^32 bit patterns, NaN/Inf
// skipped) and each divisor the kernels use it for:
//   cR = 0.040 - 0.022, cC = 0.18 - 0.11, cP = 320 - 180  (stereo blend target,
//   stereo_decoder.cpp:142-147), 2 pi (PLL error Hz, :157), 57000 (RDS NCO
//   quad-phase wrapper, liquid_wrappers.cpp:133), 3 (RDS symsync output
//   scale, liquid symsync_crcf, as k_rds restates it).
// Prints JSON: per divisor the mismatches (all at |x| < 1e-30 -- "bad_ge_1e-30"
// must be 0) among normal |x| <= 2^60 (and 0), the first few,
// and whether every mismatch is a -0 / +0 sign (which the kernels absorb).
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
static uint32_t f2bits(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return u;
}

int main(int argc, char **argv) {
  // stride 1 = every bit pattern (exhaustive, ~3 min on 8 cores); the CPU
  // suite runs stride 7 (all exponents, a seventh of the mantissas)
  const long long stride = (argc > 1) ? std::atoll(argv[1]) : 1;
  const float divs[6] = {0.040f - 0.022f, 0.18f - 0.11f, 320.0f - 180.0f, 2.0f * 3.14159265358979323846f, 57000.0f, 3.0f};
  const char *names[6] = {"cR", "cC", "cP", "2pi", "57000", "3"};
  std::printf("{");
  for (int d = 0; d < 6; ++d) {
    const float c = divs[d];
    const float rc = 1.0f / c;
    unsigned long long bad = 0, zero_sign = 0, bad_ge = 0;
    float max_bad = 0.0f;
    uint32_t first[4] = {0, 0, 0, 0};
#pragma omp parallel for reduction(+ : bad, zero_sign, bad_ge) reduction(max : max_bad) schedule(static)
    for (long long i = 0; i < (1LL << 32); i += stride) {
      const float x = bits2f((uint32_t)i);
      // normal numerators up to 2^60 (subnormal ones do not occur: the
      // kernels' numerators are 0 or >= 1e-9 in size)
      if (!std::isfinite(x) || std::fabs(x) > 1.152921504606847e18f) continue;
      if (x != 0.0f && std::fabs(x) < 1.1754943508222875e-38f) continue;
      const float a = fmx_div_const(x, c, rc);
      const float b = x / c;
      if (f2bits(a) != f2bits(b)) {
        if (a == 0.0f && b == 0.0f) {
          zero_sign++;
        } else {
          bad++;
          if (std::fabs(x) >= 1e-30f) bad_ge++;
          if (std::fabs(x) > max_bad) max_bad = std::fabs(x);
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
    }
    std::printf("%s\"%s\": {\"bad\": %llu, \"bad_ge_1e-30\": %llu, \"max_bad_abs\": %g, \"zero_sign\": %llu, "
                "\"first\": [%g, %g, %g, %g]}",
                d ? ", " : "", names[d], bad, bad_ge, max_bad, zero_sign, bits2f(first[0]), bits2f(first[1]),
                bits2f(first[2]), bits2f(first[3]));
  }
  std::printf("}\n");
  return 0;
}

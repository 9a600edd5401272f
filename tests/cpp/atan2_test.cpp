// fmx_atan2f (fmx_math.h, the discriminator's atan2) against double atan2 and
// against the C library's atan2f, over random IQ-product arguments (both
// signs, magnitudes 1e-12 .. 1e3) and the axes.  Prints JSON: max error in
// ulp of the double result, max |difference| to atan2f.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

#include "../../fmtuner-sdr_amd/csrc/fmx_math.h"

static double ulp_of(double v) {
  const float f = (float)std::fabs(v);
  return (double)std::nextafter(f, INFINITY) - (double)f;
}

int main(int argc, char **argv) {
  const long n = (argc > 1) ? std::atol(argv[1]) : 4000000;
  std::mt19937_64 rng(1234);
  std::uniform_real_distribution<double> ue(-12.0, 3.0), us(-1.0, 1.0);
  double max_ulp = 0.0, max_lib = 0.0;
  auto one = [&](float y, float x) {
    const double ref = std::atan2((double)y, (double)x);
    const float got = fmx_atan2f(y, x);
    const double e = std::fabs((double)got - ref) / ulp_of(ref == 0.0 ? 1e-30 : ref);
    if (e > max_ulp) max_ulp = e;
    const double d = std::fabs((double)got - (double)std::atan2(y, x));
    if (d > max_lib) max_lib = d;
  };
  for (long i = 0; i < n; ++i) {
    const float y = (float)(std::pow(10.0, ue(rng)) * (us(rng) < 0 ? -1.0 : 1.0));
    const float x = (float)(std::pow(10.0, ue(rng)) * (us(rng) < 0 ? -1.0 : 1.0));
    one(y, x);
    one(y, (float)(x * 1e-3));
    one((float)(y * 1e-3), x);
  }
  const float ax[] = {1.0f, -1.0f, 0.5f, -2.0f, 1e-20f, -1e-20f};
  for (float v : ax) {
    one(v, 0.0f);
    one(0.0f, v);
    one(v, v);
    one(v, -v);
  }
  std::printf("{\"max_ulp\": %.4f, \"max_abs_vs_atan2f\": %.3e, \"zero_zero\": %.1f}\n", max_ulp, max_lib,
              (double)fmx_atan2f(0.0f, 0.0f));
  return 0;
}

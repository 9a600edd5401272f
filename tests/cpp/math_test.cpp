// Accuracy of fmx_sincos (fmtuner-sdr_amd/csrc/fmx_math.h) against the
// correctly rounded sin/cos over the phase range the kernels use.
// Prints: max error in ulps of the result, max absolute error, and the
// fraction of inputs whose results differ from glibc sinf/cosf.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdint>
#include "../../fmtuner-sdr_amd/csrc/fmx_math.h"

static double ulp_of(float v) {
  float a = std::fabs(v);
  return (double)std::nextafter(a, INFINITY) - (double)a;
}
int main(int argc, char **argv) {
  const double lo = -2.0 * M_PI, hi = 2.0 * M_PI;
  const long N = argc > 1 ? atol(argv[1]) : 20000000;
  double max_ulp = 0, max_abs = 0;
  long diff_glibc = 0;
  for (long i = 0; i <= N; ++i) {
    float x = (float)(lo + (hi - lo) * (double)i / (double)N);
    float s, c;
    fmx_sincos(x, &s, &c);
    const double ds = std::sin((double)x), dc = std::cos((double)x);
    const float rs = (float)ds, rc = (float)dc;
    // error relative to ulp(max(|result|, 2^-24)) : absolute near zeros
    const double es = std::fabs((double)s - ds) / std::fmax(ulp_of(rs), ulp_of(1.0f) / 2);
    const double ec = std::fabs((double)c - dc) / std::fmax(ulp_of(rc), ulp_of(1.0f) / 2);
    max_ulp = std::fmax(max_ulp, std::fmax(es, ec));
    max_abs = std::fmax(max_abs, std::fmax(std::fabs((double)s - ds), std::fabs((double)c - dc)));
    if (s != sinf(x) || c != cosf(x)) diff_glibc++;
  }
  // NCO phases (k_pll): the float phase of theta with the quadrant count taken
  // from theta itself, every 97th word plus the quadrant edges
  double nco_ulp = 0;
  auto nco = [&](uint32_t th) {
    const float x = (float)((double)(float)th * (6.283185307179586 / 4294967296.0));
    const int qi = fmx_nco_quadrant(th);
    float s, c;
    fmx_sincos_q(x, (float)qi, qi, &s, &c);
    const double ds = std::sin((double)x), dc = std::cos((double)x);
    const double es = std::fabs((double)s - ds) / std::fmax(ulp_of((float)ds), ulp_of(1.0f) / 2);
    const double ec = std::fabs((double)c - dc) / std::fmax(ulp_of((float)dc), ulp_of(1.0f) / 2);
    nco_ulp = std::fmax(nco_ulp, std::fmax(es, ec));
  };
  for (uint64_t th = 0; th < (1ull << 32); th += 97) nco((uint32_t)th);
  for (uint32_t k = 0; k < 8; ++k)
    for (int d = -4096; d <= 4096; ++d) nco((uint32_t)(k * 0x20000000u + (uint32_t)d));
  std::printf("{\"max_ulp\": %.3f, \"max_abs\": %.3e, \"frac_diff_glibc\": %.5f, \"nco_max_ulp\": %.3f}\n", max_ulp,
              max_abs, (double)diff_glibc / (double)(N + 1), nco_ulp);
  return 0;
}

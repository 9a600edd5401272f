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
  std::printf("{\"max_ulp\": %.3f, \"max_abs\": %.3e, \"frac_diff_glibc\": %.5f}\n", max_ulp, max_abs,
              (double)diff_glibc / (double)(N + 1));
  return 0;
}

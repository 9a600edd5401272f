// pllsin_test.cpp -- the stereo PLL chain's sine (pll_sin_word, fmx_math.h)
// over NCO phase words theta (stride argv[1], 1 = all 2^32), against
//   * sin of the reference's float phase (float)(2 pi (float)theta / 2^32)
//     (liquid nco_crcf_get_phase -> std::sin in stereo_decoder.cpp:251-256),
//     evaluated in double;
//   * sin of the exact phase 2 pi theta / 2^32;
// and the same errors of the output path's fmx_sincos_q on the float phase
// (what FMX_PLL_SIN_WORD=0 puts back on the chain).  Prints JSON.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "../../fmtuner-sdr_amd/csrc/fmx_math.h"

int main(int argc, char **argv) {
  const long long stride = (argc > 1) ? std::atoll(argv[1]) : 1;
  double e_word_ref = 0.0, e_word_exact = 0.0, e_q_ref = 0.0, e_q_exact = 0.0;
#pragma omp parallel for reduction(max : e_word_ref, e_word_exact, e_q_ref, e_q_exact) schedule(static)
  for (long long i = 0; i < (1LL << 32); i += stride) {
    const uint32_t th = (uint32_t)i;
    const float ph = (float)((double)(float)th * (6.283185307179586 / 4294967296.0));
    const double s_ref = std::sin((double)ph);
    const double s_exact = std::sin(6.283185307179586 * ((double)th / 4294967296.0));
    uint32_t sg;
    float w = pll_sin_word(th, &sg);
    if (sg) w = -w;
    const int qn = fmx_nco_quadrant(th);
    float sq, cq;
    fmx_sincos_q(ph, (float)qn, qn, &sq, &cq);
    e_word_ref = std::fmax(e_word_ref, std::fabs((double)w - s_ref));
    e_word_exact = std::fmax(e_word_exact, std::fabs((double)w - s_exact));
    e_q_ref = std::fmax(e_q_ref, std::fabs((double)sq - s_ref));
    e_q_exact = std::fmax(e_q_exact, std::fabs((double)sq - s_exact));
  }
  std::printf("{\"stride\": %lld, \"pll_sin_word_vs_float_phase\": %.3e, \"pll_sin_word_vs_exact\": %.3e, "
              "\"sincos_q_vs_float_phase\": %.3e, \"sincos_q_vs_exact\": %.3e}\n",
              stride, e_word_ref, e_word_exact, e_q_ref, e_q_exact);
  return 0;
}

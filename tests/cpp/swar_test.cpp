/* Exhaustive check of fmx_word_near_clip (fmtuner-sdr_amd/csrc/fmx_math.h),
 * the word-level pre-test that lets the front end skip the per-sample clip
 * counters of computeSignalLevel (signal_level.cpp:145-204): for every
 * 32-bit word it must be nonzero exactly when some byte is <= 8 or >= 247.
 * Prints the false-negative and false-positive counts (both must be 0). */
#include <cstdio>
#include <cstdint>
#include "../../fmtuner-sdr_amd/csrc/fmx_math.h"

int main(void) {
  long fneg = 0, fpos = 0;
#pragma omp parallel for reduction(+ : fneg, fpos) schedule(static)
  for (long x = 0; x < (1L << 32); ++x) {
    const uint32_t w = (uint32_t)x;
    int ex = 0;
    for (int k = 0; k < 4; ++k) {
      const unsigned b = (w >> (8 * k)) & 255u;
      if (b <= 8u || b >= 247u) ex = 1;
    }
    const int got = fmx_word_near_clip(w) != 0;
    fneg += ex && !got;
    fpos += !ex && got;
  }
  printf("{\"false_negatives\": %ld, \"false_positives\": %ld}\n", fneg, fpos);
  return 0;
}

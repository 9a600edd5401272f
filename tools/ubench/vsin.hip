// Accuracy of the hardware v_sin_f32 / v_cos_f32 (argument in revolutions)
// for NCO words: x = theta * 2^-32, against double sin(2 pi theta / 2^32),
// and of fmx_sincos on the float phase, over a sample of theta.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>
#include "../../fmtuner-sdr_amd/csrc/fmx_math.h"

__global__ void k(uint32_t step, float *hs, float *hc, float *ps, float *pc) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t theta = i * step;
  const float rev = (float)theta * 2.3283064365386963e-10f; // 2^-32
  hs[i] = __builtin_amdgcn_sinf(rev);
  hc[i] = __builtin_amdgcn_cosf(rev);
  const float ph = (float)((double)(float)theta * (6.283185307179586 / 4294967296.0));
  float s, c;
  fmx_sincos(ph, &s, &c);
  ps[i] = s;
  pc[i] = c;
}

int main() {
  const int N = 1 << 24;
  const uint32_t step = 257; // covers 2^32 / 257 ... a spread of words
  float *d[4];
  for (auto &p : d) hipMalloc(&p, N * 4);
  hipLaunchKernelGGL(k, dim3(N / 256), dim3(256), 0, 0, step, d[0], d[1], d[2], d[3]);
  float *h[4];
  for (int j = 0; j < 4; ++j) {
    h[j] = new float[N];
    hipMemcpy(h[j], d[j], N * 4, hipMemcpyDeviceToHost);
  }
  double mh = 0, mp = 0, mhr = 0;
  for (int i = 0; i < N; ++i) {
    const uint32_t theta = (uint32_t)i * step;
    const double ex = 6.283185307179586 * (double)theta / 4294967296.0;
    const float ph = (float)((double)(float)theta * (6.283185307179586 / 4294967296.0));
    const double s_ref = std::sin((double)ph), c_ref = std::cos((double)ph); // the reference's argument
    mh = std::fmax(mh, std::fmax(std::fabs(h[0][i] - s_ref), std::fabs(h[1][i] - c_ref)));
    mhr = std::fmax(mhr, std::fmax(std::fabs(h[0][i] - std::sin(ex)), std::fabs(h[1][i] - std::cos(ex))));
    mp = std::fmax(mp, std::fmax(std::fabs(h[2][i] - s_ref), std::fabs(h[3][i] - c_ref)));
  }
  printf("v_sin/v_cos vs sin(float phase): max abs %.3e (vs exact phase %.3e); fmx_sincos: %.3e\n", mh, mhr, mp);
  return 0;
}

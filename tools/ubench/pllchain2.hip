// Microbenchmark (round 2): ns per sample of k_pll's W0 feedback chain as it
// is now (pll_sin_word on the phase word) for one wave alone on its SIMD, and
// variants of its steps, to see which ones set the chain's latency.
//   0  reference constrain (trunc / compare / double add) + pll_sin_word
//   1  fmx_nco_constrain (floor; bit-identical, exhaustive host check)
//   2  1 with the double product replaced by a float pair product (timing only)
//   3  1 with an Estrin-form sine polynomial (timing only)
//   4  2 + 3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../../fmtuner-sdr_amd/csrc/fmx_math.h"

#define NS 8192

__device__ __forceinline__ uint32_t cons_pair(float x) { // float pair product (not exact)
  const float ch = 0.159154943091895f, cl = (float)(0.159154943091895 - (double)0.159154943091895f);
  const float ph = x * ch;
  const float e = fmaf(x, ch, -ph);
  const float p = ph + fmaf(x, cl, e);
  const float f = p - floorf(p);
  const uint32_t u = (uint32_t)(f * 4294967296.0f);
  return (f == 1.0f) ? 0u : u;
}
__device__ __forceinline__ float sin_estrin(uint32_t theta, uint32_t *sg) {
  const uint32_t s = (theta + 0x40000000u) & 0x80000000u;
  const float r = (float)(int32_t)(theta ^ s) * 1.4629180792671596e-09f;
  const float z = r * r;
  const float z2 = z * z;
  const float a = fmaf(z, 2.6083159809786593541503e-06f, -0.0001981069071916863322258f);
  const float b = fmaf(z, 0.00833307858556509017944336f, -0.166666597127914428710938f);
  const float u = fmaf(z2, a, b);
  *sg = s;
  return fmaf(z * r, u, r);
}

template <int V>
__global__ void k(const float *pilot, unsigned long long *out, float *sink) {
  uint32_t theta = threadIdx.x * 7919u, dtheta = 123456789u;
  const float alpha = 1e-3f, beta = 3e-2f;
  uint32_t vsg = 0;
  float vq = 0.1f;
  uint32_t acc = 0;
  const float pv0 = pilot[threadIdx.x];
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int t = 0; t < NS; ++t) {
    const float pv = pv0 + (float)(t & 7);
    const float err = __uint_as_float(__float_as_uint(pv) ^ vsg) * vq;
    if constexpr (V == 0) {
      dtheta += fmx_nco_constrain_ref(err * alpha);
      theta += fmx_nco_constrain_ref(err * beta);
    } else if constexpr (V == 2 || V == 4) {
      dtheta += cons_pair(err * alpha);
      theta += cons_pair(err * beta);
    } else {
      dtheta += fmx_nco_constrain(err * alpha);
      theta += fmx_nco_constrain(err * beta);
    }
    theta += dtheta;
    if constexpr (V == 3 || V == 4) vq = sin_estrin(theta, &vsg);
    else vq = pll_sin_word(theta, &vsg);
    acc ^= theta;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  sink[blockIdx.x * 64 + threadIdx.x] = vq + (float)acc;
}

int main() {
  float *pilot, *sink;
  unsigned long long *out;
  hipMalloc(&pilot, 64 * 4);
  hipMemset(pilot, 0, 64 * 4);
  hipMalloc(&sink, 64 * 64 * 4);
  hipMalloc(&out, 64 * 8);
  const char *names[] = {"reference constrain + pll_sin_word", "floor constrain (exact)",
                         "floor + float pair product", "floor + Estrin sine", "pair product + Estrin"};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int v = 0; v < 5; ++v) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      if (v == 0) hipLaunchKernelGGL(k<0>, dim3(64), dim3(64), 0, 0, pilot, out, sink);
      if (v == 1) hipLaunchKernelGGL(k<1>, dim3(64), dim3(64), 0, 0, pilot, out, sink);
      if (v == 2) hipLaunchKernelGGL(k<2>, dim3(64), dim3(64), 0, 0, pilot, out, sink);
      if (v == 3) hipLaunchKernelGGL(k<3>, dim3(64), dim3(64), 0, 0, pilot, out, sink);
      if (v == 4) hipLaunchKernelGGL(k<4>, dim3(64), dim3(64), 0, 0, pilot, out, sink);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    unsigned long long h[64];
    hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
    printf("%-40s %7.2f ticks/sample  %7.2f ns/sample (wall)\n", names[v], (double)h[0] / NS, best * 1e6 / NS);
  }
  return 0;
}

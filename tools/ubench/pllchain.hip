// Microbenchmark: cycles per sample of the stereo PLL feedback chain (k_pll
// wave W0: error, two NCO constrains, phase, sincos) for one wave alone on
// its SIMD, and of its parts, to see where the chain's latency goes.
// Variants (not bit-exact, timing only) replace the double-precision steps.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../../fmtuner-sdr_amd/csrc/fmx_math.h"

#define NS 4096

__device__ __forceinline__ uint32_t cons_d(float x) {
  const float p = (float)((double)x * 0.159154943091895);
  float fpart = p - truncf(p);
  if (fpart < 0.0f) fpart = (float)((double)fpart + 1.0);
  const float s = fpart * 4294967296.0f;
  return (s >= 4294967296.0f) ? 0u : (uint32_t)s;
}
__device__ __forceinline__ uint32_t cons_f(float x) { // float-only (timing)
  const float p = x * 0.159154943091895f;
  float fpart = p - truncf(p);
  fpart = fpart < 0.0f ? fpart + 1.0f : fpart;
  const float s = fpart * 4294967296.0f;
  return (s >= 4294967296.0f) ? 0u : (uint32_t)s;
}
__device__ __forceinline__ float phase_d(uint32_t theta) {
  return (float)((double)(float)theta * (6.283185307179586 / 4294967296.0));
}
__device__ __forceinline__ float phase_f(uint32_t theta) { return (float)theta * 1.4629180792671596e-09f; }
__device__ __forceinline__ uint32_t cons_d1(float x) { // double product, float +1 (exact equivalent)
  const float p = (float)((double)x * 0.159154943091895);
  float fpart = p - truncf(p);
  fpart = fpart < 0.0f ? fpart + 1.0f : fpart;
  const float s = fpart * 4294967296.0f;
  return (s >= 4294967296.0f) ? 0u : (uint32_t)s;
}
// sincos with the quadrant taken from the NCO word (exact quadrant of the
// exact phase; the float phase is within 0.5 ulp of it)
__device__ __forceinline__ void sincos_q(float x, uint32_t theta, float *s, float *c) {
  const uint32_t qi = (theta + 0x20000000u) >> 30;
  const float q = (float)qi;
  const float r1 = fmaf(-q, 1.57079637050628662109375f, x);
  const float rh = fmaf(-q, -4.3711388286737929e-08f, r1);
  float rl = fmaf(-q, -4.3711388286737929e-08f, r1 - rh);
  rl = fmaf(-q, -1.7151245100058819e-15f, rl);
  const float z = rh * rh;
  float ps = fmaf(z, 2.6083159809786593541503e-06f, -0.0001981069071916863322258f);
  ps = fmaf(z, ps, 0.00833307858556509017944336f);
  ps = fmaf(z, ps, -0.166666597127914428710938f);
  const float sr = rh + fmaf(rh * z, ps, rl);
  float pc = fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f);
  pc = fmaf(z, pc, 4.166664568298827e-2f);
  const float hz = 0.5f * z;
  const float w = 1.0f - hz;
  const float tail = (1.0f - w) - hz;
  const float cr = w + (fmaf(z * z, pc, tail) - rh * rl);
  const bool swap = (qi & 1) != 0;
  const float s0 = swap ? cr : sr;
  const float c0 = swap ? sr : cr;
  *s = (qi & 2) ? -s0 : s0;
  *c = ((qi + 1) & 2) ? -c0 : c0;
}

template <int V>
__global__ void k(const float *pilot, unsigned long long *out, float *sink) {
  uint32_t theta = threadIdx.x * 7919u, dtheta = 123456789u;
  const float alpha = 1e-3f, beta = 3e-2f;
  float vq = 0.1f, acc = 0.0f;
  const float pv = pilot[threadIdx.x];
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int t = 0; t < NS; ++t) {
    const float err = (pv + (float)(t & 7)) * vq;
    if constexpr (V == 0 || V == 3) { // full chain, double steps
      dtheta += cons_d(err * alpha);
      theta += cons_d(err * beta);
    } else if constexpr (V >= 4) {
      dtheta += cons_d1(err * alpha);
      theta += cons_d1(err * beta);
    } else {
      dtheta += cons_f(err * alpha);
      theta += cons_f(err * beta);
    }
    theta += dtheta;
    float ph;
    if constexpr (V == 0 || V == 2 || V >= 4) ph = phase_d(theta);
    else ph = phase_f(theta);
    if constexpr (V == 3) { // no sincos: the NCO part alone
      vq = ph * 1e-3f;
    } else if constexpr (V == 5) {
      float s, c;
      sincos_q(ph, theta, &s, &c);
      vq = s;
      acc += c;
    } else {
      float s, c;
      fmx_sincos(ph, &s, &c);
      vq = s;
      acc += c;
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  sink[blockIdx.x * 64 + threadIdx.x] = vq + acc + (float)theta;
}

int main() {
  float *pilot, *sink;
  unsigned long long *out;
  hipMalloc(&pilot, 64 * 4);
  hipMemset(pilot, 0, 64 * 4);
  hipMalloc(&sink, 64 * 64 * 4);
  hipMalloc(&out, 64 * 8);
  const char *names[] = {"full chain (double NCO steps)", "float constrain + float phase",
                         "float constrain, double phase", "NCO only (double), no sincos",
                         "float +1 in constrain (exact)", "float +1, quadrant from theta"};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int v = 0; v < 6; ++v) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      if (v == 0) hipLaunchKernelGGL(k<0>, dim3(64), dim3(64), 0, 0, pilot, out, sink);
      if (v == 1) hipLaunchKernelGGL(k<1>, dim3(64), dim3(64), 0, 0, pilot, out, sink);
      if (v == 2) hipLaunchKernelGGL(k<2>, dim3(64), dim3(64), 0, 0, pilot, out, sink);
      if (v == 3) hipLaunchKernelGGL(k<3>, dim3(64), dim3(64), 0, 0, pilot, out, sink);
      if (v == 4) hipLaunchKernelGGL(k<4>, dim3(64), dim3(64), 0, 0, pilot, out, sink);
      if (v == 5) hipLaunchKernelGGL(k<5>, dim3(64), dim3(64), 0, 0, pilot, out, sink);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
    }
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[64];
    hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
    printf("%-36s %7.1f ticks/sample  %7.1f ns/sample (wall)\n", names[v], (double)h[0] / NS, ms * 1e6 / NS);
  }
  return 0;
}

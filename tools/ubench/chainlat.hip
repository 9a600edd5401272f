// Microbenchmark for the k_pll W0 chain (stereo_decoder.cpp:178-192 as k_pll
// restates it): dependent-issue latency of each instruction kind on the
// chain, one wave64 alone on its SIMD, and cycles per sample of the whole
// PLL feedback iteration in its current and candidate forms.
//   hipcc --offload-arch=gfx950 -O3 chainlat.hip -o chainlat && ./chainlat
// Ticks are s_memtime (shader clock).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include "../../fmtuner-sdr_amd/csrc/fmx_math.h"

#define NREP 1024

// ---- single-op dependent chains (8 ops per iteration, NREP iterations) ----
#define CHAIN8(stmt) stmt; stmt; stmt; stmt; stmt; stmt; stmt; stmt;
template <int OP>
__global__ void k_op(const float *in, unsigned long long *out, float *sink) {
  float x = in[threadIdx.x];
  double d = (double)x;
  uint32_t u = __float_as_uint(x);
  const float c1 = in[64], c2 = in[65];
  const uint32_t cu = __float_as_uint(in[66]);
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < NREP; ++r) {
    if constexpr (OP == 0) { CHAIN8(x = x + c1) }
    if constexpr (OP == 1) { CHAIN8(x = fmaf(x, c1, c2)) }
    if constexpr (OP == 2) { CHAIN8(x = x * c1) }
    if constexpr (OP == 3) { CHAIN8(d = d * (double)c1) }
    if constexpr (OP == 4) { CHAIN8(x = (float)((double)x * 0.159154943091895)) }  // cvt, mul_f64, cvt
    if constexpr (OP == 5) { CHAIN8(x = floorf(x) + c1) }
    if constexpr (OP == 6) { CHAIN8(x = __builtin_amdgcn_fractf(x) + c1) }
    if constexpr (OP == 7) { CHAIN8(u = (uint32_t)((float)u * c1)) }               // cvt_f32_u32, mul, cvt_u32_f32
    if constexpr (OP == 8) { CHAIN8(x = __builtin_amdgcn_sinf(x)) }
    if constexpr (OP == 9) { CHAIN8(u = u + cu) }
    if constexpr (OP == 10) { CHAIN8(u = (u ^ cu) + 1u) }
    if constexpr (OP == 11) { CHAIN8(x = (x > c1) ? x * c2 : x + c2) }           // cmp + cndmask (+ the two)
    if constexpr (OP == 12) { CHAIN8(x = __builtin_amdgcn_sinf(x) * c1) }          // trans -> VALU
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  sink[threadIdx.x] = x + (float)d + (float)u;
}

// ---- the W0 PLL feedback iteration ----
// R4: the round-4 k_pll chain: per sample two products pilot k 2^32 vcoQ,
//     two truncating converts, add3, and v_sin of (float)(int32)theta 2^-32
// R5: the round-5 chain (fmx_chain_words / fmx_chain_sin): one packed
//     multiply, two converts, add3, v_alignbit_b32 and v_sin
template <int V>
__global__ void k_pll(const float *pilot, unsigned long long *out, float *sink) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  uint32_t theta = threadIdx.x * 7919u, dtheta = 123456789u;
  const float ka = 1e-2f * 0.159154943091895f, kb = 0.1f * 0.159154943091895f;
  const float kaw = ka * 4294967296.0f, kbw = kb * 4294967296.0f;
  float pv[8];
  for (int i = 0; i < 8; ++i) pv[i] = pilot[(threadIdx.x + i) & 63];
  float s = fmx_chain_sin(theta);
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < NREP; ++r) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      uint32_t ca, cb;
      if constexpr (V == 0) {
        ca = (uint32_t)(int32_t)(pv[i] * kaw * s);
        cb = (uint32_t)(int32_t)(pv[i] * kbw * s);
      } else {
        const f2 pab = f2{pv[i], pv[i]} * f2{kaw, kbw};
        fmx_chain_words(pab.x, pab.y, s, &ca, &cb);
      }
      const uint32_t T = theta + dtheta;
      dtheta += ca;
      theta = T + ca + cb;
      if constexpr (V == 0) s = __builtin_amdgcn_sinf((float)(int32_t)theta * 2.3283064365386963e-10f);
      else s = fmx_chain_sin(theta);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  sink[blockIdx.x * 64 + threadIdx.x] = s + (float)theta + (float)dtheta;
}

template <typename K> static double run(K kern, const float *in, unsigned long long *out, float *sink, int per) {
  unsigned long long h[8];
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(kern, dim3(8), dim3(64), 0, 0, in, out, sink);
    hipDeviceSynchronize();
  }
  hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < 8; ++i) m += (double)h[i];
  return m / 8.0 / ((double)NREP * per);
}

int main() {
  float *in, *sink;
  unsigned long long *out;
  hipMalloc(&in, 128 * 4);
  hipMalloc(&sink, 8 * 64 * 4);
  hipMalloc(&out, 8 * 8);
  float hin[128];
  for (int i = 0; i < 128; ++i) hin[i] = 0.01f * (float)(i % 17) - 0.05f;
  hin[64] = 1.0001f;
  hin[65] = 1e-7f;
  hin[66] = 1.0f;
  hipMemcpy(in, hin, sizeof(hin), hipMemcpyHostToDevice);
  const char *ops[] = {"v_add_f32", "v_fma_f32", "v_mul_f32", "v_mul_f64", "cvt_f64 + mul_f64 + cvt_f32",
                       "v_floor_f32 + v_add_f32", "v_fract_f32 + v_add_f32", "cvt_f32_u32 + mul + cvt_u32_f32",
                       "v_sin_f32", "v_add_u32", "v_xor_b32 + v_add_u32", "cmp + cndmask (+mul/add)",
                       "v_sin_f32 + v_mul_f32"};
  printf("dependent chain, one wave per SIMD, ticks per op (group)\n");
  printf("%-34s %7.2f\n", ops[0], run(k_op<0>, in, out, sink, 8));
  printf("%-34s %7.2f\n", ops[1], run(k_op<1>, in, out, sink, 8));
  printf("%-34s %7.2f\n", ops[2], run(k_op<2>, in, out, sink, 8));
  printf("%-34s %7.2f\n", ops[3], run(k_op<3>, in, out, sink, 8));
  printf("%-34s %7.2f\n", ops[4], run(k_op<4>, in, out, sink, 8));
  printf("%-34s %7.2f\n", ops[5], run(k_op<5>, in, out, sink, 8));
  printf("%-34s %7.2f\n", ops[6], run(k_op<6>, in, out, sink, 8));
  printf("%-34s %7.2f\n", ops[7], run(k_op<7>, in, out, sink, 8));
  printf("%-34s %7.2f\n", ops[8], run(k_op<8>, in, out, sink, 8));
  printf("%-34s %7.2f\n", ops[9], run(k_op<9>, in, out, sink, 8));
  printf("%-34s %7.2f\n", ops[10], run(k_op<10>, in, out, sink, 8));
  printf("%-34s %7.2f\n", ops[11], run(k_op<11>, in, out, sink, 8));
  printf("%-34s %7.2f\n", ops[12], run(k_op<12>, in, out, sink, 8));
  const char *vs[] = {"R4 cvt+mul+sin word sine", "R5 pk_mul + alignbit + sin"};
  printf("PLL feedback iteration, ticks per sample\n");
  printf("%-34s %7.2f\n", vs[0], run(k_pll<0>, in, out, sink, 8));
  printf("%-34s %7.2f\n", vs[1], run(k_pll<1>, in, out, sink, 8));
  return 0;
}

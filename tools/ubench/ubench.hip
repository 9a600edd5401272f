// Microbenchmark: issue cost (cycles per instruction) of the VALU forms the
// serial kernels (k_rds, k_pll) are made of, for ONE wave alone on its SIMD.
// Each test runs N iterations of 8 independent (or dependent) instructions
// in inline asm between s_memtime reads.
#include <hip/hip_runtime.h>
#include <cstdio>

#define N 1024
#define BODY8(INS) INS INS INS INS INS INS INS INS

template <int K>
__global__ void kb(unsigned long long *out, float *sink) {
  float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  double d0 = a0, d1 = a1, d2 = a2, d3 = a3;
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7};
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; ++i) {
    if constexpr (K == 0) { // independent v_fma_f32
      asm volatile("v_fma_f32 %0, %0, %0, %0\n v_fma_f32 %1, %1, %1, %1\n v_fma_f32 %2, %2, %2, %2\n v_fma_f32 %3, %3, %3, %3\n"
                   "v_fma_f32 %4, %4, %4, %4\n v_fma_f32 %5, %5, %5, %5\n v_fma_f32 %6, %6, %6, %6\n v_fma_f32 %7, %7, %7, %7\n"
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    } else if constexpr (K == 1) { // dependent v_fma_f32 chain
      asm volatile(BODY8("v_fma_f32 %0, %0, %0, %0\n") : "+v"(a0));
    } else if constexpr (K == 2) { // independent v_pk_fma_f32
      asm volatile("v_pk_fma_f32 %0, %0, %0, %0\n v_pk_fma_f32 %1, %1, %1, %1\n v_pk_fma_f32 %2, %2, %2, %2\n v_pk_fma_f32 %3, %3, %3, %3\n"
                   "v_pk_fma_f32 %0, %0, %0, %0\n v_pk_fma_f32 %1, %1, %1, %1\n v_pk_fma_f32 %2, %2, %2, %2\n v_pk_fma_f32 %3, %3, %3, %3\n"
                   : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3));
    } else if constexpr (K == 3) { // dependent v_pk_add_f32
      asm volatile(BODY8("v_pk_add_f32 %0, %0, %0\n") : "+v"(p0));
    } else if constexpr (K == 4) { // independent v_pk_add_f32
      asm volatile("v_pk_add_f32 %0, %0, %0\n v_pk_add_f32 %1, %1, %1\n v_pk_add_f32 %2, %2, %2\n v_pk_add_f32 %3, %3, %3\n"
                   "v_pk_add_f32 %0, %0, %0\n v_pk_add_f32 %1, %1, %1\n v_pk_add_f32 %2, %2, %2\n v_pk_add_f32 %3, %3, %3\n"
                   : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3));
    } else if constexpr (K == 5) { // independent v_mul_f64
      asm volatile("v_mul_f64 %0, %0, %0\n v_mul_f64 %1, %1, %1\n v_mul_f64 %2, %2, %2\n v_mul_f64 %3, %3, %3\n"
                   "v_mul_f64 %0, %0, %0\n v_mul_f64 %1, %1, %1\n v_mul_f64 %2, %2, %2\n v_mul_f64 %3, %3, %3\n"
                   : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3));
    } else if constexpr (K == 6) { // independent v_cvt_f64_f32
      asm volatile("v_cvt_f64_f32 %0, %4\n v_cvt_f64_f32 %1, %5\n v_cvt_f64_f32 %2, %6\n v_cvt_f64_f32 %3, %7\n"
                   "v_cvt_f64_f32 %0, %4\n v_cvt_f64_f32 %1, %5\n v_cvt_f64_f32 %2, %6\n v_cvt_f64_f32 %3, %7\n"
                   : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3) : "v"(a0), "v"(a1), "v"(a2), "v"(a3));
    } else if constexpr (K == 7) { // independent v_cndmask with vcc
      asm volatile("v_cmp_gt_f32 vcc, %0, %1\n v_cndmask_b32 %2, %2, %3, vcc\n v_cndmask_b32 %3, %3, %4, vcc\n v_cndmask_b32 %4, %4, %5, vcc\n"
                   "v_cndmask_b32 %5, %5, %6, vcc\n v_cndmask_b32 %6, %6, %7, vcc\n v_cndmask_b32 %7, %7, %2, vcc\n v_cndmask_b32 %0, %0, %1, vcc\n"
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) :: "vcc");
    } else if constexpr (K == 8) { // independent v_sin_f32 (transcendental)
      asm volatile("v_sin_f32 %0, %0\n v_sin_f32 %1, %1\n v_sin_f32 %2, %2\n v_sin_f32 %3, %3\n"
                   "v_sin_f32 %4, %4\n v_sin_f32 %5, %5\n v_sin_f32 %6, %6\n v_sin_f32 %7, %7\n"
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    } else if constexpr (K == 9) { // independent v_mul_f32
      asm volatile("v_mul_f32 %0, %0, %0\n v_mul_f32 %1, %1, %1\n v_mul_f32 %2, %2, %2\n v_mul_f32 %3, %3, %3\n"
                   "v_mul_f32 %4, %4, %4\n v_mul_f32 %5, %5, %5\n v_mul_f32 %6, %6, %6\n v_mul_f32 %7, %7, %7\n"
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[K] = t1 - t0;
  sink[threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + (float)(d0 + d1 + d2 + d3) + p0.x + p1.x + p2.y + p3.y;
}

int main() {
  unsigned long long *d, h[16] = {0};
  float *s;
  hipMalloc(&d, sizeof(h));
  hipMalloc(&s, 1024 * 4);
  hipMemset(d, 0, sizeof(h));
  const char *names[] = {"v_fma_f32 indep", "v_fma_f32 dep", "v_pk_fma_f32 indep", "v_pk_add_f32 dep",
                         "v_pk_add_f32 indep", "v_mul_f64 indep", "v_cvt_f64_f32 indep", "v_cmp+v_cndmask",
                         "v_sin_f32 indep", "v_mul_f32 indep"};
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(kb<0>, 1, 64, 0, 0, d, s);
    hipLaunchKernelGGL(kb<1>, 1, 64, 0, 0, d, s);
    hipLaunchKernelGGL(kb<2>, 1, 64, 0, 0, d, s);
    hipLaunchKernelGGL(kb<3>, 1, 64, 0, 0, d, s);
    hipLaunchKernelGGL(kb<4>, 1, 64, 0, 0, d, s);
    hipLaunchKernelGGL(kb<5>, 1, 64, 0, 0, d, s);
    hipLaunchKernelGGL(kb<6>, 1, 64, 0, 0, d, s);
    hipLaunchKernelGGL(kb<7>, 1, 64, 0, 0, d, s);
    hipLaunchKernelGGL(kb<8>, 1, 64, 0, 0, d, s);
    hipLaunchKernelGGL(kb<9>, 1, 64, 0, 0, d, s);
    hipDeviceSynchronize();
  }
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int k = 0; k < 10; ++k) printf("%-22s %6.2f cycles/instr\n", names[k], (double)h[k] / (8.0 * N));
  return 0;
}

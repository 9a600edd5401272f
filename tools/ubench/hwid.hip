// Which SIMD does each wave of a workgroup land on?  Prints, for a few
// workgroups of W waves, the SIMD id (HW_ID bits 5:4) and CU id of every wave.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void probe(unsigned *out) {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(v));
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 16 + (threadIdx.x >> 6)] = v;
}
int main() {
  unsigned *d;
  hipMalloc(&d, 64 * 16 * 4);
  for (int w : {5, 6, 8}) {
    hipMemset(d, 0, 64 * 16 * 4);
    hipLaunchKernelGGL(probe, dim3(64), dim3(64 * w), 0, 0, d);
    unsigned h[64 * 16];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    for (int b = 0; b < 4; ++b) {
      printf("waves=%d wg=%d:", w, b);
      for (int k = 0; k < w; ++k) {
        unsigned v = h[b * 16 + k];
        printf(" w%d:simd%u/cu%u/wid%u", k, (v >> 4) & 3, (v >> 8) & 15, v & 15);
      }
      printf("\n");
    }
  }
  return 0;
}

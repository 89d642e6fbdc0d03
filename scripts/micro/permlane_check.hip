// Prints what __builtin_amdgcn_permlane32_swap(x, x) returns in lanes 0 and 32 (x = lane id).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
  unsigned x = threadIdx.x;
  auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  out[threadIdx.x] = r[0];
  out[64 + threadIdx.x] = r[1];
}
int main() {
  unsigned* d; hipMalloc(&d, 128 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  unsigned h[128]; hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
  printf("lane0: r0=%u r1=%u ; lane32: r0=%u r1=%u ; lane5: r0=%u r1=%u\n", h[0], h[64], h[32], h[96], h[5], h[69]);
  return 0;
}

// Cost of a grid-wide barrier between a few co-resident workgroups (the candidate replacement
// for __syncthreads() if the single-workgroup moving-mesh kernels were split over G workgroups).
// G participating blocks of 1024 threads: either all on one XCD (launch 8 G blocks, blocks
// b % 8 == 0 take part -- consecutive workgroups are dealt round-robin over the 8 XCDs) or
// spread (G blocks, one per XCD in turn).  Each barrier: __threadfence (agent release), one
// atomic arrival per block, the last arrival bumps a generation word, the others poll it
// (bounded: a poll budget, then the error word), __threadfence (acquire).
//   hipcc --offload-arch=gfx950 -O3 gridbar_bench.hip -o gridbar_bench && ./gridbar_bench
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void __launch_bounds__(1024) bar_kernel(unsigned* cnt, unsigned* gen, int* err,
                                                   int iters, int G, int stride) {
  if (blockIdx.x % stride != 0) return;
  for (int it = 0; it < iters; ++it) {
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned target = unsigned(it + 1);
      if (atomicAdd(cnt, 1u) == unsigned(G) - 1) {
        atomicExch(cnt, 0u);
        __hip_atomic_store(gen, target, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        long n = 0;
        while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
          if (++n > (1l << 24)) {
            atomicExch(err, 1);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
    }
    __syncthreads();
    __threadfence();
  }
}

int main() {
  unsigned *cnt, *gen;
  int* err;
  hipMalloc(&cnt, 4);
  hipMalloc(&gen, 4);
  hipMalloc(&err, 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 2000;
  for (int G : {2, 4, 8, 16, 32}) {
    for (int local = 1; local >= 0; --local) {
      const int stride = local ? 8 : 1;
      hipMemset(cnt, 0, 4);
      hipMemset(gen, 0, 4);
      hipMemset(err, 0, 4);
      hipLaunchKernelGGL(bar_kernel, dim3(G * stride), dim3(1024), 0, 0, cnt, gen, err, 10, G,
                         stride);  // warm
      hipMemset(gen, 0, 4);
      hipDeviceSynchronize();
      hipEventRecord(a);
      hipLaunchKernelGGL(bar_kernel, dim3(G * stride), dim3(1024), 0, 0, cnt, gen, err, iters, G,
                         stride);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      int e = 0;
      hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
      printf("G=%2d %s: %.2f us per barrier%s\n", G, local ? "one XCD " : "spread  ",
             1e3 * ms / iters, e ? "  (poll budget exhausted!)" : "");
    }
  }
  return 0;
}

// Streaming-copy ceiling of this chip (round 5): variants of a fp64 device-to-device copy
// (16 B per lane per load), for the bench's copy_bandwidth normaliser and the load shape of the
// streaming kernels.  Variants: loads in flight per thread (U), block size, grid = one chunk per
// block or a persistent grid-stride loop, non-temporal or default policy, and the gap between
// source and destination (a multiple of 2^27 B or skewed by 128 KiB).  Each variant: 20 launches
// back to back (events around all: includes the launch gaps) and 20 launches each between its
// own event pair (kernel + event, no gap).
// Build: hipcc -O3 --offload-arch=gfx950 copy_bench.hip -o copy_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef double dv2 __attribute__((ext_vector_type(2)));

template <int U, bool NT>
__global__ void chunked(const dv2* __restrict__ s, dv2* __restrict__ d, long n2) {
  const long base = long(blockIdx.x) * blockDim.x * U + threadIdx.x;
  dv2 v[U];
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const long i = base + long(k) * blockDim.x;
    if (i < n2) v[k] = NT ? __builtin_nontemporal_load(s + i) : s[i];
  }
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const long i = base + long(k) * blockDim.x;
    if (i < n2) {
      if (NT) __builtin_nontemporal_store(v[k], d + i); else d[i] = v[k];
    }
  }
}

template <int U, bool NT>
__global__ void persistent(const dv2* __restrict__ s, dv2* __restrict__ d, long n2) {
  const long step = long(gridDim.x) * blockDim.x * U;
  for (long base = long(blockIdx.x) * blockDim.x * U + threadIdx.x; base < n2; base += step) {
    dv2 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const long i = base + long(k) * blockDim.x;
      if (i < n2) v[k] = NT ? __builtin_nontemporal_load(s + i) : s[i];
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const long i = base + long(k) * blockDim.x;
      if (i < n2) {
        if (NT) __builtin_nontemporal_store(v[k], d + i); else d[i] = v[k];
      }
    }
  }
}

struct Res { float all_us, each_us; };
template <typename F>
Res timeit(F f, int reps = 20) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) f(i);
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f(i);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  float tot = 0;
  for (int i = 0; i < reps; ++i) {
    CK(hipEventRecord(a)); f(i); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float m; CK(hipEventElapsedTime(&m, a, b)); tot += m;
  }
  CK(hipGetLastError());
  return {ms * 1e3f / reps, tot * 1e3f / reps};
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 4096L * 4096L;  // doubles per copy
  int ncu = 0; CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  for (long skew : {0L, 16384L}) {  // doubles: 0 or 128 KiB between consecutive buffers
    const long stride = (n + 32767) / 32768 * 32768 + skew;
    double* pool; CK(hipMalloc(&pool, stride * 8 * 4));
    CK(hipMemset(pool, 0, stride * 8 * 4));
    const dv2* src[2] = {(const dv2*)pool, (const dv2*)(pool + 2 * stride)};
    dv2* dst[2] = {(dv2*)(pool + stride), (dv2*)(pool + 3 * stride)};
    const long n2 = n / 2;
    const double bytes = 16.0 * n;
    auto rep = [&](const char* name, Res r) {
      printf("skew%-6ld %-28s all %8.2f us %6.0f GB/s | each %8.2f us %6.0f GB/s\n", skew, name,
             r.all_us, bytes / r.all_us / 1e3, r.each_us, bytes / r.each_us / 1e3);
    };
#define CH(U, NT, B) rep("chunked U" #U " NT" #NT " B" #B, timeit([&](int i) { \
      hipLaunchKernelGGL((chunked<U, NT>), dim3(unsigned((n2 + long(B) * U - 1) / (long(B) * U))), dim3(B), 0, 0, src[i & 1], dst[i & 1], n2); }))
#define PE(U, NT, B, BPC) rep("persist U" #U " NT" #NT " B" #B " x" #BPC, timeit([&](int i) { \
      hipLaunchKernelGGL((persistent<U, NT>), dim3(unsigned(ncu * BPC)), dim3(B), 0, 0, src[i & 1], dst[i & 1], n2); }))
    CH(4, true, 256); CH(4, false, 256); CH(8, true, 256); CH(2, true, 256); CH(4, true, 512);
    CH(8, true, 512); CH(16, true, 256); CH(4, true, 1024);
    PE(4, true, 256, 8); PE(8, true, 256, 8); PE(4, true, 512, 4); PE(4, true, 256, 16);
    PE(8, true, 512, 4); PE(4, false, 256, 8); PE(2, true, 1024, 2);
    CK(hipFree(pool));
  }
  return 0;
}

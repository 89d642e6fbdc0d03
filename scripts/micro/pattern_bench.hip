// Access-pattern microbenchmark for the fused Arnoldi kernel: K fp64 vectors of N x N, each wave
// marches down a band of rows reading one row segment of every vector per step, summing into
// registers and writing one row of output.  Variants: segment width / alignment / bytes per lane.
// Build: hipcc -O3 --offload-arch=gfx950 pattern_bench.hip -o pattern_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int KMAX = 16;
typedef double dv2 __attribute__((ext_vector_type(2)));
struct Args { const double* v[KMAX]; double* out; int K; long nx, ny; int strips, nbands, RY, SW, W; };

// W = columns per lane (1: dwordx2, 2: dwordx4); SW = owned columns per wave (loads 64*W)
template <int W, int K>
__global__ void __launch_bounds__(256) march(Args A) {
  const int lane = threadIdx.x & 63;
  const long gw = long(blockIdx.x) * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (gw >= long(A.strips) * A.nbands) return;
  const long band = gw / A.strips, strip = gw % A.strips;
  long c = strip * A.SW + lane * W - (64 * W - A.SW) / 2;
  c = c < 0 ? c + A.nx : (c >= A.nx ? c - A.nx : c);
  const long r0 = band * A.RY;
  const long r1 = r0 + A.RY < A.ny ? r0 + A.RY : A.ny;
  double acc[W] = {};
  for (long r = r0; r < r1; ++r) {
    const long o = r * A.nx + c;
#pragma unroll
    for (int i = 0; i < K; ++i) {
      if constexpr (W == 2) {
        const dv2 x = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(A.v[i] + o));
        acc[0] += x.x; acc[1] += x.y;
      } else {
        acc[0] += __builtin_nontemporal_load(A.v[i] + o);
      }
    }
    if constexpr (W == 2) *reinterpret_cast<double2*>(A.out + o) = make_double2(acc[0], acc[1]);
    else A.out[o] = acc[0];
  }
}

// contiguous chunks (the Krylov kernels' pattern): block b reads chunk b of every vector
template <int K>
__global__ void __launch_bounds__(256) chunk(Args A, long n, int cpb) {
  double acc[8] = {};
  for (int cc = 0; cc < cpb; ++cc) {
    const long base = (long(blockIdx.x) * cpb + cc) * 2048 + 2 * threadIdx.x;
    if (base >= n) break;
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const dv2 x = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(A.v[i] + base + k * 512));
        acc[2 * k] += x.x; acc[2 * k + 1] += x.y;
      }
#pragma unroll
    for (int k = 0; k < 4; ++k) *reinterpret_cast<double2*>(A.out + base + k * 512) = make_double2(acc[2 * k], acc[2 * k + 1]);
  }
}

template <int W, int K>
float run_march(Args A, int waves_target, int SW) {
  A.SW = SW;
  A.strips = (A.nx + SW - 1) / SW;
  A.nbands = waves_target / A.strips; if (A.nbands < 1) A.nbands = 1;
  A.RY = (A.ny + A.nbands - 1) / A.nbands; A.nbands = (A.ny + A.RY - 1) / A.RY;
  long nw = long(A.strips) * A.nbands;
  dim3 g((nw + 3) / 4);
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((march<W, K>), g, dim3(256), 0, 0, A);
  CK(hipEventRecord(a));
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL((march<W, K>), g, dim3(256), 0, 0, A);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / 10;
}

template <int K>
float run_chunk(Args A) {
  long n = A.nx * A.ny;
  long chunks = (n + 2047) / 2048; int cpb = (chunks + 4095) / 4096;
  dim3 g((chunks + cpb - 1) / cpb);
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((chunk<K>), g, dim3(256), 0, 0, A, n, cpb);
  CK(hipEventRecord(a));
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL((chunk<K>), g, dim3(256), 0, 0, A, n, cpb);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / 10;
}

int main() {
  const long N = 4096, n = N * N;
  Args A{};
  A.nx = N; A.ny = N;
  for (int i = 0; i < KMAX; ++i) { double* p; CK(hipMalloc(&p, n * 8)); CK(hipMemset(p, 0, n * 8)); A.v[i] = p; }
  CK(hipMalloc(&A.out, n * 8));
  constexpr int K = 8;
  const double bytes = 8.0 * n * (K + 1);
  auto rep = [&](const char* name, float ms) { printf("%-40s %8.1f us  %7.1f GB/s  %.3f\n", name, ms * 1e3, bytes / ms / 1e6, bytes / ms / 1e6 / 8000); };
  rep("chunk 16KB (krylov pattern)", run_chunk<K>(A));
  for (int w : {1024, 2048, 4096, 8192}) {
    char nm[64];
    snprintf(nm, 64, "march W1 SW60 waves %d", w); rep(nm, run_march<1, K>(A, w, 60));
    snprintf(nm, 64, "march W1 SW64 waves %d", w); rep(nm, run_march<1, K>(A, w, 64));
    snprintf(nm, 64, "march W2 SW124 waves %d", w); rep(nm, run_march<2, K>(A, w, 124));
    snprintf(nm, 64, "march W2 SW128 waves %d", w); rep(nm, run_march<2, K>(A, w, 128));
  }
  return 0;
}

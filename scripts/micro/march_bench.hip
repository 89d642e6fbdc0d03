// Streaming-pattern ceiling for the fused Arnoldi kernel: K fp64 input vectors of N x N and one
// output, each wave marching down a band of rows with PF rows of loads in flight (register ring,
// as arnoldi.hip does), against the contiguous-chunk pattern of the Krylov kernels.  Variants:
// columns per lane (W), rows in flight (PF), a block barrier per row (BAR), waves per block,
// band height, occupancy.  Prints GB/s of algorithmic bytes 8 n (K + 1).
// Build: hipcc -O3 --offload-arch=gfx950 march_bench.hip -o march_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int KMAX = 40;
typedef double dv2 __attribute__((ext_vector_type(2)));
struct Args { const double* v[KMAX]; double* out; long nx, ny; int strips, nbands, RY, SW; };

template <int W> struct Vt;
template <> struct Vt<1> { typedef double T; };
template <> struct Vt<2> { typedef dv2 T; };

__device__ __forceinline__ double hsum(double x) { return x; }
__device__ __forceinline__ double hsum(dv2 x) { return x.x + x.y; }

// one wave per strip of 64*W columns; WPB waves per block on adjacent strips; rows in flight PF
template <int W, int K, int PF, bool BAR, int WPB, int MINB>
__global__ void __launch_bounds__(64 * WPB, MINB) march(Args A) {
  typedef typename Vt<W>::T T;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long b = blockIdx.x;
  const long bpx = gridDim.x / 8;
  const long L = (b % 8) * bpx + b / 8;  // XCD-contiguous
  const long ngroups = (A.strips + WPB - 1) / WPB;
  if (L >= ngroups * A.nbands) return;
  const long band = L / ngroups, grp = L % ngroups;
  const long strip = grp * WPB + wid;
  const long c = (strip * 64 * W + lane * W) % A.nx;
  const long r0 = band * A.RY;
  const long r1 = r0 + A.RY < A.ny ? r0 + A.RY : A.ny;
  constexpr int RR = PF + 1;
  T ring[RR][K];
  auto load = [&](T* s, long r) {
    r = r < r1 ? r : r1 - 1;
    const long o = r * A.nx + c;
#pragma unroll
    for (int i = 0; i < K; ++i) s[i] = __builtin_nontemporal_load(reinterpret_cast<const T*>(A.v[i] + o));
  };
  double acc = 0.0;
#pragma unroll
  for (int d = 0; d < PF; ++d) load(ring[d], r0 + d);
  for (long t0 = r0; t0 < r1; t0 += RR) {
#pragma unroll
    for (int k = 0; k < RR; ++k) {
      const long r = t0 + k;
      load(ring[(k + PF) % RR], r + PF);
      T s = ring[k][0];
#pragma unroll
      for (int i = 1; i < K; ++i) s = s * 0.5 + ring[k][i];
      if constexpr (BAR) __syncthreads();
      if (r < r1 && strip < A.strips) *reinterpret_cast<T*>(A.out + r * A.nx + c) = s;
      acc += hsum(s);
    }
  }
  if (acc == 12345.678) A.out[0] = acc;
}

// contiguous chunks (the Krylov kernels' pattern): block b reads chunk b of every vector
template <int K>
__global__ void __launch_bounds__(256) chunk(Args A, long n, int cpb) {
  for (int cc = 0; cc < cpb; ++cc) {
    const long base = (long(blockIdx.x) * cpb + cc) * 2048 + 2 * threadIdx.x;
    if (base >= n) break;
    dv2 acc[4] = {};
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const dv2 x = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(A.v[i] + base + k * 512));
        acc[k] = acc[k] * 0.5 + x;
      }
#pragma unroll
    for (int k = 0; k < 4; ++k) *reinterpret_cast<dv2*>(A.out + base + k * 512) = acc[k];
  }
}

static long g_n;
template <typename F>
float timeit(F f) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) f();
  CK(hipEventRecord(a));
  for (int i = 0; i < 10; ++i) f();
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  CK(hipGetLastError());
  return ms / 10;
}

template <int W, int K, int PF, bool BAR, int WPB, int MINB>
void run_march(Args A, int rounds, int RYmin) {
  auto kern = march<W, K, PF, BAR, WPB, MINB>;
  int nb = 0, dev = 0, ncu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, 64 * WPB, 0));
  A.SW = 64 * W;
  A.strips = int((A.nx + A.SW - 1) / A.SW);
  const long wpr = (A.strips + WPB - 1) / WPB * WPB;
  long nbands = long(ncu) * nb * WPB * rounds / wpr;
  if (nbands > A.ny / RYmin) nbands = A.ny / RYmin;
  if (nbands < 1) nbands = 1;
  A.RY = int((A.ny + nbands - 1) / nbands);
  A.nbands = int((A.ny + A.RY - 1) / A.RY);
  long blocks = (wpr / WPB) * A.nbands;
  blocks = (blocks + 7) / 8 * 8;
  float ms = timeit([&] { hipLaunchKernelGGL(kern, dim3(blocks), dim3(64 * WPB), 0, 0, A); });
  const double bytes = 8.0 * g_n * (K + 1);
  printf("march W%d K%d PF%d BAR%d WPB%d minB%d occ%d rounds%d RY%4d: %8.1f us %7.1f GB/s %.3f\n",
         W, K, PF, int(BAR), WPB, MINB, nb, rounds, A.RY, ms * 1e3, bytes / ms / 1e6, bytes / ms / 1e6 / 8000);
}

template <int K>
void run_chunk(Args A) {
  long n = A.nx * A.ny;
  long chunks = (n + 2047) / 2048; int cpb = int((chunks + 4095) / 4096);
  dim3 g(unsigned((chunks + cpb - 1) / cpb));
  float ms = timeit([&] { hipLaunchKernelGGL((chunk<K>), g, dim3(256), 0, 0, A, n, cpb); });
  const double bytes = 8.0 * n * (K + 1);
  printf("chunk16K K%d: %8.1f us %7.1f GB/s %.3f\n", K, ms * 1e3, bytes / ms / 1e6, bytes / ms / 1e6 / 8000);
}

int main(int argc, char** argv) {
  const long N = 4096, n = N * N;
  g_n = n;
  Args A{};
  A.nx = N; A.ny = N;
  // vectors in ONE pool at stride n + skew doubles (the solver's workspace layout), skew from argv
  const long skew = argc > 1 ? atol(argv[1]) : 0;
  double* pool;
  CK(hipMalloc(&pool, (n + skew) * 8 * (KMAX + 1)));
  CK(hipMemset(pool, 0, (n + skew) * 8 * (KMAX + 1)));
  for (int i = 0; i < KMAX; ++i) A.v[i] = pool + (n + skew) * i;
  A.out = pool + (n + skew) * KMAX;
  printf("pool stride %ld doubles (skew %ld)\n", n + skew, skew);
  constexpr int K = 24;
  run_chunk<K>(A);
  run_march<1, K, 2, false, 4, 1>(A, 1, 8);
  run_march<2, K, 1, false, 4, 1>(A, 1, 8);
  run_march<2, K, 2, false, 4, 1>(A, 1, 8);
  run_march<2, K, 2, false, 4, 1>(A, 1, 256);
  run_march<2, K, 3, false, 4, 1>(A, 1, 8);
  return 0;
}

// Access-pattern microbenchmark, round 2: how wide must a wave's contiguous run per vector and row
// be for the row-marching pattern of the fused Arnoldi kernel to stream near the chunked ceiling?
// K fp64 vectors of 4096 x 4096; each wave marches down a band of rows, reading W columns per
// lane (W/2 16-B loads per vector and row: a wave covers 64 W columns, 512 W bytes contiguous);
// ROWS rows are loaded before any is consumed.  Reference: contiguous 16 KB chunks per block.
// Build: hipcc -O3 --offload-arch=gfx950 pattern2_bench.hip -o pattern2_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int KMAX = 32;
typedef double dv2 __attribute__((ext_vector_type(2)));
struct Args { const double* v[KMAX]; double* out; long nx, ny; int strips, nbands, RY; };

template <int W, int K, int ROWS, bool BAR = false, bool PAIRS = false>
__global__ void __launch_bounds__(256) march(Args A) {
  const int lane = threadIdx.x & 63;
  const long gw = long(blockIdx.x) * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (gw >= long(A.strips) * A.nbands) return;
  const long band = gw / A.strips, strip = gw % A.strips;
  // load j of a vector covers columns c + 128 j, +1; PAIRS (W = 2): the fused kernel's layout --
  // half h of the wave reads vector 2i + h, 64 columns per wave, one 16-B load per lane per pair
  const long c = PAIRS ? strip * 64 + (lane & 31) * 2 : strip * 64 * W + lane * 2;
  const int hf = lane >> 5;
  const long r0 = band * A.RY;
  const long r1 = r0 + A.RY < A.ny ? r0 + A.RY : A.ny;
  dv2 acc[W / 2] = {};
  for (long r = r0; r < r1; r += ROWS) {
    dv2 x[ROWS][K][W / 2];
#pragma unroll
    for (int q = 0; q < ROWS; ++q) {
      const long rr = (r + q < r1) ? r + q : r1 - 1;
#pragma unroll
      for (int i = 0; i < K; ++i)
#pragma unroll
        for (int j = 0; j < W / 2; ++j) {
          if (PAIRS && (i & 1)) continue;
          const double* base = PAIRS ? (hf ? A.v[i + 1 < K ? i + 1 : i] : A.v[i]) : A.v[i];
          x[q][i][j] = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(base + rr * A.nx + c + 128 * j));
        }
    }
#pragma unroll
    for (int q = 0; q < ROWS; ++q) {
#pragma unroll
      for (int i = 0; i < K; ++i)
#pragma unroll
        for (int j = 0; j < W / 2; ++j)
          if (!(PAIRS && (i & 1))) acc[j] += x[q][i][j];
      if constexpr (BAR) __syncthreads();
      const long rr = (r + q < r1) ? r + q : r1 - 1;
#pragma unroll
      for (int j = 0; j < W / 2; ++j)
        *reinterpret_cast<dv2*>(A.out + rr * A.nx + c + 128 * j) = acc[j];
    }
  }
}

template <int K>
__global__ void __launch_bounds__(256) chunk(Args A, long n, int cpb) {
  dv2 acc[4] = {};
  for (int cc = 0; cc < cpb; ++cc) {
    const long base = (long(blockIdx.x) * cpb + cc) * 2048 + 2 * threadIdx.x;
    if (base >= n) break;
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        acc[k] += __builtin_nontemporal_load(reinterpret_cast<const dv2*>(A.v[i] + base + k * 512));
#pragma unroll
    for (int k = 0; k < 4; ++k) *reinterpret_cast<dv2*>(A.out + base + k * 512) = acc[k];
  }
}

template <typename F>
float timeit(F launch) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) launch();
  CK(hipEventRecord(a));
  for (int i = 0; i < 10; ++i) launch();
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / 10;
}

template <int W, int K, int ROWS, bool BAR = false, bool PAIRS = false>
float run_march(Args A, int waves_target) {
  A.strips = int(A.nx / (PAIRS ? 64 : 64 * W));
  A.nbands = waves_target / A.strips; if (A.nbands < 1) A.nbands = 1;
  A.RY = int((A.ny + A.nbands - 1) / A.nbands); A.nbands = int((A.ny + A.RY - 1) / A.RY);
  const long nw = long(A.strips) * A.nbands;
  return timeit([&] { hipLaunchKernelGGL((march<W, K, ROWS, BAR, PAIRS>), dim3((nw + 3) / 4), dim3(256), 0, 0, A); });
}

template <int K>
void sweep(Args A) {
  const long n = A.nx * A.ny;
  const double bytes = 8.0 * n * (K + 1);
  auto rep = [&](const char* name, float ms) {
    printf("K=%2d %-34s %8.1f us  %7.1f GB/s  %.3f\n", K, name, ms * 1e3, bytes / ms / 1e6, bytes / ms / 1e6 / 8000);
  };
  {
    const long chunks = (n + 2047) / 2048; const int cpb = int((chunks + 4095) / 4096);
    rep("chunk 16KB", timeit([&] { hipLaunchKernelGGL((chunk<K>), dim3((chunks + cpb - 1) / cpb), dim3(256), 0, 0, A, n, cpb); }));
  }
  char nm[64];
  for (int w : {1024}) {
    snprintf(nm, 64, "march W2 rows1 barrier waves %d", w); rep(nm, run_march<2, K, 1, true>(A, w));
    snprintf(nm, 64, "march W2 rows2 barrier waves %d", w); rep(nm, run_march<2, K, 2, true>(A, w));
    snprintf(nm, 64, "pairs rows1 waves %d", w); rep(nm, run_march<2, K, 1, false, true>(A, w));
    snprintf(nm, 64, "pairs rows2 waves %d", w); rep(nm, run_march<2, K, 2, false, true>(A, w));
    snprintf(nm, 64, "pairs rows2 barrier waves %d", w); rep(nm, run_march<2, K, 2, true, true>(A, w));
    snprintf(nm, 64, "pairs rows4 waves %d", w); rep(nm, run_march<2, K, 4, false, true>(A, w));
  }
  for (int w : {1024, 2048}) {
    snprintf(nm, 64, "march W2 (1KB) rows1 waves %d", w); rep(nm, run_march<2, K, 1>(A, w));
    snprintf(nm, 64, "march W2 (1KB) rows2 waves %d", w); rep(nm, run_march<2, K, 2>(A, w));
    snprintf(nm, 64, "march W4 (2KB) rows1 waves %d", w); rep(nm, run_march<4, K, 1>(A, w));
    snprintf(nm, 64, "march W8 (4KB) rows1 waves %d", w); rep(nm, run_march<8, K, 1>(A, w));
  }
}

int main() {
  const long N = 4096, n = N * N;
  Args A{};
  A.nx = N; A.ny = N;
  for (int i = 0; i < KMAX; ++i) { double* p; CK(hipMalloc(&p, n * 8 + (1 << 17))); CK(hipMemset(p, 0, n * 8)); A.v[i] = p; }
  CK(hipMalloc(&A.out, n * 8));
  sweep<26>(A);
  return 0;
}

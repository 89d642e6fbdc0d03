// Device-side helpers shared by the stencil and Krylov kernels (gfx950, wave64).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace nk {

// NaN-propagating max, so that max|F| of a vector holding a NaN is NaN (numpy abs(x).max()).
__device__ __forceinline__ double nmax(double a, double b) {
  if (a != a) return a;
  return (b != b || b > a) ? b : a;
}

// Sum NV values over the 64 lanes of a wave (xor butterfly); every lane ends with the sums.
template <int NV>
__device__ __forceinline__ void wave_sum(double (&v)[NV]) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] += __shfl_xor(v[k], o, 64);
  }
}

// Reduce NV values over a 1-D block of BS threads: the first NSUM values are summed, the rest
// max-reduced (NaN-propagating).  Wave64 xor-shuffle tree, then one LDS round across waves.
// Returns value `threadIdx.x` to the threads with threadIdx.x < NV (others get 0).
// `buf` selects one of two LDS buffers so that back-to-back calls need one barrier each.
template <int NV, int NSUM, int BS>
__device__ __forceinline__ double block_reduce(double (&v)[NV], int buf = 0) {
  static_assert(BS % 64 == 0, "block must be whole waves");
  constexpr int NW = BS / 64;
  __shared__ double sm[2][NV][NW];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const double t = __shfl_xor(v[k], o, 64);
      v[k] = (k < NSUM) ? v[k] + t : nmax(v[k], t);
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) sm[buf][k][wid] = v[k];
  }
  __syncthreads();
  double acc = 0.0;
  if (threadIdx.x < NV) {
    const int k = threadIdx.x;
    acc = sm[buf][k][0];
    for (int w = 1; w < NW; ++w) acc = (k < NSUM) ? acc + sm[buf][k][w] : nmax(acc, sm[buf][k][w]);
  }
  return acc;
}

// One column of a partial-sum matrix reduced by a block of RB threads: the sum (or NaN-propagating
// max) of p[0 .. nblk), in a fixed tree (the result does not depend on timing).  Thread 0's
// return value is the result.
template <int RB>
__device__ __forceinline__ double reduce_column(const double* p, int64_t nblk, bool is_sum) {
  // max reductions start from -inf (signed quantities such as -min(...) are allowed); the
  // loads of one thread are issued together (no dependent load chain)
  double acc = is_sum ? 0.0 : -INFINITY;
  int64_t b = threadIdx.x;
  for (; b + 3 * RB < nblk; b += 4 * RB) {
    const double x0 = p[b], x1 = p[b + RB], x2 = p[b + 2 * RB], x3 = p[b + 3 * RB];
    acc = is_sum ? acc + x0 + x1 + x2 + x3 : nmax(nmax(nmax(nmax(acc, x0), x1), x2), x3);
  }
  for (; b < nblk; b += RB) acc = is_sum ? acc + p[b] : nmax(acc, p[b]);
  double v[1] = {acc};
  const double s = is_sum ? block_reduce<1, 1, RB>(v) : block_reduce<1, 0, RB>(v);
  return (nblk == 0) ? 0.0 : s;  // empty input
}

// Write-through (sc1) 8-B stores and loads: the hand-off between the blocks of one launch with
// no release fence (MI355X_MICROARCH.md "Valid forms", first row: every byte stored sc1, every
// storing wave drained, one agent-scope counter add per block; every load of the bytes sc1).
// An agent-scope fence per block would write back its XCD's whole L2 (the launch's freshly
// written output vectors) and invalidate its L1 under the blocks still streaming.
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p),
                     static_cast<unsigned long long>(__double_as_longlong(v)), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __longlong_as_double(static_cast<long long>(
      __hip_atomic_load(reinterpret_cast<unsigned long long*>(const_cast<double*>(p)),
                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
}
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

}  // namespace nk

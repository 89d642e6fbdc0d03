// Device-side Arnoldi control: the per-step host arithmetic of lgmres.cpp's fused path
// (scipy/sparse/linalg/_isolve/_gcrotmk.py:114-165 as restated there) run by one wave between two
// fused Arnoldi launches, so consecutive steps queue on the stream without a host round trip.
//
// Lane i holds entry i of the step's vectors (j + 1 <= kArnMaxNV + 1 <= 64 entries).  The serial
// parts -- the Givens sweep over the previous Hessenberg column, the forward substitution of the
// inverse compact-WY MGS, |h|^2 -- run in the host loop's order (uniform loops over readlane'd
// values), so the device differs from the host only by fused multiply-adds.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstddef>
#include <cmath>

#include "nk_device.h"
#include "nk_kernels.h"
#include "arnctl_dev.h"
#include "peer_dev.h"

namespace nk {
namespace {

constexpr int RB = 1024;  // reduction block (as reduce_final_kernel)

#ifdef ARN_CTL_PROBE  // timing build (scripts/dbg/ctl_probe.py): stage times of the control launch
// [0] launches, [1] first block's entry -> last block counted in, [2] -> values collected,
// [3] -> all-reduced, [4] -> control done, [5] first entry -> last block's entry
__device__ unsigned long long g_ctl_probe[8];
__device__ unsigned long long g_ctl_t0 = ~0ull;   // this launch's first entry (reset by the last)
__device__ unsigned long long g_ctl_tl = 0;       // this launch's last entry
#define CTL_STAMP(v) const unsigned long long v = wall_clock64()
#else
#define CTL_STAMP(v)
#endif

// up > 0: first copy the host's pinned loop state H to S (the fields before R, and the Gram rows
// 0 .. up-2) -- the entry of a run of device steps, which would otherwise take two runtime blits
// (H is mapped device-visible memory).  All loads are issued before the first store.
__device__ void upload_state(ArnCtlState* S, const ArnCtlState* H, int rows) {
  const int lane = threadIdx.x & 63;
  constexpr int kHead = int(offsetof(ArnCtlState, R) / 8);  // 8-B words before R
  constexpr int kRow = kMaxVec + 1;                          // doubles per Gram row
  constexpr int kI = (kHead + 63) / 64;
  const uint64_t* h = reinterpret_cast<const uint64_t*>(H);
  uint64_t* d = reinterpret_cast<uint64_t*>(S);
  uint64_t v[kI];
#pragma unroll
  for (int i = 0; i < kI; ++i) v[i] = (lane + 64 * i < kHead) ? h[lane + 64 * i] : 0;
#pragma unroll
  for (int i = 0; i < kI; ++i)
    if (lane + 64 * i < kHead) d[lane + 64 * i] = v[i];
  const double* hg = &H->gram[0][0];
  double* dg = &S->gram[0][0];
  for (int q = lane; q < rows * kRow; q += 64) dg[q] = hg[q];
  __threadfence();  // the state before the control reads it (this wave, another lane's stores)
}

// The hand-off from the reducing blocks to the last one without fences (arnoldi.hip "Tail", the
// same form): every value stored sc1 and drained, one agent-scope counter add per block, the last
// block's wave loads the values sc1 into LDS.  (An agent-scope __threadfence per block wrote
// back and invalidated its XCD's L2 and the system fence of the one-GPU kernel did the same,
// behind every fused launch.)  true: this block arrived last.
__device__ __forceinline__ bool reduced_arrive(ArnCtlState* S) {
  drain_stores();
  return __hip_atomic_fetch_add(&S->arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
         gridDim.x - 1;
}
// the last block's first wave: the n values into LDS (vals), the counter reset for the next
// launch (stream order)
__device__ __forceinline__ void reduced_collect(ArnCtlState* S, const double* result, double* vals,
                                                int n) {
  const int lane = int(threadIdx.x);
  for (int i = lane; i < n; i += 64) vals[i] = ld_sc1(result + i);
  if (lane == 0) __hip_atomic_store(&S->arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__global__ void __launch_bounds__(64) arn_ctl_kernel(ArnCtlState* S, ArnCtlState* H,
                                                     const double* red, double* red_host,
                                                     double* prm, uint32_t* status, int t, int up) {
  __shared__ double G[kArnMaxNV + 1][kArnMaxNV + 1];
  if (up > 0) upload_state(S, H, up - 1);
  ctl_body(S, H, red, red_host, prm, status, t, G);
}

__global__ void __launch_bounds__(RB) arn_reduce_ctl_kernel(const double* partial, int64_t nblk,
                                                            double* result, double* result_host,
                                                            ArnCtlState* S, ArnCtlState* H,
                                                            double* prm, uint32_t* status, int t) {
  // the control's loads (first wave of every block), in flight during the reduction (they
  // lengthen it by ~1 us, but issued after it they cost more: profiles/r06_short_slab.md 9)
  CtlPre P;
  if (threadIdx.x < 64) ctl_load(S, t, P);
  const int k = blockIdx.x;
  const double s = reduce_column<RB>(partial + int64_t(k) * nblk, nblk, true);
  __shared__ bool last;
  __shared__ double vals[kRedMax];  // the last block's copy of every block's value
  if (threadIdx.x == 0) {
    // written through and drained before counting in (reduced_arrive)
    st_sc1(result + k, s);
    if (result_host) result_host[k] = s;  // pinned host memory: not cached
    last = reduced_arrive(S);
  }
  __syncthreads();
  if (!last || threadIdx.x >= 64) return;
  reduced_collect(S, result, vals, int(gridDim.x));
  ctl_run(S, H, vals, nullptr, prm, status, t, P);
}

// Row slabs over the peer-memory communicator: the reduction, the all-reduce of its nval sums
// (peer_dev.h, one wave writing into every rank's buffer over xGMI) and the control of step t in
// ONE launch -- the three launches (reduce, peer all-reduce, control) of the generic path.  Every
// rank's last block computes the same all-reduced values, so every rank's control takes the same
// decisions.  A failed all-reduce (a peer aborted or timed out) halts the queued fused step and
// leaves status[t] unset; the host's wait then finds the communicator failed.
__global__ void __launch_bounds__(RB) arn_reduce_allreduce_ctl_kernel(
    const double* partial, int64_t nblk, double* result, double* result_host, const PeerArgs pa,
    ArnCtlState* S, ArnCtlState* H, double* prm, uint32_t* status, int t) {
#ifdef ARN_CTL_PROBE
  if (threadIdx.x == 0) {
    const unsigned long long e = wall_clock64();
    atomicMin(&g_ctl_t0, e);
    atomicMax(&g_ctl_tl, e);
  }
#endif
  // the control's loads (first wave of every block), in flight during the reduction (they
  // lengthen it by ~1 us, but issued after it they cost more: profiles/r06_short_slab.md 9)
  CtlPre P;
  if (threadIdx.x < 64) ctl_load(S, t, P);
  const int k = blockIdx.x;
  const double s = reduce_column<RB>(partial + int64_t(k) * nblk, nblk, true);
  __shared__ bool last;
  __shared__ double vals[kRedMax];  // the last block's copy of every block's value
  if (threadIdx.x == 0) {
    st_sc1(result + k, s);
    last = reduced_arrive(S);
  }
  __syncthreads();
  if (!last || threadIdx.x >= 64) return;
  CTL_STAMP(p_last);
  const int n = int(gridDim.x);
  reduced_collect(S, result, vals, n);
  CTL_STAMP(p_coll);
  if (!peer_allreduce_wave_wt(pa, vals, n, n)) {
    if (threadIdx.x == 0) prm[kArnMaxNV + 3] = 1.0;  // the queued fused step does nothing
    return;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");  // the combined values in LDS
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  CTL_STAMP(p_ar);
  for (int i = int(threadIdx.x); i < n; i += 64) result[i] = vals[i];
  ctl_run(S, H, vals, result_host, prm, status, t, P);
#ifdef ARN_CTL_PROBE
  CTL_STAMP(p_end);
  if (threadIdx.x == 0) {
    const unsigned long long t0 = atomicAdd(&g_ctl_t0, 0ull), tl = atomicAdd(&g_ctl_tl, 0ull);
    atomicAdd(&g_ctl_probe[0], 1ull);
    atomicAdd(&g_ctl_probe[1], p_last - t0);
    atomicAdd(&g_ctl_probe[2], p_coll - p_last);
    atomicAdd(&g_ctl_probe[3], p_ar - p_coll);
    atomicAdd(&g_ctl_probe[4], p_end - p_ar);
    atomicAdd(&g_ctl_probe[5], tl - t0);
    atomicExch(&g_ctl_t0, ~0ull);
    atomicExch(&g_ctl_tl, 0ull);
  }
#endif
}

}  // namespace

#ifdef ARN_CTL_PROBE
extern "C" int nk_debug_ctl_probe(unsigned long long* out) {
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ctl_probe), sizeof(g_ctl_probe)) != hipSuccess)
    return -1;
  static const unsigned long long zero[8] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_ctl_probe), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif

hipError_t arn_ctl_launch(ArnCtlState* S, ArnCtlState* H, const double* red, double* red_host,
                          double* prm, uint32_t* status, int t, hipStream_t s, int upload_rows) {
  if (!S || !H || !red || !prm || !status || t < 0 || t > kMaxVec || upload_rows > kMaxVec + 1)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(arn_ctl_kernel, dim3(1), dim3(64), 0, s, S, H, red, red_host, prm, status,
                     t, upload_rows < 0 ? 0 : upload_rows + 1);
  return hipGetLastError();
}

hipError_t arn_reduce_ctl_launch(const double* partial, int64_t nblk, int nval, double* result,
                                 double* result_host, ArnCtlState* S, ArnCtlState* H, double* prm,
                                 uint32_t* status, int t, hipStream_t s) {
  if (!partial || !result || !S || !H || !prm || !status || nval < 1 || nval > kRedMax || t < 0 ||
      t > kMaxVec)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(arn_reduce_ctl_kernel, dim3(unsigned(nval)), dim3(RB), 0, s, partial, nblk,
                     result, result_host, S, H, prm, status, t);
  return hipGetLastError();
}

hipError_t arn_reduce_allreduce_ctl_launch(const double* partial, int64_t nblk, int nval,
                                           double* result, double* result_host, const PeerArgs& pa,
                                           ArnCtlState* S, ArnCtlState* H, double* prm,
                                           uint32_t* status, int t, hipStream_t s) {
  if (!partial || !result || !S || !H || !prm || !status || nval < 1 || nval > kRedMax || t < 0 ||
      t > kMaxVec || pa.P < 1 || pa.P > kMaxPeers)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(arn_reduce_allreduce_ctl_kernel, dim3(unsigned(nval)), dim3(RB), 0, s,
                     partial, nblk, result, result_host, pa, S, H, prm, status, t);
  return hipGetLastError();
}

}  // namespace nk

// Device-side layout and primitives of the peer-memory communicator (peer.hip), shared with the
// kernels that run a collective inside their own launch (arnctl.hip: reduction + all-reduce +
// Arnoldi control; arnoldi.hip: slab edge rows + halo exchange).  See peer.hip for the protocol.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "nk_device.h"

namespace nk {

constexpr int kMaxPeers = 64;
constexpr int kRedMax = 256;  // values per all-reduce (the fused multi-dot: 2 nv + 3 <= 73)
constexpr int kHaloBlock = 256;
// Column blocks of a halo-exchange grid (peer_halo_kernel, the slab edge + halo kernel), which
// stride over wider rows: every block of such a grid waits for flags published only once all of
// the grid's blocks have counted in, so the grid must be able to be resident as a whole even when
// several ranks' grids share one GPU -- at most 16 x 4 blocks of 4 waves = 256 waves per rank,
// against 256 CUs x 32 wave slots.
constexpr int kHaloMaxBlocks = 16;
__host__ __device__ inline int halo_blocks(int64_t nx) {
  const int64_t b = (nx + kHaloBlock - 1) / kHaloBlock;
  return int(b < kHaloMaxBlocks ? (b > 0 ? b : 1) : kHaloMaxBlocks);
}

// byte offsets inside a rank's exported buffer
constexpr int64_t kOffAbort = 0;                                  // uint64
constexpr int64_t kOffRedFlag = 64;                               // [2][kMaxPeers] uint64
constexpr int64_t kOffHaloFlag = kOffRedFlag + 2 * kMaxPeers * 8;  // [2][2] uint64
constexpr int64_t kOffRedSlot = 2048;                             // [2][P][kRedMax] double
__host__ __device__ inline int64_t off_stage(int P) {             // [2][2][2][max_nx] double
  return (kOffRedSlot + int64_t(2) * P * kRedMax * 8 + 255) / 256 * 256;
}
// chunk flags of the in-kernel slab exchange (arnoldi.hip, "Slab exchange"): [2][2][chunks] uint64
// after the staging rows, one per parity, side and kXChunk-column chunk of a staged row pair
constexpr int64_t kXChunk = 128;
__host__ __device__ inline int64_t x_chunks(int64_t max_nx) { return (max_nx + kXChunk - 1) / kXChunk; }
__host__ __device__ inline int64_t off_xflag(int P, int64_t max_nx) {
  return off_stage(P) + int64_t(2) * 2 * 2 * max_nx * 8;
}
// halo slots of the pushed-halo-rows path (arnoldi.hip "Pushed halo rows"): one per pool vector
// of the stepper that claimed them, 4 rows of max_nx doubles each, after the chunk flags
constexpr int64_t kHaloSlots = 2 * 64 + 8;  // >= the largest solver pool (vectors_needed)
__host__ __device__ inline int64_t off_slots(int P, int64_t max_nx) {
  return (off_xflag(P, max_nx) + int64_t(2) * 2 * x_chunks(max_nx) * 8 + 255) / 256 * 256;
}
__host__ __device__ inline int64_t buffer_bytes(int P, int64_t max_nx) {
  return off_slots(P, max_nx) + kHaloSlots * 4 * max_nx * 8;
}

// A store into a peer's halo slot (pushed halo rows): 16 B with the system-scope policy bits, so
// it is written through this XCD's L2 to the slot's memory and the producer only drains its own
// stores (drain_stores) before it ends -- no system fence, whose L2 write-back + invalidate of the
// whole XCD cost the fused Arnoldi launch's edge bands ~6 us at its end (round 6,
// profiles/r06_short_slab.md section 7).  The s_nop is the wait state a store of more than 8 B
// needs before its data registers are rewritten, which the compiler's hazard check does not see
// through an asm statement.  (One 16-B store rather than two 8-B atomic stores: the latter cost
// the nv-35 Arnoldi kernel, at the register ceiling, a 20-B scratch spill.)
__device__ __forceinline__ void store_sys8(double* d, double a) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(d),
                     static_cast<unsigned long long>(__double_as_longlong(a)), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void store_sys16(double* d, double a, double b) {
  typedef double d2v __attribute__((ext_vector_type(2)));
  const d2v v2 = {a, b};
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 0" ::"v"(d), "v"(v2) : "memory");
}

struct PeerArgs {
  char* base[kMaxPeers];  // every rank's buffer in this address space (mine: base[rank])
  int P, rank;
  int64_t max_nx;
  uint64_t tag;
  uint32_t* counter;  // arrival counter of the halo kernel's blocks (local, reset by the last)
  int* err;           // pinned host error word
  uint64_t wait_ticks;  // bound of one wait, in wall_clock64() ticks (NKHIP_PEER_TIMEOUT_S)
};

__device__ __forceinline__ uint64_t* red_flag(char* b, int par, int q) {
  return reinterpret_cast<uint64_t*>(b + kOffRedFlag) + par * kMaxPeers + q;
}
__device__ __forceinline__ uint64_t* halo_flag(char* b, int par, int side) {
  return reinterpret_cast<uint64_t*>(b + kOffHaloFlag) + par * 2 + side;
}
__device__ __forceinline__ double* red_slot(char* b, int P, int par, int q) {
  return reinterpret_cast<double*>(b + kOffRedSlot) + (int64_t(par) * P + q) * kRedMax;
}
// staging rows: side 0 = "lo" (the previous rank's last two rows), 1 = "hi" (the next rank's
// first two rows)
__host__ __device__ inline double* stage(char* b, int P, int64_t max_nx, int par, int side,
                                         int row) {
  return reinterpret_cast<double*>(b + off_stage(P)) + ((int64_t(par) * 2 + side) * 2 + row) * max_nx;
}

__device__ __forceinline__ uint64_t* xflag(char* b, int P, int64_t max_nx, int par, int side,
                                           int64_t ch) {
  return reinterpret_cast<uint64_t*>(b + off_xflag(P, max_nx)) + (par * 2 + side) * x_chunks(max_nx) + ch;
}

// Wait (one lane) until *flag == tag; false on abort (the abort word of my buffer `me`) or
// timeout, with the error word set.  The polls are relaxed (they read past the caches, system
// scope) and ONE acquire follows the tag: an acquire per poll would invalidate this XCD's L2 over
// and over, under the feet of every other block on it (the fused kernel's edge bands wait while
// the interior bands stream).  The bound is elapsed time on the constant-rate wall clock
// (`ticks` of wall_clock64(), set from hipDeviceAttributeWallClockRate on the host), checked
// every 64 polls, so it holds whatever one poll costs.
// ACQ false: no acquire after the tag (the caller reads the published data with system-scope
// loads, which go past the caches anyway)
template <bool ACQ = true>
__device__ inline bool wait_flag_tag(const uint64_t* flag, uint64_t tag, const char* me, int* err,
                                     uint64_t ticks) {
  const uint64_t* abort_word = reinterpret_cast<const uint64_t*>(me + kOffAbort);
  const uint64_t t0 = wall_clock64();  // once: a wrapping poll count must not restart it
  for (uint32_t n = 0;; ++n) {
    if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == tag) {
      if constexpr (ACQ) __atomic_thread_fence(__ATOMIC_ACQUIRE);  // system scope
      return true;
    }
    if ((n & 63) == 0) {
      const uint64_t now = wall_clock64();
      if (__hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0 ||
          now - t0 > ticks) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return false;
      }
    }
    __builtin_amdgcn_s_sleep(4);
  }
}
__device__ inline bool wait_tag(const PeerArgs& a, const uint64_t* flag) {
  return wait_flag_tag(flag, a.tag, a.base[a.rank], a.err, a.wait_ticks);
}

// The second half of a halo exchange, called by every block of the grid after the block wrote
// its part of the neighbours' staging rows: the last block to arrive publishes both neighbours'
// flags (release, system scope), every block waits for its own two flags, and the blockIdx.y == 0
// blocks copy their columns -- blockIdx.x * kHaloBlock + threadIdx.x, strided by the grid's
// columns (halo_blocks) -- of the staged rows into lo / hi (2 rows of nx each).  false: a peer
// failed or timed out (error word set, lo / hi untouched).
__device__ inline bool peer_halo_finish(const PeerArgs& a, int64_t nx, double* lo, double* hi) {
  const int par = int(a.tag & 1);
  const int prev = (a.rank - 1 + a.P) % a.P, next = (a.rank + 1) % a.P;
  __threadfence_system();
  __syncthreads();
  __shared__ int ok;
  if (threadIdx.x == 0) {
    ok = 1;
    const uint32_t arrived =
        __hip_atomic_fetch_add(a.counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (arrived == gridDim.x * gridDim.y - 1) {  // every block's rows are out: publish
      __hip_atomic_store(a.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence_system();
      __hip_atomic_store(halo_flag(a.base[prev], par, 1), a.tag, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(halo_flag(a.base[next], par, 0), a.tag, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    }
    char* mine = a.base[a.rank];
    if (!wait_tag(a, halo_flag(mine, par, 0)) || !wait_tag(a, halo_flag(mine, par, 1))) ok = 0;
  }
  __syncthreads();
  if (!ok) return false;
  __threadfence_system();
  if (blockIdx.y == 0) {
    char* mine = a.base[a.rank];
    const int64_t step = int64_t(gridDim.x) * blockDim.x;
    for (int64_t c = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; c < nx; c += step) {
      lo[c] = stage(mine, a.P, a.max_nx, par, 0, 0)[c];
      lo[nx + c] = stage(mine, a.P, a.max_nx, par, 0, 1)[c];
      hi[c] = stage(mine, a.P, a.max_nx, par, 1, 0)[c];
      hi[nx + c] = stage(mine, a.P, a.max_nx, par, 1, 1)[c];
    }
  }
  return true;
}

// One wave (lanes 0..63 of the calling block; the caller's other waves take no part): v[0, nv)
// summed (k < nsum) or NaN-propagating max-reduced over the ranks, in rank order (bitwise the
// same on every rank), in place.  false: a peer failed or timed out (error word set, v unchanged).
__device__ inline bool peer_allreduce_wave(const PeerArgs& a, double* v, int nsum, int nv) {
  const int lane = threadIdx.x & 63;
  const int par = int(a.tag & 1);
  for (int t = lane; t < nv; t += 64) {
    const double x = v[t];
    for (int q = 0; q < a.P; ++q) red_slot(a.base[q], a.P, par, a.rank)[t] = x;
  }
  __threadfence_system();
  __builtin_amdgcn_wave_barrier();
  for (int q = lane; q < a.P; q += 64)
    __hip_atomic_store(red_flag(a.base[q], par, a.rank), a.tag, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  bool ok = true;
  for (int q = lane; q < a.P; q += 64) ok = ok && wait_tag(a, red_flag(a.base[a.rank], par, q));
  // every lane's waits, combined (a lane with no peer to wait for reports ok)
  if (__builtin_amdgcn_ballot_w64(!ok) != 0) return false;
  __threadfence_system();
  char* mine = a.base[a.rank];
  for (int t = lane; t < nv; t += 64) {
    double acc = red_slot(mine, a.P, par, 0)[t];
    for (int q = 1; q < a.P; ++q) {
      const double x = red_slot(mine, a.P, par, q)[t];
      acc = (t < nsum) ? acc + x : nmax(acc, x);
    }
    v[t] = acc;
  }
  return true;
}

// peer_allreduce_wave without fences (the control launches, arnctl.hip; the fused launch's tail
// keeps the fenced form, its code being part of every fused kernel): the contributions are
// written through to every rank's slot (store_sys8) and drained before the flags go out, the
// flags are polled without an acquire, and the slots are read with system-scope loads.  The two
// system fences of the fenced form write back and invalidate this XCD's L2 each.
__device__ inline bool peer_allreduce_wave_wt(const PeerArgs& a, double* v, int nsum, int nv) {
  const int lane = threadIdx.x & 63;
  const int par = int(a.tag & 1);
  for (int t = lane; t < nv; t += 64) {
    const double x = v[t];
    for (int q = 0; q < a.P; ++q) store_sys8(red_slot(a.base[q], a.P, par, a.rank) + t, x);
  }
  drain_stores();
  __builtin_amdgcn_wave_barrier();
  for (int q = lane; q < a.P; q += 64)
    __hip_atomic_store(red_flag(a.base[q], par, a.rank), a.tag, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  bool ok = true;
  for (int q = lane; q < a.P; q += 64)
    ok = ok && wait_flag_tag<false>(red_flag(a.base[a.rank], par, q), a.tag, a.base[a.rank], a.err,
                                    a.wait_ticks);
  if (__builtin_amdgcn_ballot_w64(!ok) != 0) return false;
  char* mine = a.base[a.rank];
  auto ld = [](const double* p) {
    return __longlong_as_double(static_cast<long long>(
        __hip_atomic_load(reinterpret_cast<unsigned long long*>(const_cast<double*>(p)),
                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)));
  };
  for (int t = lane; t < nv; t += 64) {
    double acc = ld(red_slot(mine, a.P, par, 0) + t);
    for (int q = 1; q < a.P; ++q) {
      const double x = ld(red_slot(mine, a.P, par, q) + t);
      acc = (t < nsum) ? acc + x : nmax(acc, x);
    }
    v[t] = acc;
  }
  return true;
}

}  // namespace nk

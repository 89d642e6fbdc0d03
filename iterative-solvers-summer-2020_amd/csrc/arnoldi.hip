// Fused Arnoldi step of the Swift-Hohenberg Newton-Krylov solve (gfx950, wave64).
//
// One launch does what SciPy's _fgmres loop body does between two matvecs
// (scipy/sparse/linalg/_isolve/_gcrotmk.py:104-143) plus the matvec of the next step
// (KrylovJacobian.matvec, scipy/optimize/_nonlin.py:1500-1513 on the residual of
// sh_scipy_nk.py:47-49):
//   v      = tau*w + sum_i c_i V_i            (the Gram-Schmidt update of step j; c_i = -h_i sig_i)
//   u      = v (or an LGMRES augmentation vector z when EXT)
//   w'     = (G(x0 + alpha u) - G(x0)) / sc   (the FD Jacobian-vector product of step j+1,
//                                              evaluated in closed form, see centre())
//   sums   w'.V_i, w'.v, v.V_i, v.v, w'.w'    (the multi-dot of step j+1, Gram row included)
// so the basis V_0..V_j is read ONCE per Arnoldi step instead of twice (update + multi-dot), and
// neither v nor w' is re-read.  Unfused, a step moves (2j + 9) vectors; fused (j + 5): V_0..V_j,
// w and x0 in, v and w' out (the closed form needs no G0 = G(x0)).
//
// The stencil couples rows r-2..r+2, so a wave marches down a band of rows with the update running
// two rows AHEAD of the stencil: at row r it forms v[r+2] from V_i[r+2], evaluates w'[r] on the
// 5-row window of u, and takes the dot products of row r against V_i[r].  Loads run PF rows ahead
// in a register ring (rotated by unrolling the walk by its length, so no register is copied); the
// basis row and x0 of rows r, r+1 wait in an LDS ring for their dot products, which keeps the
// registers for loads in flight.  The basis length is a template parameter (fully unrolled).
//
// Lanes ("vector pairs", see arnoldi_kernel): a wave owns 64 aligned columns; one 16-B load per
// lane streams two 512-B row segments of two entries (an aligned wave segment streams at 62-68 %
// of peak in scripts/micro/pattern_bench.hip, an overlapping 60-column one at 52-55 %).  Column
// neighbours inside the wave come from DPP lane shifts, the edge columns of the block's waves
// through LDS (one barrier per row), and the block's outer halo (two columns each side) from
// PACKED halo loads: lane L fetches halo column L%4 of entry L/4 (16 entries per instruction),
// DPP/permlane sums form c_i V_i per column.  Each band recomputes v on the two rows above and
// below it (band halo).  Per-lane sums are wave-reduced once at the end and written as one
// partial per wave (deterministic: a fixed wave -> rows mapping and a fixed order).
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "arnctl_dev.h"
#include "nk_device.h"
#include "nk_kernels.h"
#include "peer_dev.h"

namespace nk {
namespace {

constexpr int kSW = 64;  // columns per wave (one per lane)
constexpr int WPB = 4;   // waves per block (the packed halo loads carry 16 * WPB entries)
static_assert(WPB * kSW == kEdgeW, "edge arrays are laid out for the fused kernel's blocks");
// waves per block of the mailbox instantiation: it reads no edge arrays, and its halos cost a
// record per block side, so narrower blocks (less LDS lag per block, 2-wave barriers) pay:
// nv 24 0.602-0.610 -> 0.618-0.619 of 8 TB/s with 2 waves (profiles/r02_arnoldi_ab.md)
constexpr int kMbWPB = 2;

__device__ __forceinline__ double applyL13(const SHCoef& k, double c, double a1, double dg,
                                           double a2) {
  return k.c0 * c + k.c1 * a1 + k.c2 * dg + k.c3 * a2;
}

// Loads of the once-streamed fields: non-temporal (they must not evict the band/strip halos and
// the rows the ring still holds from L2) and addressed as SGPR base + 32-bit VGPR byte offset,
// so a row's loads share one offset register.
template <bool NT>
__device__ __forceinline__ double ldb(const double* base, uint32_t off) {
  const double* p = reinterpret_cast<const double*>(reinterpret_cast<const char*>(base) + off);
  if constexpr (NT) return __builtin_nontemporal_load(p);
  return *p;
}

// A load the compiler must emit as global_load: a pointer picked per lane from a table of kernel
// arguments loses its address space in inference and becomes a flat load, whose wait the
// compiler widens to vmcnt(0) -- draining the whole row's load batch once per row.
typedef const double __attribute__((address_space(1))) gdouble;
__device__ __forceinline__ double gld(const double* p) { return *(gdouble*)p; }

// Stores through a raw buffer resource: a lane whose offset is out of range (kOOB) writes
// nothing, so masked stores need no branch.
constexpr uint32_t kOOB = 0xFFFFFFF0u;
// Cache policy of the fused kernels' streamed outputs (v, w' and their edge arrays): 0 = plain
// (the line stays dirty in the XCD's L2 until evicted or the kernel-end release writes it back),
// 16 = sc1 (written through and dropped from L2: no dirty L2 to write back at the kernel boundary;
// MI355X_MICROARCH.md "stores of each flavour").  Build-time (ARN_OUT_POL) for the A/B.
#ifndef ARN_OUT_POL
#define ARN_OUT_POL 0
#endif
constexpr int kOutPol = ARN_OUT_POL;

// Bounds-checked build (`make check` -> nkhip/libnkhip_check.so, -DNKHIP_ARN_CHECK; GPU
// AddressSanitizer is not available on this pool).  Every index the fused kernels compute --
// row and column of each streamed load, block-halo and edge-array offsets, slab halo rows,
// mailbox records, store offsets, partial-sum slots -- goes through CI()/ARN_CHK(): an index out
// of its array is counted (per lane, with the first source line) and replaced by 0, so the
// kernel cannot fault and the host reads the counters afterwards (nk_debug_bounds).  In the
// product build both are no-ops.
#ifdef NKHIP_ARN_CHECK
// [lane]: violations, [64 + lane]: 2^32 - the smallest line (all zero: nothing recorded)
__device__ unsigned long long g_arn_chk[128];
__device__ __forceinline__ void arn_chk(bool ok, int line) {
  if (!ok) {
    const int l = int(threadIdx.x & 63);  // a per-lane address: vector atomics
    atomicAdd(&g_arn_chk[l], 1ull);
    atomicMax(&g_arn_chk[64 + l], (1ull << 32) - (unsigned long long)line);
  }
}
__device__ __forceinline__ int64_t chk_idx(int64_t i, int64_t lim, int line) {
  const bool ok = i >= 0 && i < lim;
  arn_chk(ok, line);
  return ok ? i : 0;
}
#define ARN_CHK(c) arn_chk((c), __LINE__)
#else
#define ARN_CHK(c) ((void)0)
__device__ __forceinline__ int64_t chk_idx(int64_t i, int64_t, int) { return i; }
#endif
// element index i of an array of lim elements (a 16-B pair load: lim - 1)
#define CI(i, lim) chk_idx((i), (lim), __LINE__)
// a buffer-resource store offset (bytes; kOOB = masked) of a 16-B record into lim elements
#define CO(off, lim) \
  uint32_t((off) == kOOB ? kOOB : uint32_t(8 * chk_idx(int64_t(off) / 8, (lim) - 1, __LINE__)))
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(double* p, int64_t n) {
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, int(uint32_t(n * 8)), 0x00020000);
}

// Per-step scalars of a fused launch: the kernel arguments, or -- under device-side Arnoldi
// control -- the parameter block the control kernel wrote (nk_kernels.h kCtlPrm).  Read once,
// before a kernel's row loop (a load inside it would join the row's wait-count queue).  The
// block is read through a buffer resource (no records when there is none), so both sources are
// plain loads and the selection never turns into one load through a merged generic pointer.
__device__ __forceinline__ double arn_prm(const ArnoldiArgs& A, int i, double arg) {
  const __amdgpu_buffer_rsrc_t r = rsrc(const_cast<double*>(A.ctl), A.ctl ? kCtlPrm : 0);
  const double v = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, uint32_t(i) * 8, 0, 0));
  return A.ctl ? v : arg;
}
__device__ __forceinline__ double arn_c(const ArnoldiArgs& A, int e) { return arn_prm(A, e, A.c[e]); }
__device__ __forceinline__ double arn_tau(const ArnoldiArgs& A) { return arn_prm(A, kArnMaxNV, A.tau); }
__device__ __forceinline__ double arn_alpha(const ArnoldiArgs& A) {
  return arn_prm(A, kArnMaxNV + 1, A.alpha);
}
__device__ __forceinline__ double arn_sc(const ArnoldiArgs& A) { return arn_prm(A, kArnMaxNV + 2, A.sc); }
// the control kernel handed the loop back to the host: the queued launch does nothing (read in
// the same batch as the parameters: one load latency at kernel start)
__device__ __forceinline__ bool arn_halted(const ArnoldiArgs& A) {
  return arn_prm(A, kArnMaxNV + 3, 0.0) != 0.0;
}

// Rows of loads in flight per wave for a basis of NV vectors (register budget at one or two
// waves per SIMD; the wait counter tracks at most 63 loads)
// (the pair layout runs nv >= 19, where one row in flight measured 2 % faster than two at nv 19-20:
// profiles/r02_arnoldi_ab.md)
constexpr int pf_for(int nv) { return nv <= 4 ? 3 : nv <= 18 ? 2 : 1; }

__device__ __forceinline__ double readlane(double v, int l) {
  const u32x2 b = __builtin_bit_cast(u32x2, v);
  u32x2 r;
  r.x = __builtin_amdgcn_readlane(b.x, l);
  r.y = __builtin_amdgcn_readlane(b.y, l);
  return __builtin_bit_cast(double, r);
}
// x[lane] + x[lane ^ 32], summed as (lanes 0-31) + (lanes 32-63) in every lane (bitwise equal
// in both halves), and x[lane ^ 32]: one v_permlane32_swap per 32-bit half
__device__ __forceinline__ void swap32(double x, double* lo, double* hi) {
  const u32x2 b = __builtin_bit_cast(u32x2, x);
  const auto a0 = __builtin_amdgcn_permlane32_swap(b.x, b.x, false, false);
  const auto a1 = __builtin_amdgcn_permlane32_swap(b.y, b.y, false, false);
  u32x2 l, h;
  l.x = a0[0];
  l.y = a1[0];
  h.x = a0[1];
  h.y = a1[1];
  *lo = __builtin_bit_cast(double, l);  // x of lane (lane & 31)
  *hi = __builtin_bit_cast(double, h);  // x of lane (lane | 32)
}
__device__ __forceinline__ double pair_sum(double x) {
  double lo, hi;
  swap32(x, &lo, &hi);
  return lo + hi;
}
// x of row (row & ~1) + x of row (row | 1) for the lane's 16-lane row (v_permlane16_swap)
__device__ __forceinline__ double pair16_sum(double x) {
  const u32x2 b = __builtin_bit_cast(u32x2, x);
  const auto a0 = __builtin_amdgcn_permlane16_swap(b.x, b.x, false, false);
  const auto a1 = __builtin_amdgcn_permlane16_swap(b.y, b.y, false, false);
  u32x2 l, h;
  l.x = a0[0];
  l.y = a1[0];
  h.x = a0[1];
  h.y = a1[1];
  return __builtin_bit_cast(double, l) + __builtin_bit_cast(double, h);
}
__device__ __forceinline__ double partner(double x, int hf) {
  double lo, hi;
  swap32(x, &lo, &hi);
  return hf ? lo : hi;
}
typedef double dv2 __attribute__((ext_vector_type(2)));
// 16-B global load (non-temporal: a once-streamed field), kept a global_load like gld()
typedef const dv2 __attribute__((address_space(1))) gdv2;
template <bool NT>
__device__ __forceinline__ dv2 gld2(const double* a) {
  gdv2* p = (gdv2*)a;
  if constexpr (NT) return __builtin_nontemporal_load(p);
  return *p;
}

// ------------------------------------------------------------------------------------------
// Mailbox: block halos exchanged between the blocks of a band instead of recomputed.
//
// A block's stencil needs u = v on the two columns either side of it, and v there is a sum over
// every update entry: recomputing it costs each block one packed halo load per row touching ~14
// distinct lines (the block-halo cost measured in profiles/r02_arnoldi_ab.md: a variant with no
// halo load ran 10 % faster).  But the neighbouring block of the same band computes exactly those
// values one iteration away, and one launch is one resident round of blocks whose bands sit on
// one XCD (the blockIdx mapping below), so it PUBLISHES them: per row, its lanes holding the
// block's first / last column pair store {u, tag} records (16 B each, device-coherent stores),
// and the consumer polls them one row later than it used to need them (the halo of row q only
// enters the window rows that the stencil centre reaches one iteration after row q is pushed:
// push stores the edge lanes' sums without it (adding -0.0, exact), fixup adds it, and since
// a + b == b + a the result is bitwise what the packed path computes from the same values).
// The tag (unique per launch) makes stale records from earlier launches invisible, so the
// buffer is never cleared.  A neighbour that is not there in time -- not resident, another
// XCD -- is waited for a bounded number of polls, after which the lane recomputes the pair
// itself, in the producer's exact summation order (same result bits), and stops polling for
// the rest of the launch: correctness never depends on co-residency.
// cache policy of the record loads / stores: sc1 (device scope; sc0 records were never visible
// in time, profiles/r02_arnoldi_ab.md)
constexpr uint32_t kMBCoh = 16;
constexpr int kMBSpin = 2048;     // polls before a lane recomputes a missing halo pair itself
#ifdef NKHIP_ARN_MBSTAT  // diagnostic build (`make mbstat`): what the mailbox consumers did
// [0] halo pairs needed, [1] not there at the first look, [2] extra polls, [3] recomputed
__device__ unsigned long long g_mb_stat[4];
#define MB_STAT(i, v) atomicAdd(&g_mb_stat[i], static_cast<unsigned long long>(v))
#else
#define MB_STAT(i, v) ((void)0)
#endif
__device__ __forceinline__ uint32_t mb_off(uint32_t blk, uint32_t T, uint32_t t, int side,
                                           int comp) {
  return (((blk * T + t) * 4) + uint32_t(side * 2 + comp)) * 16u;  // < mb_cap * 8 < 2^32
}
__device__ __forceinline__ bool mb_tag_ok(const u32x4& a, uint64_t tag) {
  return a.z == uint32_t(tag) && a.w == uint32_t(tag >> 32);
}
__device__ __forceinline__ double mb_val(const u32x4& a) {
  return __builtin_bit_cast(double, u32x2{a.x, a.y});
}
__device__ __forceinline__ u32x4 mb_rec(double v, uint64_t tag) {
  const u32x2 b = __builtin_bit_cast(u32x2, v);
  return u32x4{b.x, b.y, uint32_t(tag), uint32_t(tag >> 32)};
}

// lane i <- lane i-1 (wave_shr:1) and lane i <- lane i+1 (wave_shl:1); lanes 0 / 63 get 0
__device__ __forceinline__ double dpp_up(double x) {
  const u32x2 b = __builtin_bit_cast(u32x2, x);
  u32x2 r;
  r.x = __builtin_amdgcn_update_dpp(0u, b.x, 0x138, 0xF, 0xF, false);
  r.y = __builtin_amdgcn_update_dpp(0u, b.y, 0x138, 0xF, 0xF, false);
  return __builtin_bit_cast(double, r);
}
template <int N>  // lane i <- lane i-N inside its 16-lane row (row_shr:N); 0 past the row start
__device__ __forceinline__ double dpp_row_shr_t(double x) {
  const u32x2 b = __builtin_bit_cast(u32x2, x);
  u32x2 r;
  r.x = __builtin_amdgcn_update_dpp(0u, b.x, 0x110 + N, 0xF, 0xF, false);
  r.y = __builtin_amdgcn_update_dpp(0u, b.y, 0x110 + N, 0xF, 0xF, false);
  return __builtin_bit_cast(double, r);
}
#define dpp_row_shr(x, n) dpp_row_shr_t<n>(x)
__device__ __forceinline__ double dpp_down(double x) {
  const u32x2 b = __builtin_bit_cast(u32x2, x);
  u32x2 r;
  r.x = __builtin_amdgcn_update_dpp(0u, b.x, 0x130, 0xF, 0xF, false);
  r.y = __builtin_amdgcn_update_dpp(0u, b.y, 0x130, 0xF, 0xF, false);
  return __builtin_bit_cast(double, r);
}

// u = v (or z) at element o of the grid, summed in the fused kernel's order -- for the pair
// layout (h0 = 0) entries 0, 2, 4, .. of [V_0 .. V_{nv-1}, w] in one partial, 1, 3, 5, .. in the
// other, then their sum; for the wide layout (h0 = nv + 1) all entries in order -- so an edge row
// sent to a neighbour equals the row its owner computes.  Every entry load is in flight at once.
template <int NV>
__device__ __forceinline__ double edge_u(const ArnoldiArgs& A, int64_t o, int h0, double a_tau) {
  if (A.z) return A.z[o];
  constexpr int NE = NV + 1;
  double x[NE], cf[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    x[e] = ((e < NV) ? A.V[e] : A.w)[o];
    cf[e] = (e < NV) ? arn_c(A, e) : a_tau;
  }
  double p0 = 0.0, p1 = 0.0;
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    if ((h0 > 0) ? (e < h0) : ((e & 1) == 0))
      p0 = __builtin_fma(cf[e], x[e], p0);
    else
      p1 = __builtin_fma(cf[e], x[e], p1);
  }
  return p0 + p1;
}

// ------------------------------------------------------------------------------------------
// March direction.  A band of rows [r0, r1) also reads its two band-halo rows on either side
// (the stencil couples rows r-2 .. r+2): r0-2, r0-1 and r1, r1+1, every update entry of them.
// Those rows are the neighbouring bands' own rows, and marching every band down, a band reads
// its upper halo at its start while the band above reads the same rows at its END (and vice
// versa): a whole launch apart, so both reads come from HBM -- on short slabs 4 extra rows per
// band are a large share (a 512-row slab: PMC traffic 1.15x of algorithmic for the pair layout's
// 32-row bands, 1.22-1.39x for the wide layout's 8-16-row bands; profiles/r06a_slab512_kernels.txt).
// In the ALT instantiations (taken for bands of at most 32 rows, arnoldi_alt_mode) the even
// bands march UP their rows: two adjacent bands then reach their shared
// boundary at the same moment -- both at their start, or both at their end.  The bands of one XCD
// are a contiguous run starting at an even band (the blockIdx mapping below), so its boundaries
// 2b | 2b+1 are start-start ones, and the prologue loads its rows temporally (the interior stays
// non-temporal): the second read of each shared row then hits the XCD's L2.  (Temporal loads for
// the end rows as well would need a second copy of the row loop; its register allocation spilled.)
// The kernels run over a logical row index t (prow(t): physical row), so a band's every
// computation is the same in either direction: v and w' are bitwise the same (the stencil adds
// the two rows either side of the centre as a + b == b + a), only the order in which a wave
// accumulates its rows' dot products changes.  Measured in profiles/r06_short_slab.md.
// ------------------------------------------------------------------------------------------
// Slab exchange inside the fused kernel (row slabs over the peer-memory communicator, A.x.me set;
// peer_dev.h holds the buffer layout).  A slab's stencil needs u on the neighbours' two edge rows,
// and u of a row needs only the basis, not the stencil: so the blocks of the FIRST band compute u
// on the slab's rows 0, 1 for their own columns and write it straight into the previous rank's
// "hi" staging rows, the blocks of the LAST band do the same with rows ny-2, ny-1 into the next
// rank's "lo" rows; each then publishes one flag per 128-column chunk it wrote (tagged, release,
// system scope) and waits for the chunks its own halo columns need in its own buffer (its
// columns plus two either side) before its march starts.  Publishing never waits, so there is no
// cycle; the interior bands (all but two per column group) never wait at all, which is the
// overlap: the exchange runs beside the interior of the pass instead of before it (the edge
// kernel + halo kernel in series, ~22 us per Arnoldi step).  The halo rows are then read from
// this rank's staging rows (A.yh, row stride A.yh_ld).  A wait that gives up (abort, timeout) sets
// the communicator's error word; the host sees it at its next synchronisation.
template <int NV>
__device__ __forceinline__ void slab_x_exchange(const ArnoldiArgs& A, int64_t band, int64_t B0, int64_t BW, int h0,
                                double a_tau, bool top, bool bot) {
  const SlabX& X = A.x;
  const int64_t nx = A.nx, ny = A.ny;
  const bool first = band == 0, last = band == int64_t(A.nbands) - 1;
  const int par = int(X.tag & 1);
  const int64_t cend = (B0 + BW < nx) ? B0 + BW : nx;  // own columns [B0, cend)
  for (int side = 0; side < 2; ++side) {  // side 0: my rows 0, 1 -> prev; 1: ny-2, ny-1 -> next
    if (side == 0 ? !first : !last) continue;
    char* dst = side == 0 ? X.prev : X.next;
    const int dside = side == 0 ? 1 : 0;  // the receiver's "hi" / "lo" staging rows
    for (int rr = 0; rr < 2; ++rr) {
      const int64_t row = side == 0 ? rr : ny - 2 + rr;
      for (int64_t j = B0 + threadIdx.x; j < cend; j += blockDim.x) {
        ARN_CHK(j < X.max_nx && row * nx + j < ny * nx);
        stage(dst, X.P, X.max_nx, par, dside, rr)[j] = edge_u<NV>(A, row * nx + j, h0, a_tau);
      }
    }
    __threadfence_system();
    __syncthreads();
    // one flag per chunk this block wrote (B0 and BW are multiples of kXChunk)
    for (int64_t ch = B0 / kXChunk + threadIdx.x; ch * kXChunk < cend; ch += blockDim.x) {
      ARN_CHK(ch < x_chunks(X.max_nx));
      __hip_atomic_store(xflag(dst, X.P, X.max_nx, par, dside, ch), X.tag, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  // the chunks my halo columns come from, in my buffer: side 0 ("lo", from prev) for the first
  // band, side 1 ("hi", from next) for the last; chunks of columns B0-2, [B0, cend), B0+BW
  const int64_t nch = (nx + kXChunk - 1) / kXChunk;
  const int64_t cl = ((B0 - 2 + nx) % nx) / kXChunk, c0 = B0 / kXChunk;
  const int64_t c1 = (cend - 1) / kXChunk, cr = ((B0 + BW) % nx) / kXChunk;
  const int64_t nown = c1 - c0 + 1;
  // every band whose stencil reaches a halo row waits for it (`top`: rows -2, -1; `bot`: rows ny,
  // ny+1), not only the first and last: a last band of one row leaves row ny to the band before
  for (int side = 0; side < 2; ++side) {
    if (side == 0 ? !top : !bot) continue;
    const int t = int(threadIdx.x);
    if (t < nown + 2) {
      const int64_t ch = (t == 0) ? cl : ((t == 1) ? cr : c0 + (t - 2));
      ARN_CHK(ch >= 0 && ch < nch);
      (void)wait_flag_tag(xflag(X.me, X.P, X.max_nx, par, side, ch), X.tag, X.me, X.err,
                          X.wait_ticks);
    }
  }
  __syncthreads();
  __atomic_thread_fence(__ATOMIC_ACQUIRE);  // the staged rows, for every thread of the block
}

// ------------------------------------------------------------------------------------------
// Pushed halo rows (row slabs over the peer-memory communicator, A.hs_ld > 0).  A slab's stencil
// needs u on the neighbours' two edge rows, and u of a row is the update sum over the entries
// [V_0 .. V_{nv-1}, w] (or z) of that row -- entries the neighbours produced in EARLIER launches.
// So every producer of an entry writes the entry's own edge rows into its ring neighbours' halo
// slots as a by-product (this kernel for its outputs v and w', the stencil passes and
// combinations through push_rows_launch), written through to the slot (store_sys16, peer_dev.h)
// and drained by the producer, with no fence and no flag: the all-reduce
// that every rank passes between producing an entry and the next fused launch (the device
// control's, or the host path's) orders the writes before this launch on every rank, and a slot
// is rewritten only when its pool vector gets new content, steps after its last reader (the same
// all-reduces order that).  Here the blocks of the first band compute u on rows -2, -1 and those
// of the last band on rows ny, ny+1 from the slots -- their own columns and the two halo columns
// either side, in the update's summation order (edge_u, bitwise the owner's v) -- into A.yh, then
// march as with exchanged halo rows.  No exchange runs between the control and this launch, and
// no block waits for another rank.  (A halo column shared with the neighbouring block is written
// by both with the same bits.)
template <int NV>
__device__ __forceinline__ void slab_push_prologue(const ArnoldiArgs& A, bool first, bool last, int64_t B0,
                                   int64_t BW, int h0, const double* cst, double a_tau) {
  const int64_t nx = A.nx, ld = A.hs_ld;
  double* yh = const_cast<double*>(A.yh);  // 4 rows of nx (yh_ld == nx), this launch's scratch
  constexpr int NE = NV + 1;
  // (row, column) items per thread and round: each round's loads are in flight together (one
  // memory latency); 2 x NE values stay below the march's register peak, so the prologue does
  // not raise the kernel's register count (and with it lower its occupancy).  (Round 6: one
  // round for all of a block's 2 (BW + 4) items measured no faster, and the larger prologue
  // tipped the compiler into wrong code for the wide EXT kernels, profiles/r06_short_slab.md 8)
  constexpr int KMAX = 2;
  const int64_t ncol = BW + 4;  // columns B0-2 .. B0+BW+1 of the two halo rows
  const int64_t nb = blockDim.x, items = 2 * ncol;
  for (int side = 0; side < 2; ++side) {
    if (side == 0 ? !first : !last) continue;
#pragma unroll 1
    for (int64_t base = 0; base < items; base += KMAX * nb) {
      int64_t off[KMAX], yo[KMAX];
      bool on[KMAX];
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        const int64_t i = base + threadIdx.x + k * nb;
        on[k] = i < items;
        const int64_t rr = (i >= ncol) ? 1 : 0;
        const int64_t j = ((B0 - 2 + (i - rr * ncol)) % nx + nx) % nx;
        const int64_t hrow = 2 * side + rr;  // slot / yh row: 0, 1 = rows -2, -1; 2, 3 = ny, ny+1
        off[k] = on[k] ? CI(hrow * ld + j, 4 * ld) : 0;
        yo[k] = on[k] ? CI(hrow * nx + j, 4 * nx) : 0;
      }
      double u[KMAX];
      if (A.z) {
#pragma unroll
        for (int k = 0; k < KMAX; ++k) u[k] = A.HS[NV + 1][off[k]];
      } else {
        double x[KMAX][NE];
#pragma unroll
        for (int e = 0; e < NE; ++e)
#pragma unroll
          for (int k = 0; k < KMAX; ++k) x[k][e] = A.HS[e][off[k]];
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
          double p0 = 0.0, p1 = 0.0;
#pragma unroll
          for (int e = 0; e < NE; ++e) {
            const double cf = (e < NV) ? cst[e] : a_tau;
            if ((h0 > 0) ? (e < h0) : ((e & 1) == 0))
              p0 = __builtin_fma(cf, x[k][e], p0);
            else
              p1 = __builtin_fma(cf, x[k][e], p1);
          }
          u[k] = p0 + p1;
        }
      }
#pragma unroll
      for (int k = 0; k < KMAX; ++k)
        if (on[k]) yh[yo[k]] = u[k];
    }
  }
  __threadfence_block();
  __syncthreads();
}

// v (or w') of own row q into the neighbours' halo slots when q is one of the slab's edge rows
// (ps[0]: the previous rank's slot, rows 2, 3 <- rows 0, 1; ps[1]: the next rank's, rows 0, 1 <-
// rows ny-2, ny-1); `st`: this lane stores row q (wave-uniform row, per-lane column); written
// through to the slot (store_sys16), drained at the band's end
__device__ __forceinline__ void push_edge_row(double* const* ps, int64_t ld, int64_t q,
                                              int64_t ny, int64_t col, bool st, dv2 val) {
  const bool top = q < 2, bot = q >= ny - 2;
  if (!(st && (top || bot))) return;
  double* d = top ? ps[0] + (2 + q) * ld : ps[1] + (q - (ny - 2)) * ld;
  ARN_CHK(col + 1 < ld);
  store_sys16(d + col, val.x, val.y);
}

// 32-bit row / column indices of the pair kernel's row loop, and a uniform value the compiler
// must keep (an SGPR, or a VGPR lane when it spills) instead of re-reading it from the kernel
// arguments
typedef int ix_t;
// ARN_OPQ 1 (default) pins the 32-bit grid scalars; 0: none.  A level 2 that also pinned the
// stencil coefficients and the x0 pointer through "+s" constraints on doubles / pointers is gone:
// its bounds-checked build of the round-5 kernel returned w' scaled by one constant (1.5e-9 x the
// true value) on every row of each band but the first, v exact, at nv 25 -- the loop-invariant FD
// scale read wrongly after the row loop's first iteration, identically with no mailbox record ever
// polled (NKHIP_ARN_MBOX=2) and with zero out-of-range indices: a code-generation fault of that
// instantiation, not a race (round 6, scripts/dbg/opq2_probe.py, opq2_pattern.py)
#ifndef ARN_OPQ
#define ARN_OPQ 1
#endif
#if ARN_OPQ > 1
#error "ARN_OPQ 2 (pinned coefficients and x0) is removed: see the note above"
#endif
template <bool PIN = true>
__device__ __forceinline__ int opaque_s(int x) {
  x = __builtin_amdgcn_readfirstlane(x);
  if constexpr (PIN && ARN_OPQ >= 1) asm volatile("" : "+s"(x));
  return x;
}
// the basis lengths whose kernels pin them: not nv >= 34, at the register limit (n35 spills
// either way, and 6 % slower with the scalars pinned; round 5, profiles/r05_arnoldi_short_end.md)
template <int NV>
constexpr bool kPinScalars = NV <= 33;

// Lane layout ("vector pairs"): a wave owns 64 aligned columns; lane l of half hf (lane = 32 hf + l)
// holds columns 2l, 2l+1 (one 16-B load) of entry 2k + hf of the row's load list
//   [V_0 .. V_{NV-1}, w, x0, (z)]
// in load k, so every load instruction streams two 512-B row segments of two vectors.  The update
// sums each half's entries and adds the other half's sum (v_permlane32_swap); both halves then
// hold v, y and w' of the wave's 64 columns, and each half takes the dot products of its own
// entries (half 0 also w'.v, v.v, w'.w').
// ------------------------------------------------------------------------------------------
// Tail (device-side Arnoldi control, ArnoldiArgs::tail): the reduction + control launch that
// would follow a fused launch, run by its last blocks instead (no kernel boundary in between).
// Every active block counts in after writing its partial columns; the last kTailR to do so wait
// until all have -- at most kTailR blocks wait, and every other block of the grid is running or
// done (a launch is one resident round of blocks), so the wait ends -- and each reduces every
// kTailR-th value over all partial columns in a fixed order (the same sums whichever blocks come
// last).  The last reducer resets the counters, on a row slab all-reduces the values over the
// peer-memory communicator, and runs the control of step t with its first wave, on the block's
// LDS lag (free once the march is over) as the control's scratch.  A reducer that waits longer
// than kTailWait gives up: the control never runs, and the host's wait for its status word ends
// in an error (a fault, not a path this protocol takes): the reducer sets the halt word (the
// queued launches do nothing) and, on a slab, the communicator's error word.  The wait bound is
// ArnTail::wait_ticks (device_wait_ticks, from the wall-clock rate); device_steps resets the
// arrival counters before every run of device steps, so a launch that gave up leaves no count
// behind for the next run.
// (st_sc1 / ld_sc1 / drain_stores: nk_device.h)

#ifdef ARN_TAIL_PROBE  // timing build (scripts/dbg/tail_probe.py): stage times of the tails
__device__ unsigned long long g_tail_probe[8];  // [0] tails, [1..5] summed stage ticks
__device__ unsigned long long g_tail_first;     // wall clock of the current launch's first arrival
// a tail that gave up: [0] 1 = its own blocks' arrival, 2 = the peer all-reduce; [1] blocks
// arrived / [2] of total when it gave up; [3] bit q = peer q's contribution missing; [4] ticks
// from the launch's first arrival to the give-up; [5] tails that gave up
__device__ unsigned long long g_tail_diag[8];
#endif
constexpr int kTailR = 8;
constexpr int kTailC = (2 * kArnMaxNV + 3 + kTailR - 1) / kTailR;  // values per reducer
template <int BS>
__device__ __forceinline__ void arn_tail(const ArnoldiArgs& A, int64_t nblocks, double (*G)[kArnMaxNV + 1]) {
  const ArnTail& T = A.tail;
  __shared__ uint32_t ticket;
  __shared__ bool ok;
  __shared__ double redl[2 * kArnMaxNV + 3];  // the controller's copy of the step's values
  drain_stores();  // this wave's partial columns (sc1 stores) have landed
  __syncthreads();
  if (threadIdx.x == 0)
    ticket = __hip_atomic_fetch_add(&T.S->arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
#ifdef ARN_TAIL_PROBE
  const uint64_t p_arr = wall_clock64();
  if (threadIdx.x == 0 && ticket == 0) g_tail_first = p_arr;
#endif
  const uint32_t total = uint32_t(nblocks);
  const uint32_t R = total < uint32_t(kTailR) ? total : uint32_t(kTailR);
  if (ticket < total - R) return;
  const int rid = int(ticket - (total - R));
  if (threadIdx.x == 0) {
    const uint64_t t0 = wall_clock64();
    bool in = true;
    while (__hip_atomic_load(&T.S->arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < total) {
      if (wall_clock64() - t0 > T.wait_ticks) {
        in = false;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    ok = in;
  }
  __syncthreads();
  if (!ok) {  // a fault, not a path of this protocol: halt the queued launches and report it
#ifdef ARN_TAIL_PROBE
    if (threadIdx.x == 0) {
      g_tail_diag[0] = 1;
      g_tail_diag[1] = __hip_atomic_load(&T.S->arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      g_tail_diag[2] = total;
      g_tail_diag[4] = wall_clock64() - g_tail_first;
      atomicAdd(&g_tail_diag[5], 1ull);
    }
#endif
    if (threadIdx.x == 0) {
      st_sc1(T.prm + kArnMaxNV + 3, 1.0);
      if (T.peer && T.pa.err)
        __hip_atomic_store(T.pa.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    return;
  }
#ifdef ARN_TAIL_PROBE
  const uint64_t p_all = wall_clock64();
#endif
  // values rid, rid + R, ..: each thread sums its columns of kTailC of them at a time (one round
  // unless the grid has fewer than kTailR blocks), four columns per value in flight per iteration
  const int64_t nw = A.pstride;
  for (int q0 = 0, round = 0; rid + q0 * int(R) < T.nval; q0 += kTailC, ++round) {
    double acc[kTailC];
#pragma unroll
    for (int q = 0; q < kTailC; ++q) acc[q] = 0.0;
    int64_t b = threadIdx.x;
    for (; b + 3 * BS < nw; b += 4 * BS) {
      double x[kTailC][4];
#pragma unroll
      for (int q = 0; q < kTailC; ++q) {
        const int c = rid + (q0 + q) * int(R);
        const double* p = A.partial + int64_t(c < T.nval ? c : 0) * nw + b;
#pragma unroll
        for (int u = 0; u < 4; ++u) x[q][u] = (c < T.nval) ? ld_sc1(p + u * BS) : 0.0;
      }
#pragma unroll
      for (int q = 0; q < kTailC; ++q) acc[q] += ((x[q][0] + x[q][1]) + (x[q][2] + x[q][3]));
    }
    for (; b < nw; b += BS) {
#pragma unroll
      for (int q = 0; q < kTailC; ++q) {
        const int c = rid + (q0 + q) * int(R);
        acc[q] += (c < T.nval) ? ld_sc1(A.partial + int64_t(c) * nw + b) : 0.0;
      }
    }
    const double s = block_reduce<kTailC, kTailC, BS>(acc, round & 1);
    if (threadIdx.x < kTailC) {
      const int c = rid + (q0 + int(threadIdx.x)) * int(R);
      if (c < T.nval) st_sc1(T.result + c, s);
    }
  }
  drain_stores();
  __syncthreads();
  if (threadIdx.x == 0)
    ok = __hip_atomic_fetch_add(&T.S->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == R - 1;
  __syncthreads();
  if (!ok || threadIdx.x >= 64) return;
  // the controller (one wave): every reducer's values, sc1 loads into LDS
  const int lane = threadIdx.x;
  for (int i = lane; i < T.nval; i += 64) redl[i] = ld_sc1(T.result + i);
  if (lane == 0) {  // for the next launch (stream order)
    __hip_atomic_store(&T.S->arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&T.S->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
#ifdef ARN_TAIL_PROBE
  const uint64_t p_red = wall_clock64();
#endif
  if (T.peer) {
    if (!peer_allreduce_wave(T.pa, redl, T.nval, T.nval)) {
#ifdef ARN_TAIL_PROBE
      {  // which peers' contributions never came (their flags in my buffer)
        const int par = int(T.pa.tag & 1);
        for (int q = lane; q < T.pa.P; q += 64)
          if (__hip_atomic_load(red_flag(T.pa.base[T.pa.rank], par, q), __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_SYSTEM) != T.pa.tag)
            atomicOr(&g_tail_diag[3], 1ull << q);
        if (lane == 0) {
          g_tail_diag[0] = 2;
          g_tail_diag[4] = wall_clock64() - g_tail_first;
          atomicAdd(&g_tail_diag[5], 1ull);
        }
      }
#endif
      if (lane == 0) T.prm[kArnMaxNV + 3] = 1.0;  // the queued fused step does nothing
      return;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    for (int i = lane; i < T.nval; i += 64) T.result[i] = redl[i];  // the combined values
  }
#ifdef ARN_TAIL_PROBE
  const uint64_t p_ar = wall_clock64();
#endif
  ctl_body(T.S, T.H, redl, T.result_host, T.prm, T.status, T.t, G);
#ifdef ARN_TAIL_PROBE
  const uint64_t p_end = wall_clock64();
  if (threadIdx.x == 0) {
    const uint64_t f = g_tail_first;
    atomicAdd(&g_tail_probe[0], 1ull);
    atomicAdd(&g_tail_probe[1], (unsigned long long)(p_arr - f));  // first -> this block's arrival
    atomicAdd(&g_tail_probe[2], (unsigned long long)(p_all - p_arr));  // -> all arrived
    atomicAdd(&g_tail_probe[3], (unsigned long long)(p_red - p_all));  // -> all reduced
    atomicAdd(&g_tail_probe[4], (unsigned long long)(p_ar - p_red));   // -> all-reduced
    atomicAdd(&g_tail_probe[5], (unsigned long long)(p_end - p_ar));   // -> control done
  }
#endif
}

template <int NV, bool EXT, int PF, bool ALT, bool MB, int WB>
__global__ void __launch_bounds__(64 * WB) arnoldi_kernel(const ArnoldiArgs A) {
  const double a_tau = arn_tau(A), a_alpha = arn_alpha(A), a_sc = arn_sc(A);
  double cst[NV];  // update coefficients, loaded together (independent loads, one wait)
#pragma unroll
  for (int e = 0; e < NV; ++e) cst[e] = arn_c(A, e);
  if (arn_halted(A)) return;
  constexpr int RR = PF + 1;               // register ring: the update row and PF rows in flight
  constexpr int NE = NV + 2 + (EXT ? 1 : 0);
  constexpr int NI = (NE + 1) / 2;         // 16-B loads per row and lane
  constexpr int NB = (NV + 1) / 2;         // loads holding basis entries
  constexpr int EX = NV + 1, EZ = NV + 2;  // entries of x0, z
  // lag rows r, r+1 of this lane's basis entries and of x0, for row r's dot products / stencil
  __shared__ dv2 lag[WB][2][NB + 1][64];
  // per row (parity slot): u on columns 0, 1, 62, 63 of every wave; the waves' partial sums of v
  // on the block's four halo columns
  __shared__ double edge[2][WB][4];
  __shared__ double hpart[2][WB][4];
  const int lane = threadIdx.x & 63;
  const int hf = lane >> 5, l = lane & 31;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // XCD-aware mapping: consecutive blocks go round-robin over the 8 XCDs; give each XCD one
  // contiguous run of blocks (whole bands), so band halos are shared inside one L2.
  const ix_t b = blockIdx.x;
  const ix_t bpx = gridDim.x / 8;  // grid is a multiple of 8
  const ix_t L = (b % 8) * bpx + b / 8;
  const ix_t ngroups = (A.strips + WB - 1) / WB;  // a block = WB adjacent strips
  if (L >= ngroups * A.nbands) return;                 // whole blocks only
  const ix_t band = L / ngroups, grp = L % ngroups;
  const ix_t gw = L * WB + wid;  // partial-sum column of this wave
  // row and column arithmetic in 32 bits (ny * nx * 8 < 2^32, arnoldi_supported), the grid
  // scalars opaque: the compiler keeps them in registers instead of reloading them from the
  // kernel arguments inside the row loop (every such reload is a scalar load whose lgkmcnt wait
  // also drains the wave's LDS queue; ~20 per row at nv 19-24 before)
  const ix_t nx = opaque_s<kPinScalars<NV>>(ix_t(A.nx));
  const ix_t ny = opaque_s<kPinScalars<NV>>(ix_t(A.ny));
  const ix_t B0 = grp * WB * kSW;        // the block's first column
  const ix_t c = B0 + wid * kSW + 2 * l;  // columns past nx compute wrapped columns, masked
  const ix_t col = c % nx;                // nx even: c and c+1 wrap together
  const bool own = c < nx;
  // block halo: h = 0, 1 -> columns B0-2, B0-1; h = 2, 3 -> B0 + WB*64, +1
  const int hh = lane & 3;
  const ix_t hc = (hh < 2) ? B0 - 2 + hh : B0 + WB * kSW - 2 + hh;
  const ix_t hcol = ((hc % nx) + nx) % nx;
  const ix_t rend = (A.r_end >= 0) ? ix_t(A.r_end) : ny;
  const ix_t r0 = opaque_s<kPinScalars<NV>>(ix_t(A.r_begin) + band * A.RY);
  const ix_t r1 = opaque_s<kPinScalars<NV>>((r0 + A.RY < rend) ? r0 + A.RY : rend);
  const ix_t nrows = r1 - r0;
  // march direction ("March direction" above): logical row t of the band is physical row
  // rb + rs t -- r0 + t marching down, r1 - 1 - t marching up (the even bands of an ALT
  // instantiation)
  const bool dn = !ALT || (band & 1) == 1;
  const ix_t rb = opaque_s<kPinScalars<NV>>(dn ? r0 : r1 - 1);
  const ix_t rs = dn ? 1 : -1;
  using NTc = std::integral_constant<bool, true>;   // the row loop: non-temporal
  using TMc = std::integral_constant<bool, !ALT>;   // the prologue: temporal under ALT
  const SHCoef K = A.k;
  const double isc = 1.0 / a_sc;
  const __amdgpu_buffer_rsrc_t rv = rsrc(A.out_v, ny * nx);
  const __amdgpu_buffer_rsrc_t rw = rsrc(A.out_w, ny * nx);
  dv2 (*lg)[NB + 1][64] = lag[wid];

  auto src = [&](int e) -> const double* {
    if (e < NV) return A.V[e];
    if (e == NV) return A.w;
    if (e == EX) return A.x0;
    return EXT ? A.z : A.x0;
  };
  auto cof = [&](int e) -> double { return e < NV ? cst[e] : (e == NV ? a_tau : 0.0); };
  // per-lane source of load k (entry 2k + hf) and its update coefficient; the padding entry
  // (NE odd) repeats the other half's address with coefficient 0
  const double* ep[NI];
  double ecf[NI];
#pragma unroll
  for (int k = 0; k < NI; ++k) {
    const int e0 = 2 * k, e1 = (2 * k + 1 < NE) ? 2 * k + 1 : 2 * k;
    ep[k] = hf ? src(e1) : src(e0);
    ecf[k] = hf ? (2 * k + 1 < NE ? cof(e1) : 0.0) : cof(e0);
  }
  // packed block-halo loads (8 B per lane), shared by the WB waves: lane L of wave w fetches
  // halo column L%4 of entry e = w + WB*(L/4) of [V_0 .. V_{NV-1}, w] with coefficient c_e (tau
  // for w); lanes past the list repeat entry w's address (same line) with coefficient 0
  const double* hp;
  double hcf;
  {
    const int e = wid + WB * (lane >> 2);
    const double* p = (wid < NV) ? A.V[wid < NV ? wid : 0] : A.w;
    double cf = 0.0;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      p = (e == j) ? A.V[j] : p;
      cf = (e == j) ? cst[j] : cf;
    }
    p = (e == NV) ? A.w : p;
    cf = (e == NV) ? a_tau : cf;
    hp = p;
    hcf = cf;
  }
  // the same entry's edge array (its left pair at boundary grp, its right pair at grp + 1)
  const bool useE = A.E[0] != nullptr;
  const double* hE;
  {
    const int e = wid + WB * (lane >> 2);
    const double* p = A.E[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) p = (e == j) ? A.E[j] : p;
    hE = p;
  }
  const ix_t grpR = (grp + 1 < ngroups) ? grp + 1 : 0;
  // edge-array stores of the outputs: the lane holding columns B, B+1 of a boundary B writes
  // them as E[b][q][2..3]; the lane holding B-2, B-1 as E[b][q][0..1] (b = 0 for nx - 2, nx - 1)
  const ix_t nbE = edge_groups(nx);  // (the 2-wave mailbox blocks are narrower than a group)
  const ix_t nelem = ny * nx, eelem = edge_elems(ny, nx);
  const bool eL = own && (c % kEdgeW == 0);
  const bool eR = own && ((c + 2) % kEdgeW == 0 || c + 2 == nx);
  const ix_t ebo =
      eL ? (c / kEdgeW) * 4 + 2 : (eR ? ((c + 2 == nx) ? 0 : (c + 2) / kEdgeW) * 4 : 0);
  const bool eOn = eL || eR;
  const __amdgpu_buffer_rsrc_t rEv = rsrc(A.Eout_v, A.Eout_v ? nbE * ny * 4 : 0);
  const __amdgpu_buffer_rsrc_t rEw = rsrc(A.Eout_w, A.Eout_w ? nbE * ny * 4 : 0);
  // byte offset of this lane's edge pair at row q (kOOB: nothing to store)
  auto eoff = [&](ix_t q) -> uint32_t {
    return eOn ? uint32_t(CI((ebo / 4) * ny * 4 + q * 4 + (ebo & 3), eelem - 1) * 8) : kOOB;
  };
  const double* x0p = A.x0;
  const double* hxp = (EXT && lane >= 4) ? A.z : x0p;  // lanes 0-3: x0 halo, 4-7: z halo
  // row slab: rows -2, -1, ny, ny+1 are the neighbours' -- their u arrives in A.yh (the x0 entry
  // and the x0 halo lanes read it there in place of x0)
  const bool slab = A.yh != nullptr;
  const double* yhb = slab ? A.yh : A.x0;
  const ix_t yld = (A.yh_ld > 0) ? A.yh_ld : nx;  // row stride of the halo rows

  // physical row of logical row t (past the band halo: its last row, re-read), -2 .. ny + 1
  auto prow = [&](ix_t t) -> ix_t {
    t = (t > nrows + 1) ? nrows + 1 : t;
    return rb + rs * t;
  };
  auto wrap = [&](ix_t t) -> ix_t {  // ... periodic
    const ix_t q = prow(t);
    return (q < 0) ? q + ny : ((q >= ny) ? q - ny : q);
  };
  // a neighbour slab's halo row (u taken from A.yh)
  auto halo_row = [&](ix_t t) -> bool {
    const ix_t qc = prow(t);
    return slab && (qc < 0 || qc >= ny);
  };

  // mailbox (see "Mailbox" above): wave 0's lanes l == 0 hold the block's first column pair and
  // need its left halo pair, wave WB-1's lanes l == 31 its last pair and the right halo pair
  constexpr int BW = WB * kSW;
  constexpr bool mb = MB && !EXT;  // a separate instantiation: the plain one has none of it
  const ix_t mbT = A.RY + 8;             // records per block and side (rows pushed <= RY + 7)
  const __amdgpu_buffer_rsrc_t rmb = rsrc(A.mb, mb ? A.mb_cap : 0);
  const uint64_t tag = A.mb_tag;
  const bool needL = mb && wid == 0 && l == 0, needR = mb && wid == WB - 1 && l == 31;
  const ix_t Lnb = band * ngroups + (needL ? (grp + ngroups - 1) % ngroups : (grp + 1) % ngroups);
  const int nside = needL ? 1 : 0;  // my left halo = the left neighbour's right-edge records
  const bool prod = mb && ((wid == 0 && lane == 0) || (wid == WB - 1 && lane == 31));
  const int pside = (wid == 0 && lane == 0) ? 0 : 1;
  const ix_t fcol = needL ? (B0 - 2 + nx) % nx : (B0 + BW) % nx;  // the halo pair's columns
  // this lane stopped polling (a neighbour was not there in time; mb_recompute: test switch)
  bool mb_dead = A.mb_recompute;
  auto mb_need = [&](ix_t t) -> bool { return (needL || needR) && !halo_row(t); };
  auto poll = [&](ix_t t, u32x4* a, u32x4* b) {  // issue the two record loads of row t
    const bool on = mb_need(t) && !mb_dead;
    const uint32_t o = mb_off(Lnb, mbT, t + 2, nside, 0);
    ARN_CHK(!on || (t + 2 >= 0 && t + 2 < mbT && int64_t(o) + 32 <= A.mb_cap * 8));
    *a = __builtin_amdgcn_raw_buffer_load_b128(rmb, on ? o : kOOB, 0, kMBCoh);
    *b = __builtin_amdgcn_raw_buffer_load_b128(rmb, on ? o + 16 : kOOB, 0, kMBCoh);
  };
  // the producer's value of the halo pair, recomputed in its summation order (rare path)
  // (a rolled loop with uniform entry indices: few registers beside the march's live state)
  auto ent = [&](int e) -> const double* {
    return e < NV ? A.V[e] : (e == NV ? A.w : ((e == EX || !EXT) ? A.x0 : A.z));
  };
  auto cfd = [&](int e) -> double { return e < NV ? arn_c(A, e) : (e == NV ? a_tau : 0.0); };
  auto recompute = [&](ix_t t) -> dv2 {
    const ix_t o2 = CI(wrap(t) * nx + fcol, nelem - 1);
    double p0x = 0.0, p0y = 0.0, p1x = 0.0, p1y = 0.0;
#pragma unroll 1
    for (int k = 0; k < NI; ++k) {
      const bool two = 2 * k + 1 < NE;
      const int e0 = 2 * k, e1 = two ? 2 * k + 1 : 2 * k;
      const dv2 x = gld2<false>(ent(e0) + o2), y = gld2<false>(ent(e1) + o2);
      const double c0 = cfd(e0), c1 = two ? cfd(e1) : 0.0;
      p0x = __builtin_fma(c0, x.x, p0x);
      p0y = __builtin_fma(c0, x.y, p0y);
      p1x = __builtin_fma(c1, y.x, p1x);
      p1y = __builtin_fma(c1, y.y, p1y);
    }
    return dv2{p0x + p1x, p0y + p1y};
  };
  // the halo pair of row q (-0.0 where the lane needs none: adding it changes nothing)
  auto mb_halo = [&](ix_t t, u32x4 a, u32x4 b) -> dv2 {
    const bool need = mb_need(t);
    bool ok = !need || (!mb_dead && mb_tag_ok(a, tag) && mb_tag_ok(b, tag));
    if (need) MB_STAT(0, 1);
    dv2 h{mb_val(a), mb_val(b)};
    if (!ok) {  // the neighbour is behind (or was not there): poll, then recompute
      MB_STAT(1, 1);
      const uint32_t o = mb_off(Lnb, mbT, t + 2, nside, 0);
      int n = 0;
      for (; n < kMBSpin && !mb_dead && !ok; ++n) {
        __builtin_amdgcn_s_sleep(2);
        a = __builtin_amdgcn_raw_buffer_load_b128(rmb, o, 0, kMBCoh);
        b = __builtin_amdgcn_raw_buffer_load_b128(rmb, o + 16, 0, kMBCoh);
        ok = mb_tag_ok(a, tag) && mb_tag_ok(b, tag);
      }
      MB_STAT(2, n);
      if (ok) {
        h = dv2{mb_val(a), mb_val(b)};
      } else {
        MB_STAT(3, 1);
        mb_dead = true;
        h = recompute(t);
      }
    }
    return need ? h : dv2{-0.0, -0.0};
  };

  struct Slot {
    dv2 e[NI];
    double hv;
    double hx;
    bool own;  // row of this slab (false: a neighbour's halo row, u taken from A.yh)
  };
  // pol: the streamed loads' cache policy -- NTc (non-temporal) in the row loop, TMc in the
  // prologue (temporal in the ALT instantiation: its rows are read by the neighbouring band as
  // well, "March direction").  A compile-time choice: a runtime select between the two load
  // forms is merged into one plain load (the non-temporal hint dropped)
  auto load = [&](Slot& s, ix_t t, auto pol) {
    const ix_t qq = wrap(t);
    const ix_t o = CI(qq * nx + col, nelem - 1);
    const ix_t qc = prow(t);  // the row wrap() reads (-2 <= qc <= ny + 1)
    const bool hrow = halo_row(t);
    const ix_t hq = hrow ? ((qc < 0) ? qc + 2 : qc - ny + 2) : 0;  // row of A.yh, 0..3
    const ix_t yo = CI(hq * yld + col, 4 * yld - 1);
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      const double* a = ep[k] + o;
      if (k == EX / 2) a = (hrow && hf == (EX & 1)) ? yhb + yo : a;
      s.e[k] = gld2<decltype(pol)::value>(a);
    }
    const ix_t ho = CI(qq * nx + hcol, nelem);
    // block halo: from the entry's edge array (four rows per line) or from the vector itself;
    // with the mailbox a load of one fixed line (keeps the row's load batch the same shape)
    if constexpr (!EXT && !mb) {
      const ix_t eo = CI(useE ? ((((hh < 2) ? grp : grpR) * ny + qq) << 2) + hh : 0, eelem);
      s.hv = gld(useE ? hE + eo : hp + ho);
    }
    // z on the halo columns (EXT, lanes 4..); u of a slab halo row (A.yh, lanes 0-3); every
    // other lane one fixed line of x0 (not of A.yh: the halo rows may sit in uncached peer memory)
    const ix_t hyo = CI(hq * yld + hcol, 4 * yld);
    s.hx = gld((hrow && lane < 4) ? yhb + hyo : (mb ? x0p : hxp + ho));
    s.own = !hrow;
  };
  // entry e of this row for both halves (e is a compile-time index)
  auto both = [&](const Slot& s, int e) -> dv2 {
    const dv2 x = s.e[e / 2];
    // the swaps run in every lane (a cross-lane read from lanes a branch switched off returns
    // stale registers), then each half selects
    const double px = partner(x.x, hf), py = partner(x.y, hf);
    const bool mine = hf == (e & 1);
    return dv2{mine ? x.x : px, mine ? x.y : py};
  };
  // the basis entries and x0 of row t wait in LDS slot t & 1 until row t's dot products
  auto stash = [&](const Slot& s, const dv2& g, ix_t t) {
    dv2 (*d)[64] = lg[t & 1];
#pragma unroll
    for (int k = 0; k < NB; ++k) d[k][lane] = s.e[k];
    d[NB][lane] = g;
  };

  // 5-row window (rows r-2 .. r+2) of y, h1 = y[c-1] + y[c+1] and v, two columns per lane
  dv2 yw[5], hw[5], vw[5];
#pragma unroll
  for (int m = 0; m < 5; ++m) yw[m] = hw[m] = vw[m] = dv2{0.0, 0.0};
  dv2 gq{0.0, 0.0};  // x0 of the last pushed row (both halves)
  auto push = [&](const Slot& s, ix_t t) {
    const ix_t q = prow(t);  // (its physical row; stored only when it is one of the band's)
    double p0 = 0.0, p1 = 0.0;
#pragma unroll
    for (int k = 0; k < NI; ++k) {  // explicit FMAs: the mailbox's recompute() repeats them
      p0 = __builtin_fma(ecf[k], s.e[k].x, p0);
      p1 = __builtin_fma(ecf[k], s.e[k].y, p1);
    }
    const dv2 v{pair_sum(p0), pair_sum(p1)};
    // the stencil input u = v (or the augmentation vector z); on a slab's halo row the x0
    // entry carries the neighbour's u
    const dv2 xe = both(s, EX);
    gq = xe;  // x0 of the row, for its centre step
    dv2 u;
    if constexpr (EXT) {
      const dv2 z = both(s, EZ);
      u = s.own ? z : xe;
    } else {
      u = s.own ? v : xe;
    }
    // block halo: this wave's share of c_i V_i on the four halo columns (sum over the 16 lanes
    // of each column), exchanged with u on the edge columns of every wave through LDS
    const int slot = int(t & 1);
    // mailbox: publish u on this block's first / last column pair
    {
      if constexpr (mb) {
        const bool pq = prod && s.own;
        const uint32_t po = mb_off(L, mbT, t + 2, pside, 0);
        ARN_CHK(!pq || (t + 2 >= 0 && t + 2 < mbT && int64_t(po) + 32 <= A.mb_cap * 8));
        __builtin_amdgcn_raw_buffer_store_b128(mb_rec(u.x, tag), rmb, pq ? po : kOOB, 0, kMBCoh);
        __builtin_amdgcn_raw_buffer_store_b128(mb_rec(u.y, tag), rmb, pq ? po + 16 : kOOB, 0,
                                               kMBCoh);
      }
    }
    if constexpr (!EXT && !mb) {
      // lane 4e + hh holds entry e (16 per instruction) of halo column hh: sum the four entries
      // of each 16-lane row (DPP row shifts), then the rows in pairs (permlane16/32 swaps);
      // lanes 12..15 end with the totals
      double hs = hcf * s.hv;
      hs += dpp_row_shr(hs, 4);
      hs += dpp_row_shr(hs, 8);
      hs = pair16_sum(hs);
      hs = pair_sum(hs);
      if ((lane & ~3) == 12) hpart[slot][wid][lane & 3] = hs;
    }
    if (lane == 0) {
      edge[slot][wid][0] = u.x;
      edge[slot][wid][1] = u.y;
    }
    if (lane == 31) {
      edge[slot][wid][2] = u.x;
      edge[slot][wid][3] = u.y;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    double hz = -0.0;  // mailbox: the halo pair is added by fixup() one iteration later
    if constexpr (EXT) {
      hz = __shfl(s.hx, hh + 4, 64);
    } else if constexpr (!mb) {
      hz = 0.0;
#pragma unroll
      for (int w = 0; w < WB; ++w) hz += hpart[slot][w][hh];  // fixed order: deterministic
    }
    // lanes 0..3: block halo columns -2, -1, +0, +1
    const double yh = s.own ? hz : s.hx;  // u on the halo columns
    const int wl = (wid > 0) ? wid - 1 : 0, wr = (wid < WB - 1) ? wid + 1 : WB - 1;
    // both candidates are read unconditionally (a uniform select, no branch around LDS reads)
    const double el2 = edge[slot][wl][2], el1 = edge[slot][wl][3];
    const double er1 = edge[slot][wr][0], er2 = edge[slot][wr][1];
    const double hl2 = readlane(yh, 0), hl1 = readlane(yh, 1);
    const double hr1 = readlane(yh, 2), hr2 = readlane(yh, 3);
    const double yl2 = (wid == 0) ? hl2 : el2, yl1 = (wid == 0) ? hl1 : el1;
    const double yr1 = (wid == WB - 1) ? hr1 : er1, yr2 = (wid == WB - 1) ? hr2 : er2;
    // neighbours inside the half: lane l-1 holds columns 2l-2, 2l-1 (the lanes whose neighbour
    // is across the half boundary take the edge values below)
    const double ux = dpp_up(u.x), uy = dpp_up(u.y);
    const double dx = dpp_down(u.x), dy = dpp_down(u.y);
    const double cm2 = (l == 0) ? yl2 : ux, cm1 = (l == 0) ? yl1 : uy;   // columns 2l-2, 2l-1
    const double cp2 = (l == 31) ? yr1 : dx, cp3 = (l == 31) ? yr2 : dy;  // columns 2l+2, 2l+3
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      yw[m] = yw[m + 1];
      hw[m] = hw[m + 1];
      vw[m] = vw[m + 1];
    }
    yw[4] = u;
    hw[4] = dv2{cm1 + u.y, u.x + cp2};
    vw[4] = v;
    // the h2 = u[c-2] + u[c+2] of row q is needed only when q is the window centre: keep the
    // four outer neighbours of the row two steps back
    const bool st = own && hf == 0 && t >= 0 && t < nrows;
    const __amdgpu_buffer_rsrc_t r = rv;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r,
                                           CO(st ? uint32_t(q * nx + col) * 8u : kOOB, nelem), 0,
                                           kOutPol);
    if (A.hs_ld > 0) push_edge_row(A.PS, A.hs_ld, q, ny, col, st, v);
    if (A.Eout_v)  // wave-uniform
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rEv,
                                             st ? eoff(q) : kOOB, 0, kOutPol);  // (eoff checks)
    return dv2{cm2 + cp2, cm1 + cp3};  // h2 of row q
  };

  double aw[NB], ag[NB];
#pragma unroll
  for (int k = 0; k < NB; ++k) aw[k] = ag[k] = 0.0;
  double awn = 0.0, avv = 0.0, aww = 0.0;
  dv2 h2w[3];  // h2 of rows r, r+1, r+2
#pragma unroll
  for (int m = 0; m < 3; ++m) h2w[m] = dv2{0.0, 0.0};
  // stencil + dot products of row r (window centre = row r; basis row r and x0 from LDS).
  // w' = (G(x0 + a u) - G(x0)) / sc in closed form: G is a cubic in its argument plus the linear
  // stencil, so the difference quotient is exactly
  //   (a/sc) [u/k - (L u + u (g (2 x0 + t) - (3 x0 (x0 + t) + t^2)))/2],  t = a u,
  // without the cancellation of two G evaluations (and without reading G0).
  const double zs = a_alpha * isc;
  auto centre = [&](ix_t t) {
    const ix_t r = prow(t);
    const dv2 (*d)[64] = lg[t & 1];
    const dv2 x0r = d[NB][lane];
    dv2 wo;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const double uc = yw[2][q];
      const double a1 = hw[2][q] + (yw[1][q] + yw[3][q]);
      const double dg = hw[1][q] + hw[3][q];
      const double a2 = h2w[0][q] + (yw[0][q] + yw[4][q]);
      const double Lu = applyL13(K, uc, a1, dg, a2);
      const double x = x0r[q];
      const double t = a_alpha * uc;
      const double D = K.g * (2.0 * x + t) - (3.0 * x * (x + t) + t * t);
      wo[q] = zs * (uc * K.ik - (Lu + uc * D) / 2);
    }
    const bool in = own && t < nrows;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, wo), rw,
                                           CO((in && hf == 0) ? uint32_t(r * nx + col) * 8u : kOOB,
                                              nelem),
                                           0, kOutPol);
    if (A.hs_ld > 0) push_edge_row(A.PS + 2, A.hs_ld, r, ny, col, in && hf == 0, wo);
    if (A.Eout_w)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, wo), rEw,
                                             (in && hf == 0) ? eoff(r) : kOOB, 0, kOutPol);
    const dv2 wm = in ? wo : dv2{0.0, 0.0};
    const dv2 vm = in ? vw[2] : dv2{0.0, 0.0};
#pragma unroll
    for (int k = 0; k < NB; ++k) {  // two chained FMAs per column pair
      const dv2 bi = d[k][lane];
      aw[k] = __builtin_fma(wm.y, bi.y, __builtin_fma(wm.x, bi.x, aw[k]));
      ag[k] = __builtin_fma(vm.y, bi.y, __builtin_fma(vm.x, bi.x, ag[k]));
    }
    // the three squares once per column (half 1 adds zeros)
    const dv2 wh = hf ? dv2{0.0, 0.0} : wm, vh = hf ? dv2{0.0, 0.0} : vm;
    awn = __builtin_fma(wh.y, vm.y, __builtin_fma(wh.x, vm.x, awn));
    avv = __builtin_fma(vh.y, vm.y, __builtin_fma(vh.x, vm.x, avv));
    aww = __builtin_fma(wh.y, wm.y, __builtin_fma(wh.x, wm.x, aww));
  };
  auto push_h2 = [&](const Slot& s, ix_t t) {
    const dv2 h2 = push(s, t);
    h2w[0] = h2w[1];
    h2w[1] = h2w[2];
    h2w[2] = h2;
  };
  // mailbox: the halo pair h of a row enters the window rows that hold it (hq: its h1 = u[c-1]
  // + u[c+1], h2q: its h2 = u[c-2] + u[c+2]); push() left -0.0 in its place, and a + b == b + a
  auto fixup = [&](dv2& hq, dv2& h2q, const dv2& h) {
    hq.x = hq.x + (needL ? h.y : -0.0);
    hq.y = hq.y + (needR ? h.x : -0.0);
    h2q.x = h2q.x + h.x;
    h2q.y = h2q.y + h.y;
  };

  // bands whose stencil reaches the slab's halo rows (rows -2, -1 / ny, ny+1): the first and
  // the last, and the one before a last band of a single row.  Each computes (or waits for) the
  // halo rows it reads itself -- the same bits from every band -- and fences the edge rows it
  // pushes (a band ending at ny - 1 pushes row ny - 2)
  const bool top = r0 < 2, bot = r1 + 2 > ny;
  if (A.x.me) slab_x_exchange<NV>(A, band, B0, BW, 0, a_tau, top, bot);  // uniform per block
  const bool edge_band = A.hs_ld > 0 && (top || bot);
  if (edge_band) slab_push_prologue<NV>(A, top, bot, B0, BW, 0, cst, a_tau);  // uniform per block
  if (nrows > 0) {
    // prologue (logical rows, march order): rows -2, -1 (band halo) and 0, 1 enter the window
    // (0, 1 also the LDS lag); rows 2 .. 1+PF go in flight.  Row t >= 2 uses register slot
    // (t - 2) mod RR.  At most 2 + PF rows of loads are live at once.
    {
      Slot S[RR];
      {
        Slot P[2];
        load(P[0], -2, TMc{});
        load(P[1], -1, TMc{});
        push_h2(P[0], -2);
        push_h2(P[1], -1);
        load(P[0], 0, TMc{});
        load(P[1], 1, TMc{});
#pragma unroll
        for (int d = 0; d < PF; ++d) load(S[d], 2 + d, TMc{});
        push_h2(P[0], 0);
        stash(P[0], gq, 0);
        push_h2(P[1], 1);
        stash(P[1], gq, 1);
      }
      {  // halo pairs of rows -1 (window slot 2) and 0 (slot 3)
        if constexpr (mb) {
          u32x4 a0, b0, a1, b1;
          poll(-1, &a0, &b0);
          poll(0, &a1, &b1);
          fixup(hw[2], h2w[0], mb_halo(-1, a0, b0));
          fixup(hw[3], h2w[1], mb_halo(0, a1, b1));
        }
      }
      // whole groups of RR rows with no branch inside the group (a branch would make the
      // compiler's wait-count analysis drain every load in flight): rows past the band end
      // are computed on clamped rows and masked out of the stores and sums
      for (ix_t t0 = 0; t0 < nrows; t0 += RR) {
#pragma unroll
        for (int k = 0; k < RR; ++k) {
          const ix_t t = t0 + k;
          u32x4 ma, mb2;
          if constexpr (mb) poll(t + 1, &ma, &mb2);  // before the row's batch: its wait
                                                     // leaves the batch in flight
          load(S[(k + PF) % RR], t + 2 + PF, NTc{});  // the slot of row t+1, consumed last step
          push_h2(S[k], t + 2);
          if constexpr (mb) fixup(hw[3], h2w[1], mb_halo(t + 1, ma, mb2));  // row t+1
          centre(t);
          stash(S[k], gq, t + 2);  // into the LDS slot row t just vacated
        }
      }
    }
  }

  if (edge_band) drain_stores();  // the pushed edge rows (push_edge_row), before the kernel ends
  // one partial per wave: [w'.V_i (nv)] [w'.v] [v.V_i (nv)] [v.v] [w'.w']; entry 2k + hf of
  // load k is summed over its half (width-32 butterflies)
#pragma unroll
  for (int o = 16; o >= 1; o >>= 1) {
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      aw[k] += __shfl_xor(aw[k], o, 64);
      ag[k] += __shfl_xor(ag[k], o, 64);
    }
  }
  double t3[3] = {awn, avv, aww};
  wave_sum<3>(t3);
  if (l == 0) {
    const int64_t nw = A.pstride;  // every wave of every block writes a column
    double* p = A.partial + A.pcol0 + gw;
    ARN_CHK(A.pcol0 + gw < nw && (2 * int64_t(NV) + 2) * nw + A.pcol0 + gw < A.partial_cap);
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int e = 2 * k + hf;
      if (e < NV) {
        st_sc1(p + int64_t(e) * nw, aw[k]);
        st_sc1(p + int64_t(NV + 1 + e) * nw, ag[k]);
      }
    }
    if (hf == 0) {
      st_sc1(p + int64_t(NV) * nw, t3[0]);
      st_sc1(p + int64_t(2 * NV + 1) * nw, t3[1]);
      st_sc1(p + int64_t(2 * NV + 2) * nw, t3[2]);
    }
  }
  if (A.tail.S) {  // uniform: the reduction + control of this step in the last blocks
    constexpr bool fits = sizeof(lag) >= sizeof(double) * (kArnMaxNV + 1) * (kArnMaxNV + 1);
    __shared__ double Gx[fits ? 1 : kArnMaxNV + 1][kArnMaxNV + 1];
    arn_tail<64 * WB>(A, ngroups * A.nbands,
                      fits ? reinterpret_cast<double (*)[kArnMaxNV + 1]>(&lag[0][0][0][0]) : Gx);
  }
}

// ------------------------------------------------------------------------------------------
// Wide layout (basis lengths up to kWideMaxNV): a wave owns 128 aligned columns, every lane holds
// columns 2l, 2l+1 of ALL entries, so each load instruction streams one 1-KB row segment of one
// vector (the vector-pair layout streams two 512-B segments: 0.69 against 0.73 of 8 TB/s for the
// bare pattern, scripts/micro/pattern2_bench.hip) and a block of W waves owns 128 W columns (W = 4:
// half the block-halo lines per column of the pair layout, whose halo costs ~9 % of a launch,
// profiles/r02_arnoldi_ab.md).  The LDS lag holds every basis entry of two rows for the W*128
// columns, 16 (nv+1) W KB: 152 KB at nv = 18, W = 4 -- which is what bounds this layout to short
// bases.  The update sum runs over the entries in order (arnoldi_edge_kernel matches it).
constexpr int kWW = 128;       // columns per wave
constexpr int kWideMaxNV = 18;  // LDS: 2 rows x (nv + 1) x 4 waves x 1 KB <= 152 KB

template <int NV, bool EXT, int PF, bool ALT, int W, bool MB>
__global__ void __launch_bounds__(64 * W) arnoldi_wide_kernel(const ArnoldiArgs A) {
  const double a_tau = arn_tau(A), a_alpha = arn_alpha(A), a_sc = arn_sc(A);
  double cst[NV];  // update coefficients, loaded together (independent loads, one wait)
#pragma unroll
  for (int e = 0; e < NV; ++e) cst[e] = arn_c(A, e);
  if (arn_halted(A)) return;
  constexpr int RR = PF + 1;
  constexpr int NE = NV + 2 + (EXT ? 1 : 0);  // [V_0 .. V_{NV-1}, w, x0, (z)]
  constexpr int EX = NV + 1, EZ = NV + 2;
  static_assert(NV + 1 <= 16 * W, "one packed halo load per row");
  __shared__ dv2 lag[W][2][NV + 1][64];  // basis rows r, r+1 and x0 (slot NV)
  __shared__ double edge[2][W][4];
  __shared__ double hpart[2][W][4];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const ix_t b = blockIdx.x;
  const ix_t bpx = gridDim.x / 8;  // XCD-aware: each XCD gets a contiguous run of blocks
  const ix_t L = (b % 8) * bpx + b / 8;
  const ix_t ngroups = (A.strips + W - 1) / W;
  if (L >= ngroups * A.nbands) return;
  const ix_t band = L / ngroups, grp = L % ngroups;
  const ix_t gw = L * W + wid;
  // 32-bit row / column arithmetic with the grid scalars pinned, as in arnoldi_kernel
  const ix_t nx = opaque_s<kPinScalars<NV>>(ix_t(A.nx));
  const ix_t ny = opaque_s<kPinScalars<NV>>(ix_t(A.ny));
  const ix_t B0 = grp * W * kWW;
  const ix_t c = B0 + wid * kWW + 2 * lane;
  const ix_t col = c % nx;
  const bool own = c < nx;
  const int hh = lane & 3;  // block halo: columns B0-2, B0-1, B0 + 128 W, +1
  const ix_t hc = (hh < 2) ? B0 - 2 + hh : B0 + W * kWW - 2 + hh;
  const ix_t hcol = ((hc % nx) + nx) % nx;
  const ix_t rend = (A.r_end >= 0) ? ix_t(A.r_end) : ny;
  const ix_t r0 = opaque_s<kPinScalars<NV>>(ix_t(A.r_begin) + band * A.RY);
  const ix_t r1 = opaque_s<kPinScalars<NV>>((r0 + A.RY < rend) ? r0 + A.RY : rend);
  const ix_t nrows = r1 - r0;
  const bool dn = !ALT || (band & 1) == 1;  // march direction, as in arnoldi_kernel
  const ix_t rb = opaque_s<kPinScalars<NV>>(dn ? r0 : r1 - 1);
  const ix_t rs = dn ? 1 : -1;
  using NTc = std::integral_constant<bool, true>;   // the row loop: non-temporal
  using TMc = std::integral_constant<bool, !ALT>;   // the prologue: temporal under ALT
  const SHCoef& K = A.k;
  const double isc = 1.0 / a_sc;
  const __amdgpu_buffer_rsrc_t rv = rsrc(A.out_v, ny * nx);
  const __amdgpu_buffer_rsrc_t rw = rsrc(A.out_w, ny * nx);
  dv2 (*lg)[NV + 1][64] = lag[wid];
  auto src = [&](int e) -> const double* {
    if (e < NV) return A.V[e];
    if (e == NV) return A.w;
    if (e == EX) return A.x0;
    return A.z;
  };
  auto cof = [&](int e) -> double { return e < NV ? cst[e] : a_tau; };  // e <= NV
  // packed block-halo loads: lane 4e' + hh of wave w fetches column hh of entry w + W e'
  const double *hp, *hE;
  double hcf;
  {
    const int e = wid + W * (lane >> 2);
    const double* p = A.w;
    const double* pe = A.E[NV];
    double cf = 0.0;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      p = (e == j) ? A.V[j] : p;
      pe = (e == j) ? A.E[j] : pe;
      cf = (e == j) ? cst[j] : cf;
    }
    cf = (e == NV) ? a_tau : cf;
    hp = p;
    hE = pe;
    hcf = cf;
  }
  const bool useE = A.E[0] != nullptr;
  const ix_t nbE = edge_groups(nx);
  const ix_t nelem = ny * nx, eelem = edge_elems(ny, nx);
  const ix_t bL = B0 / kEdgeW, bR = ((B0 + W * kWW) / kEdgeW) % nbE;
  const bool eL = own && (c % kEdgeW == 0);
  const bool eR = own && ((c + 2) % kEdgeW == 0 || c + 2 == nx);
  const ix_t ebo =
      eL ? (c / kEdgeW) * 4 + 2 : (eR ? ((c + 2 == nx) ? 0 : (c + 2) / kEdgeW) * 4 : 0);
  const bool eOn = eL || eR;
  const __amdgpu_buffer_rsrc_t rEv = rsrc(A.Eout_v, A.Eout_v ? nbE * ny * 4 : 0);
  const __amdgpu_buffer_rsrc_t rEw = rsrc(A.Eout_w, A.Eout_w ? nbE * ny * 4 : 0);
  auto eoff = [&](ix_t q) -> uint32_t {
    return eOn ? uint32_t(CI((ebo / 4) * ny * 4 + q * 4 + (ebo & 3), eelem - 1) * 8) : kOOB;
  };
  const double* hxp = (EXT && lane >= 4) ? A.z : A.x0;  // lanes 0-3: x0 halo, 4-7: z halo
  const bool slab = A.yh != nullptr;
  const double* yhb = slab ? A.yh : A.x0;
  const ix_t yld = (A.yh_ld > 0) ? A.yh_ld : nx;  // row stride of the halo rows
  auto prow = [&](ix_t t) -> ix_t {  // logical row t -> physical, as in arnoldi_kernel
    t = (t > nrows + 1) ? nrows + 1 : t;
    return rb + rs * t;
  };
  auto wrap = [&](ix_t t) -> ix_t {
    const ix_t q = prow(t);
    return (q < 0) ? q + ny : ((q >= ny) ? q - ny : q);
  };
  auto halo_row = [&](ix_t t) -> bool {
    const ix_t qc = prow(t);
    return slab && (qc < 0 || qc >= ny);
  };

  // mailbox, as in arnoldi_kernel: wave 0's lane 0 holds the first column pair and needs the
  // left halo pair, wave W-1's lane 63 the last pair and the right halo pair
  constexpr int BW = W * kWW;
  constexpr bool mb = MB && !EXT;
  const ix_t mbT = A.RY + 8;
  const __amdgpu_buffer_rsrc_t rmb = rsrc(A.mb, mb ? A.mb_cap : 0);
  const uint64_t tag = A.mb_tag;
  const bool needL = mb && wid == 0 && lane == 0, needR = mb && wid == W - 1 && lane == 63;
  const ix_t Lnb = band * ngroups + (needL ? (grp + ngroups - 1) % ngroups : (grp + 1) % ngroups);
  const int nside = needL ? 1 : 0;
  const bool prod = needL || needR;
  const int pside = needL ? 0 : 1;
  const ix_t fcol = needL ? (B0 - 2 + nx) % nx : (B0 + BW) % nx;
  bool mb_dead = A.mb_recompute;
  auto mb_need = [&](ix_t t) -> bool { return (needL || needR) && !halo_row(t); };
  auto poll = [&](ix_t t, u32x4* a, u32x4* b) {
    const bool on = mb_need(t) && !mb_dead;
    const uint32_t o = mb_off(Lnb, mbT, t + 2, nside, 0);
    ARN_CHK(!on || (t + 2 >= 0 && t + 2 < mbT && int64_t(o) + 32 <= A.mb_cap * 8));
    *a = __builtin_amdgcn_raw_buffer_load_b128(rmb, on ? o : kOOB, 0, kMBCoh);
    *b = __builtin_amdgcn_raw_buffer_load_b128(rmb, on ? o + 16 : kOOB, 0, kMBCoh);
  };
  auto recompute = [&](ix_t t) -> dv2 {  // push()'s update sum, entry order (rolled loop)
    const ix_t o2 = CI(wrap(t) * nx + fcol, nelem - 1);
    dv2 v{0.0, 0.0};
#pragma unroll 1
    for (int e = 0; e <= NV; ++e) {
      const dv2 x = gld2<false>((e < NV ? A.V[e] : A.w) + o2);
      const double cf = e < NV ? arn_c(A, e) : a_tau;
      v.x = __builtin_fma(cf, x.x, v.x);
      v.y = __builtin_fma(cf, x.y, v.y);
    }
    return v;
  };
  auto mb_halo = [&](ix_t t, u32x4 a, u32x4 b) -> dv2 {
    const bool need = mb_need(t);
    bool ok = !need || (!mb_dead && mb_tag_ok(a, tag) && mb_tag_ok(b, tag));
    dv2 h{mb_val(a), mb_val(b)};
    if (!ok) {
      const uint32_t o = mb_off(Lnb, mbT, t + 2, nside, 0);
      for (int n = 0; n < kMBSpin && !mb_dead && !ok; ++n) {
        __builtin_amdgcn_s_sleep(2);
        a = __builtin_amdgcn_raw_buffer_load_b128(rmb, o, 0, kMBCoh);
        b = __builtin_amdgcn_raw_buffer_load_b128(rmb, o + 16, 0, kMBCoh);
        ok = mb_tag_ok(a, tag) && mb_tag_ok(b, tag);
      }
      if (ok) {
        h = dv2{mb_val(a), mb_val(b)};
      } else {
        mb_dead = true;
        h = recompute(t);
      }
    }
    return need ? h : dv2{-0.0, -0.0};
  };

  struct Slot {
    dv2 e[NE];
    double hv, hx;
    bool own;
  };
  auto load = [&](Slot& s, ix_t t, auto pol) {  // pol as in arnoldi_kernel
    const ix_t qq = wrap(t);
    const ix_t o = CI(qq * nx + col, nelem - 1);
    const ix_t qc = prow(t);
    const bool hrow = halo_row(t);
    const ix_t hq = hrow ? ((qc < 0) ? qc + 2 : qc - ny + 2) : 0;
    const ix_t yo = CI(hq * yld + col, 4 * yld - 1);
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const double* a = src(e) + o;
      if (e == EX) a = hrow ? yhb + yo : a;
      s.e[e] = gld2<decltype(pol)::value>(a);
    }
    const ix_t ho = CI(qq * nx + hcol, nelem);
    if constexpr (!EXT && !mb) {
      const ix_t eo = CI(useE ? ((((hh < 2) ? bL : bR) * ny + qq) << 2) + hh : 0, eelem);
      s.hv = gld(useE ? hE + eo : hp + ho);
    }
    const ix_t hyo = CI(hq * yld + hcol, 4 * yld);
    s.hx = gld((hrow && lane < 4) ? yhb + hyo : (mb ? A.x0 : hxp + ho));
    s.own = !hrow;
  };
  auto stash = [&](const Slot& s, const dv2& g, ix_t t) {
    dv2 (*d)[64] = lg[t & 1];
#pragma unroll
    for (int e = 0; e < NV; ++e) d[e][lane] = s.e[e];
    d[NV][lane] = g;
  };

  dv2 yw[5], hw[5], vw[5];
#pragma unroll
  for (int m = 0; m < 5; ++m) yw[m] = hw[m] = vw[m] = dv2{0.0, 0.0};
  dv2 gq{0.0, 0.0};
  auto push = [&](const Slot& s, ix_t t) {
    const ix_t q = prow(t);
    dv2 v{0.0, 0.0};
#pragma unroll
    for (int e = 0; e <= NV; ++e) {  // entry order (the slab edge kernel sums the same way)
      v.x = __builtin_fma(cof(e), s.e[e].x, v.x);
      v.y = __builtin_fma(cof(e), s.e[e].y, v.y);
    }
    const dv2 xe = s.e[EX];
    gq = xe;
    dv2 u;
    if constexpr (EXT)
      u = s.own ? s.e[EZ] : xe;
    else
      u = s.own ? v : xe;
    const int slot = int(t & 1);
    {  // mailbox: publish u on this block's first / last column pair
      if constexpr (mb) {
        const bool pq = prod && s.own;
        const uint32_t po = mb_off(L, mbT, t + 2, pside, 0);
        ARN_CHK(!pq || (t + 2 >= 0 && t + 2 < mbT && int64_t(po) + 32 <= A.mb_cap * 8));
        __builtin_amdgcn_raw_buffer_store_b128(mb_rec(u.x, tag), rmb, pq ? po : kOOB, 0, kMBCoh);
        __builtin_amdgcn_raw_buffer_store_b128(mb_rec(u.y, tag), rmb, pq ? po + 16 : kOOB, 0,
                                               kMBCoh);
      }
    }
    if constexpr (!EXT && !mb) {
      double hs = hcf * s.hv;
      hs += dpp_row_shr(hs, 4);
      hs += dpp_row_shr(hs, 8);
      hs = pair16_sum(hs);
      hs = pair_sum(hs);
      if ((lane & ~3) == 12) hpart[slot][wid][lane & 3] = hs;
    }
    if (lane == 0) {
      edge[slot][wid][0] = u.x;
      edge[slot][wid][1] = u.y;
    }
    if (lane == 63) {
      edge[slot][wid][2] = u.x;
      edge[slot][wid][3] = u.y;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    double hz = -0.0;  // mailbox: added by fixup()
    if constexpr (EXT) {
      hz = __shfl(s.hx, hh + 4, 64);
    } else if constexpr (!mb) {
      hz = 0.0;
#pragma unroll
      for (int w = 0; w < W; ++w) hz += hpart[slot][w][hh];
    }
    const double yh = s.own ? hz : s.hx;
    const int wl = (wid > 0) ? wid - 1 : 0, wr = (wid < W - 1) ? wid + 1 : W - 1;
    const double el2 = edge[slot][wl][2], el1 = edge[slot][wl][3];
    const double er1 = edge[slot][wr][0], er2 = edge[slot][wr][1];
    const double hl2 = readlane(yh, 0), hl1 = readlane(yh, 1);
    const double hr1 = readlane(yh, 2), hr2 = readlane(yh, 3);
    const double yl2 = (wid == 0) ? hl2 : el2, yl1 = (wid == 0) ? hl1 : el1;
    const double yr1 = (wid == W - 1) ? hr1 : er1, yr2 = (wid == W - 1) ? hr2 : er2;
    // lane l-1 / l+1 hold columns 2l-2, 2l-1 / 2l+2, 2l+3 (whole-wave DPP shifts)
    const double ux = dpp_up(u.x), uy = dpp_up(u.y);
    const double dx = dpp_down(u.x), dy = dpp_down(u.y);
    const double cm2 = (lane == 0) ? yl2 : ux, cm1 = (lane == 0) ? yl1 : uy;
    const double cp2 = (lane == 63) ? yr1 : dx, cp3 = (lane == 63) ? yr2 : dy;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      yw[m] = yw[m + 1];
      hw[m] = hw[m + 1];
      vw[m] = vw[m + 1];
    }
    yw[4] = u;
    hw[4] = dv2{cm1 + u.y, u.x + cp2};
    vw[4] = v;
    const bool st = own && t >= 0 && t < nrows;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rv,
                                           CO(st ? uint32_t(q * nx + col) * 8u : kOOB, nelem), 0,
                                           kOutPol);
    if (A.hs_ld > 0) push_edge_row(A.PS, A.hs_ld, q, ny, col, st, v);
    if (A.Eout_v)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rEv,
                                             st ? eoff(q) : kOOB, 0, kOutPol);  // (eoff checks)
    return dv2{cm2 + cp2, cm1 + cp3};
  };

  double aw[NV + 3], ag[NV];  // aw: w'.V_i, then w'.v, v.v, w'.w'
#pragma unroll
  for (int i = 0; i < NV + 3; ++i) aw[i] = 0.0;
#pragma unroll
  for (int i = 0; i < NV; ++i) ag[i] = 0.0;
  dv2 h2w[3];
#pragma unroll
  for (int m = 0; m < 3; ++m) h2w[m] = dv2{0.0, 0.0};
  const double zs = a_alpha * isc;
  auto centre = [&](ix_t t) {  // closed-form FD quotient as in arnoldi_kernel
    const ix_t r = prow(t);
    const dv2 (*d)[64] = lg[t & 1];
    const dv2 x0r = d[NV][lane];
    dv2 wo;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const double uc = yw[2][q];
      const double a1 = hw[2][q] + (yw[1][q] + yw[3][q]);
      const double dg = hw[1][q] + hw[3][q];
      const double a2 = h2w[0][q] + (yw[0][q] + yw[4][q]);
      const double Lu = applyL13(K, uc, a1, dg, a2);
      const double x = x0r[q];
      const double t = a_alpha * uc;
      const double D = K.g * (2.0 * x + t) - (3.0 * x * (x + t) + t * t);
      wo[q] = zs * (uc * K.ik - (Lu + uc * D) / 2);
    }
    const bool in = own && t < nrows;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, wo), rw,
                                           CO(in ? uint32_t(r * nx + col) * 8u : kOOB, nelem), 0, kOutPol);
    if (A.hs_ld > 0) push_edge_row(A.PS + 2, A.hs_ld, r, ny, col, in, wo);
    if (A.Eout_w)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, wo), rEw,
                                             in ? eoff(r) : kOOB, 0, kOutPol);
    const dv2 wm = in ? wo : dv2{0.0, 0.0};
    const dv2 vm = in ? vw[2] : dv2{0.0, 0.0};
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const dv2 bi = d[i][lane];
      aw[i] = __builtin_fma(wm.y, bi.y, __builtin_fma(wm.x, bi.x, aw[i]));
      ag[i] = __builtin_fma(vm.y, bi.y, __builtin_fma(vm.x, bi.x, ag[i]));
    }
    aw[NV] = __builtin_fma(wm.y, vm.y, __builtin_fma(wm.x, vm.x, aw[NV]));
    aw[NV + 1] = __builtin_fma(vm.y, vm.y, __builtin_fma(vm.x, vm.x, aw[NV + 1]));
    aw[NV + 2] = __builtin_fma(wm.y, wm.y, __builtin_fma(wm.x, wm.x, aw[NV + 2]));
  };
  auto push_h2 = [&](const Slot& s, ix_t t) {
    const dv2 h2 = push(s, t);
    h2w[0] = h2w[1];
    h2w[1] = h2w[2];
    h2w[2] = h2;
  };
  auto fixup = [&](dv2& hq, dv2& h2q, const dv2& h) {  // as in arnoldi_kernel
    hq.x = hq.x + (needL ? h.y : -0.0);
    hq.y = hq.y + (needR ? h.x : -0.0);
    h2q.x = h2q.x + h.x;
    h2q.y = h2q.y + h.y;
  };

  const bool top = r0 < 2, bot = r1 + 2 > ny;  // as in arnoldi_kernel
  if (A.x.me) slab_x_exchange<NV>(A, band, B0, BW, NV + 1, a_tau, top, bot);  // uniform per block
  const bool edge_band = A.hs_ld > 0 && (top || bot);
  if (edge_band) slab_push_prologue<NV>(A, top, bot, B0, BW, NV + 1, cst, a_tau);
  if (nrows > 0) {  // logical rows, march order (see arnoldi_kernel)
    Slot S[RR];
    {
      Slot P[2];
      load(P[0], -2, TMc{});
      load(P[1], -1, TMc{});
      push_h2(P[0], -2);
      push_h2(P[1], -1);
      load(P[0], 0, TMc{});
      load(P[1], 1, TMc{});
#pragma unroll
      for (int d = 0; d < PF; ++d) load(S[d], 2 + d, TMc{});
      push_h2(P[0], 0);
      stash(P[0], gq, 0);
      push_h2(P[1], 1);
      stash(P[1], gq, 1);
    }
    {
      if constexpr (mb) {
        u32x4 a0, b0, a1, b1;
        poll(-1, &a0, &b0);
        poll(0, &a1, &b1);
        fixup(hw[2], h2w[0], mb_halo(-1, a0, b0));
        fixup(hw[3], h2w[1], mb_halo(0, a1, b1));
      }
    }
    for (ix_t t0 = 0; t0 < nrows; t0 += RR) {  // no branch inside a group (see arnoldi_kernel)
#pragma unroll
      for (int k = 0; k < RR; ++k) {
        const ix_t t = t0 + k;
        u32x4 ma, mb2;
        if constexpr (mb) poll(t + 1, &ma, &mb2);
        load(S[(k + PF) % RR], t + 2 + PF, NTc{});
        push_h2(S[k], t + 2);
        if constexpr (mb) fixup(hw[3], h2w[1], mb_halo(t + 1, ma, mb2));
        centre(t);
        stash(S[k], gq, t + 2);
      }
    }
  }

  if (edge_band) drain_stores();  // the pushed edge rows (push_edge_row), before the kernel ends
  wave_sum<NV + 3>(aw);
  wave_sum<NV>(ag);
  if (lane == 0) {
    const int64_t nw = A.pstride;
    double* p = A.partial + A.pcol0 + gw;
    ARN_CHK(A.pcol0 + gw < nw && (2 * int64_t(NV) + 2) * nw + A.pcol0 + gw < A.partial_cap);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      st_sc1(p + int64_t(i) * nw, aw[i]);
      st_sc1(p + int64_t(NV + 1 + i) * nw, ag[i]);
    }
    st_sc1(p + int64_t(NV) * nw, aw[NV]);
    st_sc1(p + int64_t(2 * NV + 1) * nw, aw[NV + 1]);
    st_sc1(p + int64_t(2 * NV + 2) * nw, aw[NV + 2]);
  }
  if (A.tail.S) {  // uniform: the reduction + control of this step in the last blocks
    constexpr bool fits = sizeof(lag) >= sizeof(double) * (kArnMaxNV + 1) * (kArnMaxNV + 1);
    __shared__ double Gx[fits ? 1 : kArnMaxNV + 1][kArnMaxNV + 1];
    arn_tail<64 * W>(A, ngroups * A.nbands,
                     fits ? reinterpret_cast<double (*)[kArnMaxNV + 1]>(&lag[0][0][0][0]) : Gx);
  }
}

int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::atoi(v) : dflt;
}

std::atomic<int64_t> g_mbox_launches{0};

// the alternating march (the ALT instantiations) for bands of at most kAltMaxRY rows;
// NKHIP_ARN_ALT=1 / 0 forces it on / off (read per launch, for A/B runs and tests)
constexpr int64_t kAltMaxRY = 32;
bool arnoldi_alt_mode(int64_t ry) {
  const char* e = std::getenv("NKHIP_ARN_ALT");
  if (e && (e[0] == '0' || e[0] == '1')) return e[0] == '1';
  return ry <= kAltMaxRY;
}

struct Occ {
  int ncu = 0, blocks_per_cu = 0;
};

// Grid of one resident round of waves (NKHIP_ARN_ROUNDS scales it) for a kernel whose blocks own
// `nwb` waves of `cw` columns each; bands of >= 8 rows, and no more partial columns than the
// caller's buffer holds.  `occ` = that kernel's occupancy.
// The instantiations of one launch: the plain / mailbox kernels and their alternating-march
// twins (ALT), with their occupancies
template <class K>
struct Kerns {
  K kern, kern_mb, kern_a, kern_mb_a;
  Occ occ, occ_mb, occ_a, occ_mb_a;
};

template <int NV, class K>
hipError_t launch_grid(const Kerns<K>& KS, int nwb, int nwb_mb, bool has_mb, int cw,
                       ArnoldiArgs A, hipStream_t s, int64_t* nwaves) {
  const Occ &occ = KS.occ, &occ_mb = KS.occ_mb;
  K kern = KS.kern, kern_mb = KS.kern_mb;
  if (occ.ncu == 0 || occ_mb.ncu == 0 || KS.occ_a.ncu == 0 || KS.occ_mb_a.ncu == 0)
    return hipErrorUnknown;
  static const int rounds = env_int("NKHIP_ARN_ROUNDS", 1);
  // the shortest band (NKHIP_ARN_MIN_RY, default 8 rows): short slabs trade resident waves for
  // fewer band prologues
  static const int min_ry = env_int("NKHIP_ARN_MIN_RY", 8) > 0 ? env_int("NKHIP_ARN_MIN_RY", 8) : 8;
  const int64_t strips = (A.nx + cw - 1) / cw;
  const int64_t rb = A.r_begin, re = (A.r_end >= 0) ? A.r_end : A.ny;
  if (rb < 0 || re > A.ny || re <= rb) return hipErrorInvalidValue;
  const int64_t rows = re - rb;
  // bands of one resident round of `w`-wave blocks at occupancy `o`; with the mailbox a
  // multiple of 8 bands, so that each XCD's contiguous run of blocks (the blockIdx mapping in
  // the kernels) holds whole bands
  struct Plan {
    int64_t nbands, RY, wpr, nw;
  };
  auto plan = [&](const Occ& o, int w, bool mbox) {
    const int64_t ncu_use = (o.ncu - A.reserve_cus > 0) ? o.ncu - A.reserve_cus : 1;
    const int64_t target = ncu_use * o.blocks_per_cu * w * (rounds > 0 ? rounds : 1);
    Plan p;
    p.wpr = (strips + w - 1) / w * w;  // waves per band (whole blocks)
    p.nbands = target / p.wpr;
    const int64_t cap_bands = A.partial_cap / ((2 * int64_t(NV) + 3) * p.wpr);
    if (p.nbands > cap_bands) p.nbands = cap_bands;
    if (p.nbands > rows / min_ry) p.nbands = rows / min_ry;
    if (p.nbands < 1) p.nbands = 1;
    if (mbox && p.nbands >= 8) p.nbands -= p.nbands % 8;
    p.RY = (rows + p.nbands - 1) / p.nbands;
    p.nbands = (rows + p.RY - 1) / p.RY;
    p.nw = p.wpr * p.nbands;
    return p;
  };
  // the mailbox: whole periodic rows of >= 2 of its blocks, records for every block
  const int64_t ngr = (strips + nwb_mb - 1) / nwb_mb;
  bool mbox = has_mb && A.mb && !A.z && A.nx % (int64_t(nwb_mb) * cw) == 0 && ngr >= 2 &&
              rb == 0 && re == A.ny;
  Plan P = plan(occ_mb, nwb_mb, true);
  if (mbox && ngr * P.nbands * (P.RY + 8) * 8 > A.mb_cap) mbox = false;
  if (!mbox) P = plan(occ, nwb, false);
  const int w = mbox ? nwb_mb : nwb;
  if (A.plan_only) {
    *nwaves = P.nw;
    return hipSuccess;
  }
  if (A.pstride == 0) A.pstride = P.nw;
  if (A.pcol0 < 0 || A.pcol0 + P.nw > A.pstride ||
      A.pstride * (2 * int64_t(NV) + 3) > A.partial_cap)
    return hipErrorInvalidValue;
  // a tail reduces this launch's partials alone: one launch over the whole slab
  if (A.tail.S && (A.pcol0 != 0 || A.pstride != P.nw || A.tail.nval != 2 * NV + 3 ||
                   A.tail.nval > kRedMax || !A.tail.result || !A.tail.prm || !A.tail.status ||
                   !A.tail.H || A.ctl != A.tail.prm || (A.tail.peer && !A.tail.result_host)))
    return hipErrorInvalidValue;
  A.strips = int(strips);
  A.nbands = int(P.nbands);
  A.RY = int(P.RY);
  // the alternating march where bands are short (its temporal prologue costs on tall bands:
  // profiles/r06_short_slab.md), with the same occupancy as the plan's kernel
  const Occ& oa = mbox ? KS.occ_mb_a : KS.occ_a;
  const Occ& op = mbox ? occ_mb : occ;
  if (A.alt < 0) A.alt = arnoldi_alt_mode(P.RY) ? 1 : 0;
  if (A.alt && oa.blocks_per_cu != op.blocks_per_cu) A.alt = 0;
  if (A.alt) {
    kern = KS.kern_a;
    kern_mb = KS.kern_mb_a;
  }
  if (mbox) {
    kern = kern_mb;  // the mailbox instantiation
    g_mbox_launches.fetch_add(1, std::memory_order_relaxed);
  } else {
    A.mb = nullptr;
  }
  int64_t blocks = (P.nw + w - 1) / w;
  blocks = (blocks + 7) / 8 * 8;
  *nwaves = P.nw;
  hipLaunchKernelGGL(kern, dim3(unsigned(blocks)), dim3(64 * w), 0, s, A);
  return hipGetLastError();
}

// occupancy of one kernel instantiation, queried once by a thread-safe static initialiser (slab
// threads of the loopback communicator launch the same instantiation concurrently)
template <class K>
Occ query_occ(K kern, int threads) {
  Occ o;
  int dev = 0, ncu = 0, nb = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, threads, 0) != hipSuccess)
    return o;  // ncu == 0: reported by launch_grid
  o.blocks_per_cu = nb > 0 ? nb : 1;
  o.ncu = ncu > 0 ? ncu : 1;
  return o;
}

template <int NV, bool EXT, int PF>
hipError_t launch_t(const ArnoldiArgs& A, hipStream_t s, int64_t* nwaves) {
  constexpr int WM = EXT ? WPB : kMbWPB;
  if (NV + 1 > 16 * WPB) return hipErrorInvalidValue;  // one packed halo load per row
  using K = decltype(&arnoldi_kernel<NV, EXT, PF, false, false, WPB>);
  // EXT: no mailbox, the same kernel
  static const Kerns<K> KS = [] {
    Kerns<K> k{arnoldi_kernel<NV, EXT, PF, false, false, WPB>,
               arnoldi_kernel<NV, EXT, PF, false, !EXT, WM>,
               arnoldi_kernel<NV, EXT, PF, true, false, WPB>,
               arnoldi_kernel<NV, EXT, PF, true, !EXT, WM>, {}, {}, {}, {}};
    k.occ = query_occ(k.kern, 64 * WPB);
    k.occ_mb = query_occ(k.kern_mb, 64 * WM);
    k.occ_a = query_occ(k.kern_a, 64 * WPB);
    k.occ_mb_a = query_occ(k.kern_mb_a, 64 * WM);
    return k;
  }();
  return launch_grid<NV>(KS, WPB, WM, !EXT, kSW, A, s, nwaves);
}

constexpr int kWideW = 4;  // waves per block of the wide layout (512 columns)
template <int NV, bool EXT, int PF>
hipError_t launch_wide(const ArnoldiArgs& A, hipStream_t s, int64_t* nwaves) {
  // no mailbox instantiation: with 512-column blocks the packed halo is the cheaper one
  // (4096^2, one box: n4 0.63 vs 0.55, n12 0.64 vs 0.63, n18 0.62 vs 0.57 of 8 TB/s)
  // (the wide kernel keeps a mailbox instantiation parameter, MB; it measured no gain with 2- or
  // 4-wave blocks, profiles/r02_arnoldi_ab.md, and is not instantiated)
  using K = decltype(&arnoldi_wide_kernel<NV, EXT, PF, false, kWideW, false>);
  static const Kerns<K> KS = [] {
    Kerns<K> k{arnoldi_wide_kernel<NV, EXT, PF, false, kWideW, false>,
               arnoldi_wide_kernel<NV, EXT, PF, false, kWideW, false>,
               arnoldi_wide_kernel<NV, EXT, PF, true, kWideW, false>,
               arnoldi_wide_kernel<NV, EXT, PF, true, kWideW, false>, {}, {}, {}, {}};
    k.occ = k.occ_mb = query_occ(k.kern, 64 * kWideW);
    k.occ_a = k.occ_mb_a = query_occ(k.kern_a, 64 * kWideW);
    return k;
  }();
  return launch_grid<NV>(KS, kWideW, kWideW, false, kWW, A, s, nwaves);
}

template <int NV, bool EXT>
hipError_t launch_pf(const ArnoldiArgs& A, hipStream_t s, int64_t* nwaves) {
  constexpr int PF = pf_for(NV);
#ifdef NKHIP_ARN_TUNE  // tuning build (`make tune`): NKHIP_ARN_PF selects the rows in flight
  static const int pf = env_int("NKHIP_ARN_PF", 0);
  if constexpr (NV % 4 == 0) {
    switch (pf) {
      case 1: return launch_t<NV, EXT, 1>(A, s, nwaves);
      case 2: return launch_t<NV, EXT, 2>(A, s, nwaves);
      case 3: return launch_t<NV, EXT, 3>(A, s, nwaves);
      case 4: return launch_t<NV, EXT, 4>(A, s, nwaves);
      case 6: return launch_t<NV, EXT, 6>(A, s, nwaves);
      default: break;
    }
  }
#endif
  if constexpr (NV <= kWideMaxNV) {
    if (arnoldi_wide(NV)) {
      constexpr int PFW = NV <= 4 ? 3 : (NV <= 10 ? 2 : 1);
      return launch_wide<NV, EXT, PFW>(A, s, nwaves);
    }
  }
  return launch_t<NV, EXT, PF>(A, s, nwaves);
}

template <bool EXT, int NV = 1>
hipError_t launch_e(const ArnoldiArgs& A, hipStream_t s, int64_t* nwaves) {
  if constexpr (NV > kArnMaxNV) {
    return hipErrorInvalidValue;
  } else {
#ifdef ARN_NV_ONLY  // ISA inspection builds: instantiate one basis length only
    if constexpr (NV != ARN_NV_ONLY) {
      return launch_e<EXT, NV + 1>(A, s, nwaves);
    } else {
      return launch_pf<NV, EXT>(A, s, nwaves);
    }
#else
    if (A.nv == NV) return launch_pf<NV, EXT>(A, s, nwaves);
    return launch_e<EXT, NV + 1>(A, s, nwaves);
#endif
  }
}

// u (= v, or z) on the edge rows 0, 1, ny-2, ny-1 of a slab (grid: column blocks x 4 rows).
// The update sum runs in the fused kernel's order -- for the pair layout (h0 = 0) entries 0, 2,
// 4, .. of [V_0 .. V_{nv-1}, w] in one partial, 1, 3, 5, .. in the other, then their sum; for the
// wide layout (h0 = nv + 1) all entries in order -- so a halo row
// equals the row its owner computes.
// PEER (row slabs over the peer-memory communicator): the kernel also performs the halo exchange
// -- it writes its rows straight into the neighbours' staging rows (peer_dev.h), publishes,
// waits for its own and copies them into yh (lo = rows 0, 1, hi = rows 2, 3) -- one launch
// instead of this kernel plus the communicator's halo kernel.  A halted step (handed back by the
// device control, identically on every rank) exchanges nothing on any rank.
template <int NV, bool PEER>
__global__ void __launch_bounds__(256) arnoldi_edge_kernel(const ArnoldiArgs A, double* y4,
                                                           int h0, const PeerArgs pa) {
  const double a_tau = arn_tau(A);
  if (arn_halted(A)) return;
  const int t = blockIdx.y;
  const int64_t row = (t < 2) ? t : A.ny - 4 + t;
  if constexpr (!PEER) {
    const int64_t j = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (j >= A.nx) return;
    const int64_t o = CI(row * A.nx + j, A.ny * A.nx);
    // the stencil input u of the fused kernel (the kernel is latency-bound: 4 rows of a slab --
    // every entry load in flight at once; batches of 8 took 10 us per launch)
    y4[int64_t(t) * A.nx + j] = edge_u<NV>(A, o, h0, a_tau);
  } else {
    // rows 0, 1 are the previous rank's "hi" staging rows, rows ny-2, ny-1 the next rank's "lo";
    // a grid of at most kHaloMaxBlocks column blocks strides over wider rows (peer_dev.h: every
    // block waits in peer_halo_finish, so the grid must fit the GPU as a whole)
    const int par = int(pa.tag & 1);
    const int q = (t < 2) ? (pa.rank - 1 + pa.P) % pa.P : (pa.rank + 1) % pa.P;
    double* dst = stage(pa.base[q], pa.P, pa.max_nx, par, t < 2 ? 1 : 0, t & 1);
    const int64_t step = int64_t(gridDim.x) * 256;
    for (int64_t j = int64_t(blockIdx.x) * 256 + threadIdx.x; j < A.nx; j += step) {
      ARN_CHK(j < pa.max_nx);
      dst[j] = edge_u<NV>(A, CI(row * A.nx + j, A.ny * A.nx), h0, a_tau);
    }
    (void)peer_halo_finish(pa, A.nx, y4, y4 + 2 * A.nx);  // failure: the host finds it
  }
}

template <int NV = 1>
hipError_t edge_launch_nv(const ArnoldiArgs& A, double* y4, int h0, const PeerArgs* pa,
                          hipStream_t s) {
  if constexpr (NV > kArnMaxNV) {
    return hipErrorInvalidValue;
  } else {
    if (A.nv != NV) return edge_launch_nv<NV + 1>(A, y4, h0, pa, s);
    const dim3 grid(unsigned((A.nx + 255) / 256), 4);
    if (pa)
      hipLaunchKernelGGL((arnoldi_edge_kernel<NV, true>), dim3(unsigned(halo_blocks(A.nx)), 4),
                         dim3(256), 0, s, A, y4, h0, *pa);
    else
      hipLaunchKernelGGL((arnoldi_edge_kernel<NV, false>), grid, dim3(256), 0, s, A, y4, h0,
                         PeerArgs{});
    return hipGetLastError();
  }
}

// E[(b ny + q) 4 + 0..3] = v[q][B-2], v[q][B-1], v[q][B], v[q][B+1], B = kEdgeW b, columns mod nx
__global__ void __launch_bounds__(256) edge_gather_kernel(const double* __restrict__ v,
                                                          double* __restrict__ E, int64_t ny,
                                                          int64_t nx, int64_t nb) {
  const int64_t t = int64_t(blockIdx.x) * 256 + threadIdx.x;  // t = b ny + q
  if (t >= nb * ny) return;
  const int64_t b = t / ny, q = t - b * ny;
  const int64_t B = b * kEdgeW;
  const double* row = v + q * nx;
  const int64_t cl = (B >= 2) ? B - 2 : B - 2 + nx;
  dv2 lo{row[cl], row[cl + 1]};  // B - 2 and B - 1 (even nx: a pair never straddles the wrap)
  dv2 hi{row[B], row[B + 1]};
  reinterpret_cast<dv2*>(E)[2 * t] = lo;
  reinterpret_cast<dv2*>(E)[2 * t + 1] = hi;
}

}  // namespace

hipError_t edge_gather_launch(const double* v, double* E, int64_t ny, int64_t nx, hipStream_t s) {
  if (!v || !E || ny < 1 || nx < 4 || nx % 2) return hipErrorInvalidValue;
  const int64_t nb = edge_groups(nx);
  hipLaunchKernelGGL(edge_gather_kernel, dim3(unsigned((nb * ny + 255) / 256)), dim3(256), 0, s,
                     v, E, ny, nx, nb);
  return hipGetLastError();
}

// where the layout of basis length nv splits its update sum in two (0: the pair layout's even /
// odd entries; nv + 1: the wide layout's whole sum in entry order)
int edge_split_point(int nv) {
  if (arnoldi_wide(nv)) return nv + 1;
  return 0;
}

hipError_t arnoldi_edge_launch(const ArnoldiArgs& A, double* y4, hipStream_t s) {
  if (A.ny < 4 || A.nx < 1 || !y4) return hipErrorInvalidValue;
  return edge_launch_nv(A, y4, edge_split_point(A.nv), nullptr, s);
}

hipError_t arnoldi_edge_halo_launch(const ArnoldiArgs& A, const PeerArgs& pa, double* yh,
                                    hipStream_t s) {
  if (A.ny < 4 || A.nx < 1 || !yh || A.nx > pa.max_nx || pa.P < 1 || pa.P > kMaxPeers)
    return hipErrorInvalidValue;
  return edge_launch_nv(A, yh, edge_split_point(A.nv), &pa, s);
}

int64_t arnoldi_mbox_launches() { return g_mbox_launches.load(std::memory_order_relaxed); }

int arnoldi_mbox_mode() {
  const char* e = std::getenv("NKHIP_ARN_MBOX");
  return (e && *e) ? std::atoi(e) : 1;
}

#ifdef ARN_TAIL_PROBE
extern "C" int nk_debug_tail_probe(unsigned long long* out) {
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tail_probe), sizeof(g_tail_probe)) != hipSuccess)
    return -1;
  static const unsigned long long zero[8] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_tail_probe), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
// g_tail_diag (a tail that gave up), read without synchronising the device (it may be the one
// whose stream failed)
extern "C" int nk_debug_tail_diag(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tail_diag), sizeof(g_tail_diag)) == hipSuccess ? 0
                                                                                             : -1;
}
#endif

bool arnoldi_wide(int nv) {
  static const bool on = env_int("NKHIP_ARN_WIDE", 1) != 0;
  return on && nv <= kWideMaxNV;
}

bool arnoldi_supported(int nv, int64_t ny, int64_t nx) {
  static const int maxnv = env_int("NKHIP_ARN_MAXNV", kArnMaxNV);
  return nv >= 1 && nv <= kArnMaxNV && nv <= maxnv && ny >= 8 && nx >= 4 && nx % 2 == 0 &&
         ny * nx * 8 < (int64_t(1) << 32);  // 32-bit byte offsets
}

hipError_t arnoldi_launch(const ArnoldiArgs& A, hipStream_t s, int64_t* nwaves) {
  if (!arnoldi_supported(A.nv, A.ny, A.nx)) return hipErrorInvalidValue;
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; };
  bool al = al16(A.w) && al16(A.x0) && al16(A.z) && al16(A.out_v) && al16(A.out_w);
  for (int i = 0; i < A.nv; ++i) al = al && al16(A.V[i]);
  if (!al) return hipErrorInvalidValue;  // 16-B loads and stores
  if (A.z) return launch_e<true>(A, s, nwaves);
  return launch_e<false>(A, s, nwaves);
}

int arnoldi_mailbox_counters(int64_t out[4], bool reset) {
#ifdef NKHIP_ARN_MBSTAT
  unsigned long long c[4];
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpyFromSymbol(c, HIP_SYMBOL(g_mb_stat), sizeof(c), 0, hipMemcpyDeviceToHost) != hipSuccess)
    return -2;
  for (int i = 0; i < 4; ++i) out[i] = int64_t(c[i]);
  if (reset) {
    for (int i = 0; i < 4; ++i) c[i] = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_mb_stat), c, sizeof(c), 0, hipMemcpyHostToDevice) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess)
      return -2;
  }
  return 0;
#else
  (void)out;
  (void)reset;
  return -1;  // not the mailbox-statistics build
#endif
}

int arnoldi_check_counters(int64_t* violations, int32_t* first_line, bool reset) {
#ifdef NKHIP_ARN_CHECK
  unsigned long long c[128];
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpyFromSymbol(c, HIP_SYMBOL(g_arn_chk), sizeof(c), 0, hipMemcpyDeviceToHost) != hipSuccess)
    return -2;
  int64_t n = 0;
  unsigned long long m = 0;
  for (int l = 0; l < 64; ++l) {
    n += int64_t(c[l]);
    m = (c[64 + l] > m) ? c[64 + l] : m;
  }
  if (violations) *violations = n;
  if (first_line) *first_line = n ? int32_t((1ull << 32) - m) : 0;
  if (reset) {
    for (int l = 0; l < 128; ++l) c[l] = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_arn_chk), c, sizeof(c), 0, hipMemcpyHostToDevice) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess)
      return -2;
  }
  return 0;
#else
  (void)violations;
  (void)first_line;
  (void)reset;
  return -1;  // not the bounds-checked build
#endif
}

}  // namespace nk

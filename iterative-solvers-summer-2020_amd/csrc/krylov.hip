// Krylov BLAS-1 kernels for the Arnoldi process (gfx950, wave64).
//
// Replaces the per-vector BLAS dot/axpy/nrm2/scal loop of SciPy's MGS Arnoldi
// (scipy/sparse/linalg/_isolve/_gcrotmk.py:104-143) with two fused passes per Arnoldi step:
//   mdot  -- all inner products V^T w (and the new Gram row V^T v_j, and w.w) in ONE read of
//            w and the basis, partial sums per block;
//   combo -- w <- w - sum_i c_i v_i together with |w|^2 and max|w| in ONE read-modify-write.
// A block owns a contiguous 2048-element chunk (256 threads x 4 double2), keeps its chunk of w
// in registers and streams the basis vectors through it; reductions are wave64 xor-shuffles, one
// LDS round, then a deterministic second-stage kernel (fixed summation order, so a run is
// bit-reproducible).
#include <cmath>
#include <cstdlib>

#include "nk_device.h"
#include "nk_kernels.h"

namespace nk {
namespace {

constexpr int BS = kKrylovBlock;
constexpr int PAIRS = kKrylovPerThread / 2;  // double2 per thread and vector

template <bool VEC>
__device__ __forceinline__ double2 ld2(const double* p, int64_t i, int64_t n) {
  if (VEC && i + 1 < n) return *reinterpret_cast<const double2*>(p + i);
  double2 r;
  r.x = (i < n) ? p[i] : 0.0;
  r.y = (i + 1 < n) ? p[i + 1] : 0.0;
  return r;
}

// A basis vector streamed once per pass: a non-temporal load, so the once-read basis does not
// evict w / the fresh basis vector from L2 and the Infinity Cache (mdot 5.65 -> 6.05 TB/s, combo
// 5.62 -> 6.47 TB/s at 4096^2; NKHIP_NT=0 restores plain loads).
typedef double dv2 __attribute__((ext_vector_type(2)));
template <bool VEC, bool NT>
__device__ __forceinline__ double2 ld2s(const double* p, int64_t i, int64_t n) {
  if (NT && VEC && i + 1 < n) {
    const dv2 v = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(p + i));
    return make_double2(v.x, v.y);
  }
  return ld2<VEC>(p, i, n);
}

template <bool VEC>
__device__ __forceinline__ void st2(double* p, int64_t i, int64_t n, double2 v) {
  if (VEC && i + 1 < n) {
    *reinterpret_cast<double2*>(p + i) = v;
    return;
  }
  if (i < n) p[i] = v.x;
  if (i + 1 < n) p[i + 1] = v.y;
}

template <bool VEC, bool NT>
__global__ void __launch_bounds__(BS) mdot_kernel(const double* a, const double* g, VecList P,
                                                  int np, int64_t n, int cpb, double* partial,
                                                  bool rev) {
  // One block walks `cpb` consecutive 2048-element chunks; per chunk the block keeps its slice of
  // a (and g) in registers and streams the vectors through it.  Per-vector block sums are
  // accumulated in LDS, so only one partial per block and value reaches HBM.
  __shared__ double accw[BS / 64][2 * kMaxVec + 1];
  const int64_t nblk = gridDim.x;
  const int64_t bid = blockIdx.x;
  const int nv = 2 * np + 1;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  // small vectors (few chunks): blockIdx.y splits the basis into runs of vpy vectors, so the
  // runs stream in parallel instead of one after another (each value's partial is summed in the
  // same order either way)
  const int vpy = (np + gridDim.y - 1) / gridDim.y;
  const int vlo = min(np, int(blockIdx.y) * ((vpy + 3) / 4 * 4));
  const int vhi = min(np, vlo + (vpy + 3) / 4 * 4);
  for (int t = lane; t < nv; t += 64) accw[wid][t] = 0.0;  // each wave zeroes its own slice
  double aa = 0.0;
  // rev: the blocks dispatched first take the last chunk groups; a group's chunks, their order and
  // its partial slot do not depend on rev, so the sums are bitwise the same in both directions
  const int64_t grp = rev ? nblk - 1 - bid : bid;
  for (int c = 0; c < cpb; ++c) {
    const int64_t chunk = grp * cpb + c;
    if (chunk * kKrylovChunk >= n) break;  // uniform
    const int64_t base = chunk * kKrylovChunk + 2 * int64_t(threadIdx.x);
    double2 av[PAIRS], gv[PAIRS];
#pragma unroll
    for (int k = 0; k < PAIRS; ++k) {
      av[k] = ld2<VEC>(a, base + k * 2 * BS, n);
      gv[k] = g ? ld2<VEC>(g, base + k * 2 * BS, n) : make_double2(0.0, 0.0);
      aa += av[k].x * av[k].x + av[k].y * av[k].y;
    }
    for (int i0 = vlo; i0 < vhi; i0 += 4) {
      double s[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) s[u] = 0.0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (i0 + u < vhi) {
          const double* p = P.p[i0 + u];
          double2 pv[PAIRS];
          if (p == g) {  // the Gram-row vector is already in registers: no second read
#pragma unroll
            for (int k = 0; k < PAIRS; ++k) pv[k] = gv[k];
          } else {
#pragma unroll
            for (int k = 0; k < PAIRS; ++k) pv[k] = ld2s<VEC, NT>(p, base + k * 2 * BS, n);
          }
#pragma unroll
          for (int k = 0; k < PAIRS; ++k) {
            s[u] += av[k].x * pv[k].x + av[k].y * pv[k].y;
            s[4 + u] += gv[k].x * pv[k].x + gv[k].y * pv[k].y;
          }
        }
      }
      // wave-level sums only (no block barrier inside the streaming loop); each wave keeps its
      // own LDS accumulators, combined once at the end
      wave_sum<8>(s);
      if (lane == 0) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (i0 + u < vhi) {
            accw[wid][i0 + u] += s[u];
            accw[wid][np + i0 + u] += s[4 + u];
          }
        }
      }
    }
  }
  double t[1] = {aa};
  wave_sum<1>(t);
  if (lane == 0) accw[wid][2 * np] += t[0];
  __syncthreads();
  for (int k = threadIdx.x; k < nv; k += BS) {
    const int kv = (k < np) ? k : ((k < 2 * np) ? k - np : -1);  // vector of value k (-1: |a|^2)
    if (kv >= 0 ? (kv < vlo || kv >= vhi) : blockIdx.y != 0) continue;  // another run's value
    double v = accw[0][k];
#pragma unroll
    for (int w = 1; w < BS / 64; ++w) v += accw[w][k];
    partial[int64_t(k) * nblk + grp] = v;
  }
}

// UNR: basis vectors whose loads are in flight together (2 at 4096^2, where the stream is
// bandwidth-bound; 8 for small vectors, where each batch is one memory latency)
template <bool VEC, bool NT, int UNR>
__global__ void __launch_bounds__(BS) combo_kernel(double* out, const double* in, double cin,
                                                   VecList P, int np, int64_t n, int cpb,
                                                   double* partial, bool rev, const double* prm,
                                                   EdgeOut eo) {
  // prm (device-side Arnoldi control): cin and the coefficients from the control's parameter
  // block; a step the control handed back does nothing
  if (prm) {
    if (prm[kArnMaxNV + 3] != 0.0) return;
    cin = prm[kArnMaxNV];
  }
  const int64_t nblk = gridDim.x;
  const int64_t bid = blockIdx.x;
  double red[2] = {0.0, 0.0};
  const int64_t grp = rev ? nblk - 1 - bid : bid;  // see mdot_kernel
  for (int cc = 0; cc < cpb; ++cc) {
    const int64_t chunk = grp * cpb + cc;
    if (chunk * kKrylovChunk >= n) break;  // uniform
    const int64_t base = chunk * kKrylovChunk + 2 * int64_t(threadIdx.x);
    double2 acc[PAIRS];
#pragma unroll
    for (int k = 0; k < PAIRS; ++k) {
      if (in) {
        const double2 x = ld2<VEC>(in, base + k * 2 * BS, n);
        acc[k] = make_double2(cin * x.x, cin * x.y);
      } else {
        acc[k] = make_double2(0.0, 0.0);
      }
    }
    int i = 0;
    for (; i + UNR <= np; i += UNR) {  // the sums stay in vector order
      double2 pv[UNR][PAIRS];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
#pragma unroll
        for (int k = 0; k < PAIRS; ++k) pv[u][k] = ld2s<VEC, NT>(P.p[i + u], base + k * 2 * BS, n);
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const double c = prm ? prm[i + u] : P.c[i + u];
#pragma unroll
        for (int k = 0; k < PAIRS; ++k) {
          acc[k].x += c * pv[u][k].x;
          acc[k].y += c * pv[u][k].y;
        }
      }
    }
    for (; i < np; ++i) {
      const double* p = P.p[i];
      const double c = prm ? prm[i] : P.c[i];
      double2 pv[PAIRS];
#pragma unroll
      for (int k = 0; k < PAIRS; ++k) pv[k] = ld2s<VEC, NT>(p, base + k * 2 * BS, n);
#pragma unroll
      for (int k = 0; k < PAIRS; ++k) {
        acc[k].x += c * pv[k].x;
        acc[k].y += c * pv[k].y;
      }
    }
    if (eo.E) {  // out's edge array (edge_gather_kernel's layout): the pairs at group borders
      const uint32_t nx = uint32_t(eo.nx), ny = uint32_t(eo.ny);
      uint32_t q = uint32_t(base) / nx, c = uint32_t(base) - q * nx;
#pragma unroll
      for (int k = 0; k < PAIRS; ++k) {
        if (base + k * 2 * BS < n) {
          const dv2 ev = {acc[k].x, acc[k].y};
          if (c % kEdgeW == 0)
            reinterpret_cast<dv2*>(eo.E)[2 * ((c / kEdgeW) * ny + q) + 1] = ev;
          if ((c + 2) % kEdgeW == 0 || c + 2 == nx)
            reinterpret_cast<dv2*>(eo.E)[2 * ((c + 2 == nx ? 0 : (c + 2) / kEdgeW) * ny + q)] = ev;
        }
        for (c += 2 * BS; c >= nx; c -= nx) ++q;
      }
    }
#pragma unroll
    for (int k = 0; k < PAIRS; ++k) {
      st2<VEC>(out, base + k * 2 * BS, n, acc[k]);
      const int64_t i = base + k * 2 * BS;
      if (i < n) {
        red[0] += acc[k].x * acc[k].x;
        red[1] = nmax(red[1], fabs(acc[k].x));
      }
      if (i + 1 < n) {
        red[0] += acc[k].y * acc[k].y;
        red[1] = nmax(red[1], fabs(acc[k].y));
      }
    }
  }
  if (partial) {
    const double v = block_reduce<2, 1, BS>(red);
    if (threadIdx.x < 2) partial[int64_t(threadIdx.x) * nblk + grp] = v;
  }
}

constexpr int RB = 1024;  // reduce_final block: <= 4 partials per thread at 4096 producer blocks

__global__ void __launch_bounds__(RB) reduce_final_kernel(const double* partial, int64_t nblk,
                                                          int nsum, double* result,
                                                          double* result_host) {
  const int k = blockIdx.x;
  const double s = reduce_column<RB>(partial + int64_t(k) * nblk, nblk, k < nsum);
  if (threadIdx.x == 0) {
    result[k] = s;
    if (result_host) result_host[k] = s;  // pinned, device-mapped host memory: no D2H blit
  }
}

template <bool VEC>
__global__ void __launch_bounds__(256) axpby_kernel(double a, const double* x, double b,
                                                    const double* y, double* out, int64_t n) {
  const int64_t i = 2 * (int64_t(blockIdx.x) * 256 + threadIdx.x);
  if (i >= n) return;
  const double2 xv = ld2<VEC>(x, i, n);
  double2 r = make_double2(a * xv.x, a * xv.y);
  if (y) {
    const double2 yv = ld2<VEC>(y, i, n);
    r.x += b * yv.x;
    r.y += b * yv.y;
  }
  st2<VEC>(out, i, n, r);
}

__global__ void __launch_bounds__(256) fddiff_kernel(double* w, const double* f0, double sc,
                                                     int64_t n) {
  const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i < n) w[i] = (w[i] - f0[i]) / sc;
}

// CG update (sh_linearised's solve): x += alpha p; r -= alpha q; per-block sum of the new r^2.
// Grid-stride over double2 pairs; one partial per block.
template <bool VEC>
__global__ void __launch_bounds__(256) cg_update_kernel(double* x, double* r, const double* p,
                                                        const double* q, double alpha, int64_t n,
                                                        double* partial) {
  double acc[1] = {0.0};
  const int64_t stride = 2 * int64_t(gridDim.x) * 256;
  for (int64_t i = 2 * (int64_t(blockIdx.x) * 256 + threadIdx.x); i < n; i += stride) {
    const double2 xv = ld2<VEC>(x, i, n), rv = ld2<VEC>(r, i, n);
    const double2 pv = ld2<VEC>(p, i, n), qv = ld2<VEC>(q, i, n);
    const double2 xn = make_double2(xv.x + alpha * pv.x, xv.y + alpha * pv.y);
    const double2 rn = make_double2(rv.x - alpha * qv.x, rv.y - alpha * qv.y);
    st2<VEC>(x, i, n, xn);
    st2<VEC>(r, i, n, rn);
    acc[0] += rn.x * rn.x;
    if (i + 1 < n) acc[0] += rn.y * rn.y;
  }
  const double v = block_reduce<1, 1, 256>(acc);
  if (threadIdx.x == 0) partial[blockIdx.x] = v;
}

// D of sh_linearised.py:50: d = (5U - Uo)(5U - Uo) k/16 - g k U
__global__ void __launch_bounds__(256) shlin_diag_kernel(const double* U, const double* Uo,
                                                         double k, double g, double* d,
                                                         int64_t n) {
  const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  const double a = 5 * U[i] - Uo[i];
  d[i] = a * a * k / 16 - g * k * U[i];
}

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// vectors of at most this many 2048-element chunks take the latency-bound variants (the
// moving-mesh problems' 5551 / 2601 points; the SH grids have thousands of chunks)
constexpr int64_t kSmallChunks = 32;

}  // namespace

static int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::atoi(v) : dflt;
}

int64_t krylov_grid(int64_t n, int* cpb, int64_t target) {
  // at most `target` blocks of 256 threads; each walks ceil(chunks / target) chunks.
  const int64_t chunks = krylov_blocks(n);
  const int64_t c = chunks <= target ? 1 : (chunks + target - 1) / target;
  *cpb = int(c);
  return (chunks + c - 1) / c;
}

bool traversal_reverse() {
  static const bool on = env_int("NKHIP_PINGPONG", 1) != 0;
  thread_local bool flip = false;
  if (!on) return false;
  flip = !flip;
  return !flip;
}

hipError_t mdot_launch(const double* a, const double* g, const VecList& P, int np, int64_t n,
                       double* partial, hipStream_t s, int64_t* nblk) {
  if (np < 0 || np > kMaxVec) return hipErrorInvalidValue;
  static const int target = env_int("NKHIP_MDOT_BLOCKS", 4096);
  int cpb = 0;
  const int64_t nb = krylov_grid(n, &cpb, target);
  if (nblk) *nblk = nb;
  if (nb == 0) return hipSuccess;
  bool vec = al16(a) && al16(g);
  for (int i = 0; i < np; ++i) vec = vec && al16(P.p[i]);
  const bool rev = traversal_reverse();
  static const bool nt = env_int("NKHIP_NT", 1) != 0;
  // small vectors (the moving-mesh problems: 5551 points = 3 chunks): one block row per run of
  // four basis vectors; the 4096^2 grid keeps one row
  const dim3 grid(unsigned(nb), nb <= kSmallChunks ? unsigned((np + 3) / 4 > 0 ? (np + 3) / 4 : 1) : 1u);
  if (vec && nt)
    hipLaunchKernelGGL((mdot_kernel<true, true>), grid, dim3(BS), 0, s, a, g, P, np, n, cpb,
                       partial, rev);
  else if (vec)
    hipLaunchKernelGGL((mdot_kernel<true, false>), grid, dim3(BS), 0, s, a, g, P, np, n, cpb,
                       partial, rev);
  else
    hipLaunchKernelGGL((mdot_kernel<false, false>), grid, dim3(BS), 0, s, a, g, P, np, n, cpb,
                       partial, rev);
  return hipGetLastError();
}

namespace {
hipError_t combo_any(double* out, const double* in, double cin, const VecList& P, int np,
                     int64_t n, double* partial, hipStream_t s, int64_t* nblk, const double* prm,
                     const EdgeOut& eo) {
  if (np < 0 || np > kMaxVec) return hipErrorInvalidValue;
  if (eo.E && (eo.nx < 4 || eo.nx % 2 || eo.ny < 1 || eo.nx * eo.ny != n || n >= (int64_t(1) << 31)))
    return hipErrorInvalidValue;
  static const int target = env_int("NKHIP_COMBO_BLOCKS", 1 << 30);
  int cpb = 0;
  const int64_t nb = krylov_grid(n, &cpb, target);
  if (nblk) *nblk = nb;
  if (nb == 0) return hipSuccess;
  bool vec = al16(out) && al16(in);
  for (int i = 0; i < np; ++i) vec = vec && al16(P.p[i]);
  const bool rev = traversal_reverse();
  static const bool nt = env_int("NKHIP_NT", 1) != 0;
  const dim3 grid{unsigned(nb)}, block{unsigned(BS)};
  if (nb <= kSmallChunks) {  // small vectors: 8 basis vectors' loads in flight per batch
    if (vec)
      hipLaunchKernelGGL((combo_kernel<true, false, 8>), grid, block, 0, s, out, in, cin, P, np, n,
                         cpb, partial, rev, prm, eo);
    else
      hipLaunchKernelGGL((combo_kernel<false, false, 8>), grid, block, 0, s, out, in, cin, P, np,
                         n, cpb, partial, rev, prm, eo);
  } else if (vec && nt) {
    hipLaunchKernelGGL((combo_kernel<true, true, 2>), grid, block, 0, s, out, in, cin, P, np, n,
                       cpb, partial, rev, prm, eo);
  } else if (vec) {
    hipLaunchKernelGGL((combo_kernel<true, false, 2>), grid, block, 0, s, out, in, cin, P, np, n,
                       cpb, partial, rev, prm, eo);
  } else {
    hipLaunchKernelGGL((combo_kernel<false, false, 2>), grid, block, 0, s, out, in, cin, P, np, n,
                       cpb, partial, rev, prm, eo);
  }
  return hipGetLastError();
}
}  // namespace

hipError_t combo_launch(double* out, const double* in, double cin, const VecList& P, int np,
                        int64_t n, double* partial, hipStream_t s, int64_t* nblk,
                        const EdgeOut& eo) {
  return combo_any(out, in, cin, P, np, n, partial, s, nblk, nullptr, eo);
}

hipError_t combo_prm_launch(double* out, const double* in, const double* prm, const VecList& P,
                            int np, int64_t n, hipStream_t s) {
  if (!prm || np > kArnMaxNV) return hipErrorInvalidValue;
  return combo_any(out, in, 0.0, P, np, n, nullptr, s, nullptr, prm, EdgeOut{});
}

hipError_t reduce_final_launch(const double* partial, int64_t nblk, int nsum, int nv,
                               double* result, double* result_host, hipStream_t s) {
  if (nv <= 0) return hipSuccess;
  hipLaunchKernelGGL(reduce_final_kernel, dim3(unsigned(nv)), dim3(RB), 0, s, partial, nblk, nsum,
                     result, result_host);
  return hipGetLastError();
}

namespace {
// Streaming copy in contiguous 16-KB chunks per block (256 lanes x 4 x 16 B, all four loads in
// flight before the first store; non-temporal both ways): the pattern that streams fastest on
// this chip (scripts/micro/pattern2_bench.hip), used as the bench's per-box bandwidth probe.
typedef double sdv2 __attribute__((ext_vector_type(2)));
__global__ void __launch_bounds__(256) stream_copy_kernel(const sdv2* __restrict__ src,
                                                          sdv2* __restrict__ dst, int64_t n2) {
  const int64_t base = int64_t(blockIdx.x) * 1024 + threadIdx.x;
  sdv2 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t i = base + k * 256;
    if (i < n2) v[k] = __builtin_nontemporal_load(src + i);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t i = base + k * 256;
    if (i < n2) __builtin_nontemporal_store(v[k], dst + i);
  }
}

}  // namespace

hipError_t stream_copy_launch(const double* src, double* dst, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (!al16(src) || !al16(dst) || n % 2) return hipErrorInvalidValue;
  const int64_t n2 = n / 2;
  hipLaunchKernelGGL(stream_copy_kernel, dim3(unsigned((n2 + 1023) / 1024)), dim3(256), 0, s,
                     reinterpret_cast<const sdv2*>(src), reinterpret_cast<sdv2*>(dst), n2);
  return hipGetLastError();
}

hipError_t axpby_launch(double a, const double* x, double b, const double* y, double* out,
                        int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t g = (n + 511) / 512;
  const bool vec = al16(x) && al16(y) && al16(out);
  if (vec)
    hipLaunchKernelGGL(axpby_kernel<true>, dim3(unsigned(g)), dim3(256), 0, s, a, x, b, y, out, n);
  else
    hipLaunchKernelGGL(axpby_kernel<false>, dim3(unsigned(g)), dim3(256), 0, s, a, x, b, y, out,
                       n);
  return hipGetLastError();
}

hipError_t cg_update_launch(double* x, double* r, const double* p, const double* q, double alpha,
                            int64_t n, double* partial, hipStream_t s, int64_t* nblk) {
  const int64_t pairs = (n + 1) / 2;
  int64_t g = (pairs + 255) / 256;
  if (g > 1024) g = 1024;
  if (g < 1) g = 1;
  *nblk = g;
  if (al16(x) && al16(r) && al16(p) && al16(q))
    hipLaunchKernelGGL(cg_update_kernel<true>, dim3(unsigned(g)), dim3(256), 0, s, x, r, p, q,
                       alpha, n, partial);
  else
    hipLaunchKernelGGL(cg_update_kernel<false>, dim3(unsigned(g)), dim3(256), 0, s, x, r, p, q,
                       alpha, n, partial);
  return hipGetLastError();
}

hipError_t shlin_diag_launch(const double* U, const double* Uo, double k, double g, double* d,
                             int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(shlin_diag_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, s, U, Uo, k,
                     g, d, n);
  return hipGetLastError();
}

hipError_t fddiff_launch(double* w, const double* f0, double sc, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(fddiff_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, s, w, f0, sc, n);
  return hipGetLastError();
}

}  // namespace nk

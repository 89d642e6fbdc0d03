// Fused Arnoldi step of the Swift-Hohenberg Newton-Krylov solve (gfx950, wave64).
//
// One launch does what SciPy's _fgmres loop body does between two matvecs
// (scipy/sparse/linalg/_isolve/_gcrotmk.py:104-143) plus the matvec of the next step
// (KrylovJacobian.matvec, scipy/optimize/_nonlin.py:1500-1513 on the residual of
// sh_scipy_nk.py:47-49):
//   v      = tau*w + sum_i c_i V_i            (the Gram-Schmidt update of step j; c_i = -h_i sig_i)
//   y      = x0 + alpha*z,  z = v (or an LGMRES augmentation vector when EXT)
//   w'     = (G(y) - G0) / sc                 (the FD Jacobian-vector product of step j+1)
//   sums   w'.V_i, w'.v, v.V_i, v.v, w'.w'    (the multi-dot of step j+1, Gram row included)
// so the basis V_0..V_j is read ONCE per Arnoldi step instead of twice (update + multi-dot), and
// neither v nor w' is re-read.  Unfused, a step moves (2j + 9) vectors; fused (j + 6).
//
// The stencil couples rows r-2..r+2, so a wave marches down a band of rows with the update running
// two rows AHEAD of the stencil: at row r it forms v[r+2] from V_i[r+2], evaluates w'[r] on the
// 5-row window of y, and takes the dot products of row r against V_i[r].  Loads run PF rows ahead
// in a register ring (rotated by unrolling the walk by its length, so no register is copied); the
// basis row and G0 of rows r, r+1 wait in an LDS ring for their dot products, which keeps the
// registers for loads in flight.  The basis length is a template parameter (fully unrolled).
//
// Lanes: one column per lane, 64 consecutive 512-B-aligned columns per wave (an aligned wave
// segment streams at 62-68 % of peak in scripts/micro/pattern_bench.hip, an overlapping 60-column
// one at 52-55 %).  The stencil's column halo (two columns each side) comes from PACKED halo loads:
// in one instruction lane L fetches halo column L%4 of vector L/4 (16 vectors per instruction), a
// 4-step xor-shuffle sums c_i V_i over the lanes of each column, and the four halo values of y are
// read out to scalars.  Column neighbours inside the wave come from lane shuffles; no block
// barrier.  Each band recomputes v on the two rows above and below it (band halo).  Per-lane sums
// are wave-reduced once at the end and written as one partial per wave (deterministic: a fixed
// wave -> rows mapping and a fixed order).
#include <cmath>
#include <cstdlib>

#include "nk_device.h"
#include "nk_kernels.h"

namespace nk {
namespace {

constexpr int kSW = 64;  // columns per wave (one per lane)
constexpr int WPB = 4;   // waves per block

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

// Stores through a raw buffer resource: a lane whose offset is out of range (kOOB) writes
// nothing, so masked stores need no branch.
constexpr uint32_t kOOB = 0xFFFFFFF0u;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(double* p, int64_t n) {
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, int(uint32_t(n * 8)), 0x00020000);
}
__device__ __forceinline__ void stb(__amdgpu_buffer_rsrc_t r, uint32_t off, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, off, 0, 0);
}

// Rows of loads in flight per wave for a basis of NV vectors: as many as the registers allow at
// the occupancy the register count gives (and the 63 loads the wait counter tracks).
constexpr int pf_for(int nv) {
  return nv <= 2 ? 4 : nv <= 6 ? 3 : nv <= 16 ? 2 : 1;
}

__device__ __forceinline__ double readlane(double v, int l) {
  const u32x2 b = __builtin_bit_cast(u32x2, v);
  u32x2 r;
  r.x = __builtin_amdgcn_readlane(b.x, l);
  r.y = __builtin_amdgcn_readlane(b.y, l);
  return __builtin_bit_cast(double, r);
}

template <int NV, bool EXT, int PF, bool NT>
__global__ void __launch_bounds__(64 * WPB) arnoldi_kernel(const ArnoldiArgs A) {
  constexpr int RR = PF + 1;  // register ring: the update row r+2 and PF rows in flight
  // lag rows r, r+1 of the basis (and G0) for the dot products, one region per wave
  __shared__ double lag[WPB][2][NV + 1][64];
  // per row (parity slot): y on lanes 0, 1, 62, 63 of every wave; the waves' partial sums of v on
  // the block's four halo columns
  __shared__ double edge[2][WPB][4];
  __shared__ double hpart[2][WPB][4];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // XCD-aware mapping: consecutive blocks go round-robin over the 8 XCDs; give each XCD one
  // contiguous run of blocks (whole bands), so band halos are shared inside one L2.
  const int64_t b = blockIdx.x;
  const int64_t bpx = gridDim.x / 8;  // grid is a multiple of 8
  const int64_t L = (b % 8) * bpx + b / 8;
  const int64_t ngroups = (A.strips + WPB - 1) / WPB;  // a block = WPB adjacent strips
  if (L >= ngroups * A.nbands) return;                 // whole blocks only
  const int64_t band = L / ngroups, grp = L % ngroups;
  const int64_t gw = L * WPB + wid;  // partial-sum column of this wave
  const int64_t nx = A.nx, ny = A.ny;
  const int64_t B0 = grp * WPB * kSW;  // the block's first column
  const int64_t c = B0 + wid * kSW + lane;  // columns past nx compute wrapped columns, masked
  const int64_t col = c % nx;
  const bool own = c < nx;
  // block halo: h = 0, 1 -> columns B0-2, B0-1; h = 2, 3 -> B0 + WPB*64, +1
  const int hh = lane & 3;
  const int64_t hc = (hh < 2) ? B0 - 2 + hh : B0 + WPB * kSW - 2 + hh;
  const int64_t hcol = ((hc % nx) + nx) % nx;
  const int64_t r0 = band * A.RY;
  const int64_t r1 = (r0 + A.RY < ny) ? r0 + A.RY : ny;
  const int64_t nrows = r1 - r0;
  const SHCoef& K = A.k;
  const double isc = 1.0 / A.sc;
  const __amdgpu_buffer_rsrc_t rv = rsrc(A.out_v, ny * nx);
  const __amdgpu_buffer_rsrc_t rw = rsrc(A.out_w, ny * nx);
  double (*lg)[NV + 1][64] = lag[wid];
  // packed block-halo loads, shared by the WPB waves: lane L of wave w fetches halo column L%4 of
  // entry e = w + WPB*(L/4) of [V_0 .. V_{NV-1}, w] with coefficient c_e (tau for w); lanes past
  // the list repeat entry w's address (same cache line, no extra traffic) with coefficient 0
  const double* hp;
  double hcf;
  {
    const int e = wid + WPB * (lane >> 2);
    const double* p = (wid < NV) ? A.V[wid < NV ? wid : 0] : A.w;
    double cf = 0.0;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      p = (e == j) ? A.V[j] : p;
      cf = (e == j) ? A.c[j] : cf;
    }
    p = (e == NV) ? A.w : p;
    cf = (e == NV) ? A.tau : cf;
    hp = p;
    hcf = cf;
  }
  const double* hxp = (EXT && lane >= 4) ? A.z : A.x0;  // lanes 0-3: x0 halo, 4-7: z halo

  auto wrap = [&](int64_t q) -> int64_t {
    q = (q > r1 + 1) ? r1 + 1 : q;  // past the band halo: re-read its last row
    return (q < 0) ? q + ny : ((q >= ny) ? q - ny : q);
  };

  struct Slot {
    double v[NV];
    double w, x, z, g;
    double hv, hx;
  };
  auto load = [&](Slot& s, int64_t q) {
    const int64_t qq = wrap(q);
    const uint32_t o = uint32_t((qq * nx + col) * 8);
#pragma unroll
    for (int i = 0; i < NV; ++i) s.v[i] = ldb<NT>(A.V[i], o);
    s.w = ldb<NT>(A.w, o);
    s.x = ldb<NT>(A.x0, o);
    if constexpr (EXT) s.z = ldb<NT>(A.z, o);
    s.g = ldb<NT>(A.g0, o);
    const int64_t ho = qq * nx + hcol;
    if constexpr (!EXT) s.hv = hp[ho];
    s.hx = hxp[ho];
  };
  // the basis row and G0 of row q wait in LDS slot (q - r0) & 1 until row q's dot products
  auto stash = [&](const Slot& s, int64_t q) {
    double (*d)[64] = lg[(q - r0) & 1];
#pragma unroll
    for (int i = 0; i < NV; ++i) d[i][lane] = s.v[i];
    d[NV][lane] = s.g;
  };

  // 5-row window (rows r-2 .. r+2): y, the horizontal pair sums h1 = y[c-1] + y[c+1] and
  // h2 = y[c-2] + y[c+2], and v
  double yw[5], hw[5], h2w[5], vw[5];
#pragma unroll
  for (int m = 0; m < 5; ++m) yw[m] = hw[m] = h2w[m] = vw[m] = 0.0;
  auto push = [&](const Slot& s, int64_t q) {
    double v = A.tau * s.w;
#pragma unroll
    for (int i = 0; i < NV; ++i) v += A.c[i] * s.v[i];
    const double y = s.x + A.alpha * (EXT ? s.z : v);
    // block halo: this wave's share of c_i V_i on the four halo columns (sum over the 16 lanes
    // of each column), exchanged with y on the edge lanes of every wave through LDS
    const int slot = int(q & 1);
    if constexpr (!EXT) {
      double hs = hcf * s.hv;
      hs += __shfl_xor(hs, 4, 64);
      hs += __shfl_xor(hs, 8, 64);
      hs += __shfl_xor(hs, 16, 64);
      hs += __shfl_xor(hs, 32, 64);
      if (lane < 4) hpart[slot][wid][lane] = hs;
    }
    const int el = (lane < 2) ? lane : lane - 60;  // lanes 0, 1, 62, 63 -> 0..3
    if (lane < 2 || lane >= 62) edge[slot][wid][el] = y;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    double hz = 0.0;
    if constexpr (EXT) {
      hz = __shfl(s.hx, hh + 4, 64);
    } else {
#pragma unroll
      for (int w = 0; w < WPB; ++w) hz += hpart[slot][w][hh];  // fixed order: deterministic
    }
    const double yh = s.hx + A.alpha * hz;  // lanes 0..3: block halo columns -2, -1, +0, +1
    const int wl = (wid > 0) ? wid - 1 : 0, wr = (wid < WPB - 1) ? wid + 1 : WPB - 1;
    const double yl2 = (wid == 0) ? readlane(yh, 0) : edge[slot][wl][2];
    const double yl1 = (wid == 0) ? readlane(yh, 1) : edge[slot][wl][3];
    const double yr1 = (wid == WPB - 1) ? readlane(yh, 2) : edge[slot][wr][0];
    const double yr2 = (wid == WPB - 1) ? readlane(yh, 3) : edge[slot][wr][1];
    const double su1 = __shfl_up(y, 1, 64), sd1 = __shfl_down(y, 1, 64);
    const double su2 = __shfl_up(y, 2, 64), sd2 = __shfl_down(y, 2, 64);
    const double l1 = (lane == 0) ? yl1 : su1;
    const double r1v = (lane == 63) ? yr1 : sd1;
    const double l2 = (lane == 0) ? yl2 : ((lane == 1) ? yl1 : su2);
    const double r2v = (lane == 63) ? yr2 : ((lane == 62) ? yr1 : sd2);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      yw[m] = yw[m + 1];
      hw[m] = hw[m + 1];
      h2w[m] = h2w[m + 1];
      vw[m] = vw[m + 1];
    }
    yw[4] = y;
    hw[4] = l1 + r1v;
    h2w[4] = l2 + r2v;
    vw[4] = v;
    const bool st = own && q >= r0 && q < r1;
    stb(rv, st ? uint32_t((q * nx + col) * 8) : kOOB, v);
  };

  double aw[NV], ag[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) aw[i] = ag[i] = 0.0;
  double awn = 0.0, avv = 0.0, aww = 0.0;
  // stencil + dot products of row r (window centre = row r; basis row r from LDS)
  auto centre = [&](int64_t r) {
    const double (*d)[64] = lg[(r - r0) & 1];
    const double yc = yw[2];
    const double a1 = hw[2] + (yw[1] + yw[3]);
    const double dg = hw[1] + hw[3];
    const double a2 = h2w[2] + (yw[0] + yw[4]);
    const double Ly = applyL13(K, yc, a1, dg, a2);
    const double yy = yc * yc;
    const double G = yc / K.k - (Ly + K.g * yy - yc * yy) / 2;
    const double wo = (G - d[NV][lane]) * isc;
    const bool in = own && r < r1;
    stb(rw, in ? uint32_t((r * nx + col) * 8) : kOOB, wo);
    const double wm = in ? wo : 0.0;
    const double vm = in ? vw[2] : 0.0;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const double bi = d[i][lane];
      aw[i] += wm * bi;
      ag[i] += vm * bi;
    }
    awn += wm * vm;
    avv += vm * vm;
    aww += wm * wm;
  };

  if (nrows > 0) {
    // prologue: rows r0-2, r0-1 (band halo), r0, r0+1 enter the window (r0, r0+1 also the
    // LDS lag); rows r0+2 .. r0+1+PF go in flight.  Row q >= r0+2 uses register slot
    // (q - r0 - 2) mod RR.
    // (at most max(4, 2 + PF) rows of loads live at once: the register peak of the kernel)
    Slot P[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) load(P[d], r0 - 2 + d);
    push(P[0], r0 - 2);
    push(P[1], r0 - 1);
    Slot S[RR];
#pragma unroll
    for (int d = 0; d < PF; ++d) load(S[d], r0 + 2 + d);
    push(P[2], r0);
    push(P[3], r0 + 1);
    stash(P[2], r0);
    stash(P[3], r0 + 1);
    // whole groups of RR rows with no branch inside the group (a branch would make the
    // compiler's wait-count analysis drain every load in flight): rows past the band end are
    // computed on clamped rows and masked out of the stores and sums
    for (int64_t t0 = 0; t0 < nrows; t0 += RR) {
#pragma unroll
      for (int k = 0; k < RR; ++k) {
        const int64_t r = r0 + t0 + k;
        load(S[(k + PF) % RR], r + 2 + PF);  // the slot of row r+1, consumed last step
        push(S[k], r + 2);
        centre(r);
        stash(S[k], r + 2);  // into the LDS slot row r just vacated
      }
    }
  }

  // one partial per wave: [w'.V_i (nv)] [w'.v] [v.V_i (nv)] [v.v] [w'.w']
  wave_sum<NV>(aw);
  wave_sum<NV>(ag);
  double t3[3] = {awn, avv, aww};
  wave_sum<3>(t3);
  if (lane == 0) {
    const int64_t nw = ngroups * WPB * A.nbands;  // every wave of every block writes a column
    double* p = A.partial + gw;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      p[int64_t(i) * nw] = aw[i];
      p[int64_t(NV + 1 + i) * nw] = ag[i];
    }
    p[int64_t(NV) * nw] = t3[0];
    p[int64_t(2 * NV + 1) * nw] = t3[1];
    p[int64_t(2 * NV + 2) * nw] = t3[2];
  }
}

int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::atoi(v) : dflt;
}

struct Occ {
  int ncu = 0, blocks_per_cu = 0;
};

template <int NV, bool EXT, int PF, bool NT>
hipError_t launch_t(ArnoldiArgs A, hipStream_t s, int64_t* nwaves) {
  auto kern = arnoldi_kernel<NV, EXT, PF, NT>;
  static Occ occ;  // per instantiation
  if (occ.ncu == 0) {
    int dev = 0, ncu = 0, nb = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, 64 * WPB, 0) != hipSuccess)
      return hipErrorUnknown;
    occ.blocks_per_cu = nb > 0 ? nb : 1;
    occ.ncu = ncu > 0 ? ncu : 1;
  }
  // one resident round of waves (NKHIP_ARN_ROUNDS scales it); bands of >= 8 rows, and no more
  // partial columns than the caller's buffer holds
  static const int rounds = env_int("NKHIP_ARN_ROUNDS", 1);
  const int64_t strips = (A.nx + kSW - 1) / kSW;
  const int64_t target = int64_t(occ.ncu) * occ.blocks_per_cu * WPB * (rounds > 0 ? rounds : 1);
  const int64_t wpr = (strips + WPB - 1) / WPB * WPB;  // waves per band (whole blocks)
  int64_t nbands = target / wpr;
  const int64_t cap_bands = A.partial_cap / ((2 * int64_t(NV) + 3) * wpr);
  if (nbands > cap_bands) nbands = cap_bands;
  if (nbands > A.ny / 8) nbands = A.ny / 8;
  if (nbands < 1) nbands = 1;
  const int64_t RY = (A.ny + nbands - 1) / nbands;
  nbands = (A.ny + RY - 1) / RY;
  const int64_t nw = wpr * nbands;
  if (nw * (2 * int64_t(NV) + 3) > A.partial_cap) return hipErrorInvalidValue;
  A.strips = int(strips);
  A.nbands = int(nbands);
  A.RY = int(RY);
  int64_t blocks = (nw + WPB - 1) / WPB;
  blocks = (blocks + 7) / 8 * 8;
  *nwaves = nw;
  hipLaunchKernelGGL(kern, dim3(unsigned(blocks)), dim3(64 * WPB), 0, s, A);
  return hipGetLastError();
}

template <int NV, bool EXT>
hipError_t launch_pf(const ArnoldiArgs& A, hipStream_t s, int64_t* nwaves) {
  static const bool nt = env_int("NKHIP_ARN_NT", 1) != 0;
  constexpr int PF = pf_for(NV);
#ifdef NKHIP_ARN_TUNE  // tuning build (`make tune`): NKHIP_ARN_PF selects the rows in flight
  static const int pf = env_int("NKHIP_ARN_PF", 0);
  if constexpr (NV % 4 == 0) {
    switch (pf) {
      case 1: return launch_t<NV, EXT, 1, true>(A, s, nwaves);
      case 2: return launch_t<NV, EXT, 2, true>(A, s, nwaves);
      case 3: return launch_t<NV, EXT, 3, true>(A, s, nwaves);
      case 4: return launch_t<NV, EXT, 4, true>(A, s, nwaves);
      case 6: return launch_t<NV, EXT, 6, true>(A, s, nwaves);
      default: break;
    }
  }
#endif
  return nt ? launch_t<NV, EXT, PF, true>(A, s, nwaves) : launch_t<NV, EXT, PF, false>(A, s, nwaves);
}

template <bool EXT, int NV = 1>
hipError_t launch_e(const ArnoldiArgs& A, hipStream_t s, int64_t* nwaves) {
  if constexpr (NV > kArnMaxNV) {
    return hipErrorInvalidValue;
  } else {
    if (A.nv == NV) return launch_pf<NV, EXT>(A, s, nwaves);
    return launch_e<EXT, NV + 1>(A, s, nwaves);
  }
}

}  // namespace

bool arnoldi_supported(int nv, int64_t ny, int64_t nx) {
  static const int maxnv = env_int("NKHIP_ARN_MAXNV", kArnMaxNV);
  return nv >= 1 && nv <= kArnMaxNV && nv <= maxnv && ny >= 8 && nx >= 4 &&
         ny * nx * 8 < (int64_t(1) << 32);  // 32-bit byte offsets
}

hipError_t arnoldi_launch(const ArnoldiArgs& A, hipStream_t s, int64_t* nwaves) {
  if (!arnoldi_supported(A.nv, A.ny, A.nx)) return hipErrorInvalidValue;
  if (A.z) return launch_e<true>(A, s, nwaves);
  return launch_e<false>(A, s, nwaves);
}

}  // namespace nk

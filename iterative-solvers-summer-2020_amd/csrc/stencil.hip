// Matrix-free stencil kernels of the Swift-Hohenberg Crank-Nicolson residual (gfx950).
//
// Replaces the scipy CSR SpMVs `Lap @ v` / `L @ u` and the NumPy element-wise passes of
// residual() (sh_scipy_nk.py:32-49) and the Eigen SpMV of the C++ twin (main.cpp:19-32):
// no matrix is stored, the 13 coefficients are closed-form (nk::sh_coef).
//
// Fast path ("march"): a thread owns two adjacent columns (one 16-B double2 per row and field),
// a block owns 2*BX columns x RY rows and marches down its rows keeping a 5-row register window
// (3 rows for the 5-point Laplacian).  Each input row enters the window with three coalesced
// double2 loads (columns c-2.., c.., c+2..); the side loads are L1/L2 hits shared with the
// neighbouring lanes, so HBM sees each input byte once per block plus the 2*R halo rows.
// The next row is prefetched one iteration ahead.  Requires nx even and 16-B aligned rows.
// Generic path ("point"): one output per thread with modular indexing (odd nx, e.g. 61x61).
#include <cmath>
#include <cstdlib>

#include "nk_device.h"
#include "nk_kernels.h"
#include "peer_dev.h"

namespace nk {

SHCoef sh_coef(double h, double r, double k, double g) {
  const double e = 1.0 / (h * h);
  SHCoef c;
  c.c0 = -20.0 * e * e + 8.0 * e + r - 1.0;
  c.c1 = 8.0 * e * e - 2.0 * e;
  c.c2 = -2.0 * e * e;
  c.c3 = -e * e;
  c.k = k;
  c.ik = 1.0 / k;
  c.g = g;
  return c;
}

namespace {

struct Nb {
  double c, a1, dg, a2;  // centre, axial +-1 sum, diagonal sum, axial +-2 sum
};

struct Res {
  double o0, o1, o2;
};

__device__ __forceinline__ const double* rowp(const Field& f, int64_t r, int64_t ny, int64_t nx) {
  if (r >= 0 && r < ny) return f.base + r * nx;
  if (f.lo == nullptr) {
    r %= ny;
    if (r < 0) r += ny;
    return f.base + r * nx;
  }
  return (r < 0) ? f.lo + (r + 2) * nx : f.hi + (r - ny) * nx;
}

// Row pointer for the march kernel: lo/hi are always set there (the launcher points them into
// the slab itself for a periodic single slab), so the choice is two scalar selects.
__device__ __forceinline__ const double* rowp_fast(const Field& f, int64_t r, int64_t ny,
                                                   int64_t nx) {
  const double* b = (r < 0) ? f.lo : ((r >= ny) ? f.hi : f.base);
  const int64_t rr = (r < 0) ? r + 2 : ((r >= ny) ? r - ny : r);
  return b + rr * nx;
}

__device__ __forceinline__ double applyL(const SHCoef& k, const Nb& n) {
  return k.c0 * n.c + k.c1 * n.a1 + k.c2 * n.dg + k.c3 * n.a2;
}

// G(w) = w/k - (L w + g w^2 - w^3)/2, so that F(u) = G(u) + B(uo) (sh_scipy_nk.py:49).  The
// solver's kernels all scale by the host-rounded 1/k (no per-point division); the reference
// residual (RESID) keeps the reference's (u - Uo)/k.
__device__ __forceinline__ double Gfun(const SHCoef& k, double w, double Lw) {
  const double ww = w * w;
  return w * k.ik - (Lw + k.g * ww - w * ww) / 2;
}

template <SMode M>
__device__ __forceinline__ Res finish(const StencilArgs& A, const Nb& na, const Nb& nb, double pv,
                                      double alpha, double sc) {
  Res r{0.0, 0.0, 0.0};
  const SHCoef& k = A.c;
  if constexpr (M == SMode::LAP5) {
    r.o0 = A.e * (na.a1 - 4.0 * na.c);
  } else if constexpr (M == SMode::SH13) {
    r.o0 = applyL(k, na);
  } else if constexpr (M == SMode::RESID) {
    const double u = na.c, uo = nb.c;
    const double uu = u * u, uouo = uo * uo;
    r.o0 = (u - uo) / k.k -
           (applyL(k, na) + k.g * uu - u * uu + applyL(k, nb) + k.g * uouo - uo * uouo) / 2;
  } else if constexpr (M == SMode::BOLD) {
    const double uo = na.c;
    const double uouo = uo * uo;
    r.o0 = -uo * k.ik - (applyL(k, na) + k.g * uouo - uo * uouo) / 2;
  } else if constexpr (M == SMode::TRIAL) {
    const double G = Gfun(k, na.c, applyL(k, na));
    r.o0 = G + pv;
    r.o1 = G;
    r.o2 = na.c;
  } else if constexpr (M == SMode::FDJVP) {
    r.o0 = (Gfun(k, na.c, applyL(k, na)) - pv) * sc;  // sc = 1/step here
  } else if constexpr (M == SMode::LINOP) {
    r.o0 = (1.0 + pv) * na.c - A.theta * applyL(k, na);
    r.o2 = na.c;
  } else {  // AJVP
    const double z = na.c, u = pv;
    r.o0 = alpha * (z * k.ik - (applyL(k, na) + (2.0 * k.g * u - 3.0 * u * u) * z) / 2);
  }
  return r;
}

template <SMode M>
constexpr bool kComb = (M == SMode::TRIAL || M == SMode::FDJVP || M == SMode::LINOP);
template <SMode M>
constexpr bool kRed = (M == SMode::TRIAL || M == SMode::LINOP);
template <SMode M>
constexpr bool kTwo = (M == SMode::RESID);
template <SMode M>
constexpr bool kHasP0 =
    (M == SMode::TRIAL || M == SMode::FDJVP || M == SMode::AJVP || M == SMode::LINOP);
template <SMode M>
constexpr int kRad = (M == SMode::LAP5) ? 1 : 2;

// JVP scale: either from the host (A.alpha, A.sc) or, when A.znorm2 is set, from the device
// norm |z_raw|^2 left by the previous fused update (KrylovJacobian.matvec with v = z_raw/|z_raw|:
// sc = omega/|v|, step = sc/|z_raw|), so the host need not synchronise before the JVP.
template <SMode M>
__device__ __forceinline__ bool jvp_scale(const StencilArgs& A, double* alpha, double* sc) {
  *alpha = A.alpha;
  *sc = A.sc;
  bool go = true;  // false: a speculative JVP the trial's outcome cancelled (the pass does nothing)
  if constexpr (M == SMode::FDJVP || M == SMode::AJVP) {
    if (A.znorm2) {
      const double hn = sqrt(*A.znorm2);
      double sig = 1.0 / hn;
      if (!isfinite(sig)) sig = 1.0;
      if constexpr (M == SMode::FDJVP) {
        *sc = A.omega / (sig * hn);
        *alpha = *sc * sig;
      } else {
        *alpha = sig;
      }
    }
  }
  if constexpr (M == SMode::FDJVP) {
    if (A.spec) {  // the same expressions, in the same order, as the host's (NewtonKrylov)
      const double red0 = A.spec[0], fm = A.spec[1], xm = A.spec[2];
      go = isfinite(red0) && red0 <= A.spec_thr && !(fm <= A.spec_ftol);
      const double omega = A.spec_rdiff * fmax(1.0, xm) / fmax(1.0, fm);
      *sc = omega / A.spec_zn;
      *alpha = *sc * A.spec_zs;
    }
    *sc = 1.0 / *sc;  // finish() scales by the reciprocal
  }
  return go;
}

// The point-wise input (G0, B, u or D) is streamed once per pass: optionally non-temporal, so it
// does not evict the stencil fields from L2 / the Infinity Cache.
typedef double dv2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 ld_p0(const StencilArgs& A, const double* p) {
  if (A.nt_p0) {
    const dv2 v = __builtin_nontemporal_load(reinterpret_cast<const dv2*>(p));
    return make_double2(v.x, v.y);
  }
  return *reinterpret_cast<const double2*>(p);
}

// ------------------------------------------------------------------------------------------
// march kernel
// ------------------------------------------------------------------------------------------
// A band of rows is walked with a ring of RING = NR + PF row slots: NR rows form the stencil
// window, PF more are in flight.  The walk is unrolled by RING, so the window "shift" is a
// compile-time renaming of ring slots, not a register copy: a copy would need the freshly loaded
// row to have arrived, and the in-order vmcnt would then drain every load at the end of each
// row (the previous design's limit: one row of loads in flight per wave).  Here the compute of
// row r waits only for the loads issued PF rows earlier.  Raw rows are kept per field; the FD
// combination a + alpha*b is formed when a row is first used, not when it is loaded.
template <SMode M>
constexpr int kFields = (kComb<M> || kTwo<M>) ? 2 : 1;

// Grid: gx column blocks x gy bands, launched as one dimension rounded up to a multiple of 8 and
// mapped XCD-aware: the hardware deals consecutive workgroups round-robin over the 8 XCDs, so
// logical block L = (b % 8) (blocks / 8) + b / 8 gives each XCD one contiguous run of whole
// bands.  The two neighbouring column blocks of a band (whose edge lines a block's c-2 / c+2 side
// loads touch) and the neighbouring bands (whose halo rows it re-reads) then share one L2: with
// the plain mapping adjacent column blocks sat on different XCDs and every block edge line was
// fetched from HBM twice (FD JVP traffic 1.107x algorithmic, profiles/r02f_traffic.json).
template <SMode M, int BX, int PF>
__global__ void __launch_bounds__(BX) march_kernel(StencilArgs A, int RY, int gx, int gy) {
  constexpr int R = kRad<M>;
  constexpr int NR = 2 * R + 1;
  constexpr int RING = NR + PF;
  constexpr int NF = kFields<M>;
  const int64_t nx = A.nx, ny = A.ny;
  const int64_t lb = (int64_t(blockIdx.x) % 8) * (int64_t(gridDim.x) / 8) + blockIdx.x / 8;
  if (lb >= int64_t(gx) * gy) return;  // padding of the grid to a multiple of 8
  const int64_t bx = lb % gx, by = lb / gx;
  const int64_t c0 = 2 * (bx * BX + threadIdx.x);
  const bool active = c0 < nx;
  const int64_t cc = active ? c0 : 0;
  const int64_t cm = (cc >= 2) ? cc - 2 : cc - 2 + nx;
  const int64_t cp = (cc + 2 < nx) ? cc + 2 : cc + 2 - nx;
  double alpha, sc;
  if (!jvp_scale<M>(A, &alpha, &sc)) return;  // uniform: a cancelled speculative JVP

  // the block's side columns (two each side) of an own row from the fields' edge arrays: the
  // first thread's c-2, c-1 are boundary B0's slots 0, 1, the last thread's c+2, c+3 boundary
  // B0 + 2 BX's slots 2, 3 (nk_kernels.h edge layout; 2 BX == kEdgeW)
  static_assert(2 * BX == kEdgeW, "a march block is one edge group wide");
  const int64_t nbE = edge_groups(nx);
  const int64_t eL = (cc / kEdgeW) * A.e_ny * 4, eR = (((cc + 2) / kEdgeW) % nbE) * A.e_ny * 4 + 2;
  const bool sideL = threadIdx.x == 0, sideR = threadIdx.x == BX - 1;
  auto ld = [&](const Field& f, const double* E, int64_t r, double (&v)[6]) {
    const double* p = rowp_fast(f, r, ny, nx);
    const double* pl = p + cm;
    const double* pr = p + cp;
    if (E && r >= 0 && r < ny) {  // own rows of this launch (halo rows come from lo / hi)
      const int64_t er = (A.e_row0 + r) * 4;
      pl = sideL ? E + eL + er : pl;
      pr = sideR ? E + eR + er : pr;
    }
    const double2 x0 = *reinterpret_cast<const double2*>(pl);
    const double2 x1 = *reinterpret_cast<const double2*>(p + cc);
    const double2 x2 = *reinterpret_cast<const double2*>(pr);
    v[0] = x0.x; v[1] = x0.y; v[2] = x1.x; v[3] = x1.y; v[4] = x2.x; v[5] = x2.y;
  };
  // ring[f][slot][6]: raw rows of field f (a, then b)
  double ring[NF][RING][6];
  auto load_row = [&](int slot, int64_t r) {
    r = (r > ny + 1) ? ny + 1 : ((r < -2) ? -2 : r);  // past the band: a valid halo / edge row
    ld(A.a, A.Ea, r, ring[0][slot]);
    if constexpr (NF == 2) ld(A.b, A.Eb, r, ring[1][slot]);
  };
  // a + alpha b, formed once when the row enters the window
  auto combine = [&](int slot) {
    if constexpr (kComb<M>) {
#pragma unroll
      for (int q = 0; q < 6; ++q) ring[0][slot][q] = ring[0][slot][q] + alpha * ring[1][slot][q];
    }
  };
  auto ldp = [&](int64_t r) {
    r = (r >= ny) ? ny - 1 : ((r < 0) ? 0 : r);
    return ld_p0(A, A.p0 + r * nx + cc);
  };

  // Odd bands march upwards: a band boundary is then reached by both adjacent bands at the same
  // time (both at their start or both at their end), so the halo rows one band re-reads are still
  // in L2.  The window sums pair the rows symmetrically about the centre, so the result is
  // bitwise the same in either direction (fp addition is commutative).
  // A.rev walks the bands from the top of the grid (see traversal_reverse)
  const int64_t band = A.rev ? int64_t(gy) - 1 - by : by;
  const int64_t r0 = band * RY;
  const int64_t r1 = (r0 + RY < ny) ? r0 + RY : ny;
  const bool up = (band & 1) != 0;
  const int64_t dir = up ? -1 : 1;
  const int64_t rs = up ? r1 - 1 : r0;
  const int64_t nrows = r1 - r0;

  // prologue: slot k holds row rs + dir*(k - R) (window rows and PF - 1 rows in flight)
#pragma unroll
  for (int k = 0; k < RING - 1; ++k) load_row(k, rs + dir * (k - R));
  double2 pq[RING];
#pragma unroll
  for (int d = 0; d < RING; ++d) pq[d] = make_double2(0.0, 0.0);
  if constexpr (kHasP0<M>) {
#pragma unroll
    for (int d = 0; d < PF; ++d) pq[d] = ldp(rs + dir * d);
  }
#pragma unroll
  for (int k = 0; k < NR - 1; ++k) combine(k);

  double red[3] = {0.0, 0.0, 0.0};
  bool pushed = false;  // this thread wrote rows into a neighbour's halo slot (drained at the end)
  // a pushed edge row (global slab row g of e_ny) of an output into the neighbours' slots,
  // written through (store_sys16)
  auto push_row = [&](double* const* ps, int64_t g, double2 v) {
    const bool top = g < 2, bot = g >= A.e_ny - 2;
    if (!(top || bot)) return;
    double* d = top ? ps[0] + (2 + g) * A.ps_ld : ps[1] + (g - (A.e_ny - 2)) * A.ps_ld;
    store_sys16(d + cc, v.x, v.y);
    pushed = true;
  };
  for (int64_t base = 0; base < nrows; base += RING) {
#pragma unroll
    for (int u = 0; u < RING; ++u) {
      const int64_t it = base + u;  // rows past the band end are computed but not stored
      const int64_t r = rs + dir * it;
      load_row((u + RING - 1) % RING, r + dir * (R + PF));
      if constexpr (kHasP0<M>) pq[(u + PF) % RING] = ldp(r + dir * PF);
      combine((u + NR - 1) % RING);
      const double2 pv = pq[u % RING];
      auto W = [&](int m, int q) -> double { return ring[0][(u + m) % RING][q]; };
      auto Wb = [&](int m, int q) -> double { return ring[NF - 1][(u + m) % RING][q]; };
      Res res[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        Nb na, nb{0.0, 0.0, 0.0, 0.0};
        if constexpr (R == 2) {
          na.c = W(2, 2 + q);
          na.a1 = (W(2, 1 + q) + W(2, 3 + q)) + (W(1, 2 + q) + W(3, 2 + q));
          na.dg = (W(1, 1 + q) + W(1, 3 + q)) + (W(3, 1 + q) + W(3, 3 + q));
          na.a2 = (W(2, q) + W(2, 4 + q)) + (W(0, 2 + q) + W(4, 2 + q));
          if constexpr (kTwo<M>) {
            nb.c = Wb(2, 2 + q);
            nb.a1 = (Wb(2, 1 + q) + Wb(2, 3 + q)) + (Wb(1, 2 + q) + Wb(3, 2 + q));
            nb.dg = (Wb(1, 1 + q) + Wb(1, 3 + q)) + (Wb(3, 1 + q) + Wb(3, 3 + q));
            nb.a2 = (Wb(2, q) + Wb(2, 4 + q)) + (Wb(0, 2 + q) + Wb(4, 2 + q));
          }
        } else {
          na.c = W(1, 2 + q);
          na.a1 = (W(1, 1 + q) + W(1, 3 + q)) + (W(0, 2 + q) + W(2, 2 + q));
          na.dg = 0.0;
          na.a2 = 0.0;
        }
        res[q] = finish<M>(A, na, nb, q == 0 ? pv.x : pv.y, alpha, sc);
      }
      if (active && it < nrows) {
        const int64_t o = r * nx + cc;
        *reinterpret_cast<double2*>(A.out0 + o) = make_double2(res[0].o0, res[1].o0);
        if (A.PS0[0]) push_row(A.PS0, A.e_row0 + r, make_double2(res[0].o0, res[1].o0));
        if (A.E0) {  // the edge array: E[(b e_ny + row) 4 + 0..3] = columns B-2, B-1, B, B+1
          const int64_t er = A.e_row0 + r;
          const double2 ev = make_double2(res[0].o0, res[1].o0);
          if (cc % kEdgeW == 0)
            *reinterpret_cast<double2*>(A.E0 + ((cc / kEdgeW) * A.e_ny + er) * 4 + 2) = ev;
          if ((cc + 2) % kEdgeW == 0 || cc + 2 == nx) {
            const int64_t b = (cc + 2 == nx) ? 0 : (cc + 2) / kEdgeW;
            *reinterpret_cast<double2*>(A.E0 + (b * A.e_ny + er) * 4) = ev;
          }
        }
        if constexpr (M == SMode::TRIAL) {
          *reinterpret_cast<double2*>(A.out1 + o) = make_double2(res[0].o1, res[1].o1);
          if (A.out2) *reinterpret_cast<double2*>(A.out2 + o) = make_double2(res[0].o2, res[1].o2);
          if (A.PS2[0]) push_row(A.PS2, A.e_row0 + r, make_double2(res[0].o2, res[1].o2));
          if (A.E2) {  // out2's edge array, as out0's above
            const int64_t er = A.e_row0 + r;
            const double2 ev = make_double2(res[0].o2, res[1].o2);
            if (cc % kEdgeW == 0)
              *reinterpret_cast<double2*>(A.E2 + ((cc / kEdgeW) * A.e_ny + er) * 4 + 2) = ev;
            if ((cc + 2) % kEdgeW == 0 || cc + 2 == nx) {
              const int64_t b = (cc + 2 == nx) ? 0 : (cc + 2) / kEdgeW;
              *reinterpret_cast<double2*>(A.E2 + (b * A.e_ny + er) * 4) = ev;
            }
          }
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            red[0] += res[q].o0 * res[q].o0;
            red[1] = nmax(red[1], fabs(res[q].o0));
            red[2] = nmax(red[2], fabs(res[q].o2));
          }
        } else if constexpr (M == SMode::LINOP) {
          *reinterpret_cast<double2*>(A.out2 + o) = make_double2(res[0].o2, res[1].o2);
#pragma unroll
          for (int q = 0; q < 2; ++q) red[0] += res[q].o2 * res[q].o0;
        }
      }
    }
  }
  if (pushed) drain_stores();  // the pushed rows, before the pass ends
  if constexpr (kRed<M>) {
    const double v = block_reduce<3, 1, BX>(red);
    const int64_t nblk = int64_t(gx) * gy;
    const int64_t bid = band * gx + bx;  // slot by band: independent of A.rev
    if (threadIdx.x < 3) A.partial[threadIdx.x * nblk + bid] = v;
  }
}

// ------------------------------------------------------------------------------------------
// generic point kernel (any nx, any alignment)
// ------------------------------------------------------------------------------------------
template <SMode M>
__global__ void __launch_bounds__(256) point_kernel(StencilArgs A) {
  constexpr int R = kRad<M>;
  const int64_t nx = A.nx, ny = A.ny;
  const int64_t idx = int64_t(blockIdx.x) * 256 + threadIdx.x;
  const bool active = idx < nx * ny;
  double alpha, sc;
  if (!jvp_scale<M>(A, &alpha, &sc)) return;  // uniform: a cancelled speculative JVP
  double red[3] = {0.0, 0.0, 0.0};
  if (active) {
    const int64_t i = idx / nx, j = idx % nx;
    auto col = [&](int64_t dj) {
      int64_t c = (j + dj) % nx;
      if (c < 0) c += nx;
      return c;
    };
    auto val = [&](const Field& f, int64_t di, int64_t dj) {
      return rowp(f, i + di, ny, nx)[col(dj)];
    };
    auto wv = [&](int64_t di, int64_t dj) {
      double v = val(A.a, di, dj);
      if constexpr (kComb<M>) v = v + alpha * val(A.b, di, dj);
      return v;
    };
    Nb a, b{0.0, 0.0, 0.0, 0.0};
    a.c = wv(0, 0);
    a.a1 = (wv(0, -1) + wv(0, 1)) + (wv(-1, 0) + wv(1, 0));
    if constexpr (R == 2) {
      a.dg = (wv(-1, -1) + wv(-1, 1)) + (wv(1, -1) + wv(1, 1));
      a.a2 = (wv(0, -2) + wv(0, 2)) + (wv(-2, 0) + wv(2, 0));
    } else {
      a.dg = 0.0;
      a.a2 = 0.0;
    }
    if constexpr (kTwo<M>) {
      b.c = val(A.b, 0, 0);
      b.a1 = (val(A.b, 0, -1) + val(A.b, 0, 1)) + (val(A.b, -1, 0) + val(A.b, 1, 0));
      b.dg = (val(A.b, -1, -1) + val(A.b, -1, 1)) + (val(A.b, 1, -1) + val(A.b, 1, 1));
      b.a2 = (val(A.b, 0, -2) + val(A.b, 0, 2)) + (val(A.b, -2, 0) + val(A.b, 2, 0));
    }
    double pv = 0.0;
    if constexpr (kHasP0<M>) pv = A.p0[idx];
    const Res res = finish<M>(A, a, b, pv, alpha, sc);
    A.out0[idx] = res.o0;
    if constexpr (M == SMode::TRIAL) {
      A.out1[idx] = res.o1;
      if (A.out2) A.out2[idx] = res.o2;
      red[0] = res.o0 * res.o0;
      red[1] = fabs(res.o0);
      red[2] = fabs(res.o2);
    } else if constexpr (M == SMode::LINOP) {
      A.out2[idx] = res.o2;
      red[0] = res.o2 * res.o0;
    }
  }
  if constexpr (kRed<M>) {
    const double v = block_reduce<3, 1, 256>(red);
    if (threadIdx.x < 3) A.partial[threadIdx.x * int64_t(gridDim.x) + blockIdx.x] = v;
  }
}

// ------------------------------------------------------------------------------------------
// tile kernel: the pure operators (Lap v, L v) on small grids (config 2: 1024^2 in 6.4 us by the
// march, 4 rows per band).  A thread owns two adjacent columns of ROWS rows and issues all of its
// loads at once (3 x 16 B per window row, as the march's ld(): columns c-2.., c.., c+2..), so a
// launch is one round of memory latency; non-temporal stores by default.  Blocks map to rows
// XCD by XCD and never reversed: each XCD reads the same rows every launch, whose 2 x 1 MB slice
// (input and output) stays in its 4 MB L2 between back-to-back launches.  Same neighbour sums in
// the same order as the march kernel: bitwise its results.
// ------------------------------------------------------------------------------------------
template <SMode M, int ROWS, bool NTS>
__global__ void __launch_bounds__(256) tile_kernel(StencilArgs A, int gxt) {
  constexpr int R = kRad<M>;
  constexpr int NR = 2 * R + ROWS;  // window rows of ROWS output rows
  const int64_t nx = A.nx, ny = A.ny;
  const int64_t lb = (int64_t(blockIdx.x) % 8) * (int64_t(gridDim.x) / 8) + blockIdx.x / 8;
  const int64_t nrb = (ny + ROWS - 1) / ROWS;
  if (lb >= int64_t(gxt) * nrb) return;  // padding of the grid to a multiple of 8
  const int64_t r0 = (lb / gxt) * ROWS;
  const int64_t c0 = 2 * ((lb % gxt) * 256 + threadIdx.x);
  if (c0 >= nx) return;
  const int64_t cm = (c0 >= 2) ? c0 - 2 : c0 - 2 + nx;
  const int64_t cp = (c0 + 2 < nx) ? c0 + 2 : c0 + 2 - nx;
  double w[NR][6];
#pragma unroll
  for (int m = 0; m < NR; ++m) {
    int64_t rr = r0 + m - R;
    rr = (rr > ny + 1) ? ny + 1 : rr;  // rows past a short last block: a valid (halo) row
    const double* p = rowp_fast(A.a, rr, ny, nx);
    const double2 x0 = *reinterpret_cast<const double2*>(p + cm);
    const double2 x1 = *reinterpret_cast<const double2*>(p + c0);
    const double2 x2 = *reinterpret_cast<const double2*>(p + cp);
    w[m][0] = x0.x; w[m][1] = x0.y; w[m][2] = x1.x; w[m][3] = x1.y; w[m][4] = x2.x; w[m][5] = x2.y;
  }
#pragma unroll
  for (int t = 0; t < ROWS; ++t) {
    Res res[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      Nb na, nb{0.0, 0.0, 0.0, 0.0};
      if constexpr (R == 2) {
        na.c = w[t + 2][2 + q];
        na.a1 = (w[t + 2][1 + q] + w[t + 2][3 + q]) + (w[t + 1][2 + q] + w[t + 3][2 + q]);
        na.dg = (w[t + 1][1 + q] + w[t + 1][3 + q]) + (w[t + 3][1 + q] + w[t + 3][3 + q]);
        na.a2 = (w[t + 2][q] + w[t + 2][4 + q]) + (w[t][2 + q] + w[t + 4][2 + q]);
      } else {
        na.c = w[t + 1][2 + q];
        na.a1 = (w[t + 1][1 + q] + w[t + 1][3 + q]) + (w[t][2 + q] + w[t + 2][2 + q]);
        na.dg = 0.0;
        na.a2 = 0.0;
      }
      res[q] = finish<M>(A, na, nb, 0.0, 0.0, 1.0);
    }
    if (r0 + t < ny) {
      dv2* o = reinterpret_cast<dv2*>(A.out0 + (r0 + t) * nx + c0);
      const dv2 v{res[0].o0, res[1].o0};
      if constexpr (NTS)
        __builtin_nontemporal_store(v, o);
      else
        *o = v;
    }
  }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::atoi(v) : dflt;
}

bool field_ok(const Field& f) {
  return f.base == nullptr ||
         (aligned16(f.base) && (f.lo == nullptr || (aligned16(f.lo) && aligned16(f.hi))));
}

template <SMode M>
hipError_t launch_mode(const StencilArgs& A, hipStream_t s, int64_t* nblk) {
  const bool fast = (A.nx % 2 == 0) && A.nx >= 2 && A.ny >= 2 && field_ok(A.a) && field_ok(A.b) &&
                    aligned16(A.p0) && aligned16(A.out0) && aligned16(A.out1) && aligned16(A.out2);
  if (fast) {
    StencilArgs B = A;  // periodic single slab: halo rows are rows ny-2, ny-1 and 0, 1
    for (Field* f : {&B.a, &B.b}) {
      if (f->base && !f->lo) {
        f->lo = f->base + (A.ny - 2) * A.nx;
        f->hi = f->base;
      }
    }
    // The pure operators on a grid of at most NKHIP_TILE_MAX points (default 2^21: 16.8 MB for
    // input and output at 1024^2, L2-resident per XCD): one row per thread, the tile kernel
    if constexpr (M == SMode::LAP5 || M == SMode::SH13) {
      static const int64_t tile_max = env_int("NKHIP_TILE_MAX", 1 << 21);
      if (A.nx * A.ny <= tile_max && !A.E0 && !A.PS0[0]) {
        // rows per thread and the store policy (NKHIP_TILE_ROWS 1 / 2 / 4, NKHIP_TILE_NT): at
        // 1024^2, rocprofv3, one box (profiles/r05_config2.md): march 6.43 us; rows 1 / 2 / 4
        // 5.93 / 5.13 / 5.21 us with plain stores, 5.18-5.41 / 4.83 / 4.80-4.86 us non-temporal
        static const int rows = env_int("NKHIP_TILE_ROWS", 2);
        static const bool nts = env_int("NKHIP_TILE_NT", 1) != 0;
        const int rt = (rows == 4 || rows == 2) ? rows : 1;
        const int gxt = int((A.nx / 2 + 255) / 256);
        const int64_t nb = int64_t(gxt) * ((A.ny + rt - 1) / rt);
        if (nblk) *nblk = nb;
        const dim3 grid{unsigned((nb + 7) / 8 * 8), 1u, 1u};
        auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, dim3(256), 0, s, B, gxt); };
        if (rt == 4)
          nts ? go(tile_kernel<M, 4, true>) : go(tile_kernel<M, 4, false>);
        else if (rt == 2)
          nts ? go(tile_kernel<M, 2, true>) : go(tile_kernel<M, 2, false>);
        else
          nts ? go(tile_kernel<M, 1, true>) : go(tile_kernel<M, 1, false>);
        return hipGetLastError();
      }
    }
    // Row band per block: a multiple of the ring length RING (the unroll of the walk), aiming at
    // >= ~4096 blocks (16 per CU) for the grid (NKHIP_BLOCKS / NKHIP_PF override for tuning).
    static const int blocks = env_int("NKHIP_BLOCKS", 4096);
    static const int pf = env_int("NKHIP_PF", 1);
    constexpr int BX = 128;
    constexpr int R = kRad<M>;
    const int ring = 2 * R + 1 + (pf == 2 ? 2 : 1);
    const int64_t gx = (A.nx / 2 + BX - 1) / BX;
    const int64_t want = (A.ny * gx) / blocks;  // rows per band for `blocks` blocks
    int64_t k = (want + ring / 2) / ring;
    if (k < 1) k = 1;
    if (k > 6) k = 6;
    const int RY = int(k * ring);
    const int64_t gy = (A.ny + RY - 1) / RY;
    if (gx * gy > (int64_t(1) << 31) - 8) return hipErrorInvalidValue;
    if (nblk) *nblk = gx * gy;
    B.rev = traversal_reverse();
    static const bool nt_p0 = env_int("NKHIP_NT_P0", 1) != 0;
    B.nt_p0 = nt_p0;
    const dim3 grid{unsigned((gx * gy + 7) / 8 * 8), 1u, 1u};
    if (pf == 2)
      hipLaunchKernelGGL((march_kernel<M, BX, 2>), grid, dim3(BX), 0, s, B, RY, int(gx), int(gy));
    else
      hipLaunchKernelGGL((march_kernel<M, BX, 1>), grid, dim3(BX), 0, s, B, RY, int(gx), int(gy));
  } else {
    if (A.E0 || A.E2 || A.Ea || A.Eb || A.PS0[0] || A.PS2[0])
      return hipErrorInvalidValue;  // march path only
    const int64_t n = A.nx * A.ny;
    const int64_t g = (n + 255) / 256;
    if (nblk) *nblk = g;
    hipLaunchKernelGGL((point_kernel<M>), dim3(unsigned(g)), dim3(256), 0, s, A);
  }
  return hipGetLastError();
}

}  // namespace

hipError_t stencil_launch(SMode m, const StencilArgs& a, hipStream_t s, int64_t* nblk) {
  if (a.nx <= 0 || a.ny <= 0) return hipSuccess;
  switch (m) {
    case SMode::LAP5: return launch_mode<SMode::LAP5>(a, s, nblk);
    case SMode::SH13: return launch_mode<SMode::SH13>(a, s, nblk);
    case SMode::RESID: return launch_mode<SMode::RESID>(a, s, nblk);
    case SMode::BOLD: return launch_mode<SMode::BOLD>(a, s, nblk);
    case SMode::TRIAL: return launch_mode<SMode::TRIAL>(a, s, nblk);
    case SMode::FDJVP: return launch_mode<SMode::FDJVP>(a, s, nblk);
    case SMode::AJVP: return launch_mode<SMode::AJVP>(a, s, nblk);
    case SMode::LINOP: return launch_mode<SMode::LINOP>(a, s, nblk);
  }
  return hipErrorInvalidValue;
}

int64_t stencil_partial_slots(int64_t ny, int64_t nx) {
  const int64_t march = ((nx / 2 + 127) / 128) * ((ny + 3) / 4);  // RY >= 4 (a ring), BX = 128
  const int64_t point = (nx * ny + 255) / 256;
  return 3 * (march > point ? march : point) + 3;
}

double stencil_bytes_per_point(SMode m, bool has_xt) {
  switch (m) {
    case SMode::LAP5: return 16.0;   // read v, write y
    case SMode::SH13: return 16.0;
    case SMode::RESID: return 24.0;  // read u, uo, write F
    case SMode::BOLD: return 16.0;
    case SMode::TRIAL: return has_xt ? 48.0 : 40.0;  // read x, d, B; write F, G (, xt)
    case SMode::FDJVP: return 32.0;  // read x0, z, G0; write Jz
    case SMode::AJVP: return 24.0;   // read u, z; write Jz
    case SMode::LINOP: return 40.0;  // read r, p, d; write p', A p
  }
  return 0.0;
}

}  // namespace nk

// Droplet (python_work/droplet.py) device kernels -- see droplet.h.
//
// Each launch is ONE workgroup of 1024 threads walking the 5551-point grid stage by stage
// (workgroup barriers between stages; intermediate fields in L2-resident scratch).  Formulas and
// their association order follow the reference line by line (cited per function); derivative
// matrices of make_M (droplet.py:778-833) are applied matrix-free with their exact coefficients
// (integer weights divided by 12*h or 12*h^2, as the reference builds them).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "droplet.h"
#include "nk_device.h"
#include "nk_kernels.h"

namespace nk {
namespace {

constexpr int DB = 1024;
constexpr size_t kPmaLdsMax = 156 * 1024;  // dynamic LDS cap (160 KB per CU minus static use)

int env_flag(const char* name) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::atoi(v) : 0;
}

// The four 1-D derivative operators (kron factors of make_M, droplet.py:778-833): 0 = D1 along
// xi, 1 = D1 along eta (dksiCentre / detaCentre, :795-806), 2 / 3 = D2 along xi / eta (d2ksi /
// d2eta, :782-793).  Entries are the reference's weights divided by s = 12h (D1) or 12h^2 (D2).
// The 5-point interior weights travel as a small kernel argument (SGPR-resident); the two
// boundary rows at each end live in a per-launch LDS table built by coef_rows_init, so a kernel
// never holds the ~100 boundary weights in scalar registers.
struct Coefs {
  double in[4][5];
  double s[4];
};
constexpr int kCoefRows = 4 * 4 * 6;
__shared__ double g_rows[kCoefRows];  // [op][row 0, 1, n-2, n-1][6], filled per launch

// Boundary-row weights before division (row lengths 5, 5, 5, 5 for D1 and 5, 6, 6, 5 for D2;
// rows n-2 / n-1 end at column n-1).
__constant__ double kRowW[2][4][6] = {
    {{-25, 48, -36, 16, -3, 0}, {-3, -10, 18, -6, 1, 0}, {-1, 6, -18, 10, 3, 0},
     {3, -16, 36, -48, 25, 0}},
    {{-415.0 / 6, 96, -36, 32.0 / 3, -1.5, 0}, {10, -15, -4, 14, -6, 1}, {1, -6, 14, -4, -15, 10},
     {-1.5, 32.0 / 3, -36, 96, -415.0 / 6, 0}}};

__device__ __forceinline__ void coef_rows_init(const Coefs& C) {
  for (int t = threadIdx.x; t < kCoefRows; t += DB) {
    const int op = t / 24, row = (t / 6) % 4, k = t % 6;
    const double sc = op == 0 ? C.s[0] : op == 1 ? C.s[1] : op == 2 ? C.s[2] : C.s[3];
    g_rows[t] = kRowW[op >= 2][row][k] / sc;  // selects: no dynamic index into the argument
  }
  __syncthreads();
}

// Apply operator OP at position `pos` of an axis of length n; element k of the axis is
// v[k*stride].  Summation runs over the row's columns in increasing order (CSR row order).
template <int OP, bool kIn = false>
__device__ __forceinline__ double op1(const Coefs& C, const double* v, int pos, int n, int stride) {
  constexpr bool kD2 = OP >= 2;
  const double* in = C.in[OP];
  double acc;
  if (kIn || (pos >= 2 && pos <= n - 3)) {
    acc = in[0] * v[(pos - 2) * stride] + in[1] * v[(pos - 1) * stride];
    if (kD2) acc += in[2] * v[pos * stride];  // the D1 centre weight is zero
    acc += in[3] * v[(pos + 1) * stride] + in[4] * v[(pos + 2) * stride];
    return acc;
  }
  const double* r = g_rows + OP * 24;
  constexpr int L1 = kD2 ? 6 : 5;
  acc = 0.0;
  if (pos == 0) {
#pragma nounroll
    for (int k = 0; k < 5; ++k) acc += r[k] * v[k * stride];
  } else if (pos == 1) {
#pragma nounroll
    for (int k = 0; k < L1; ++k) acc += r[6 + k] * v[k * stride];
  } else if (pos == n - 2) {
#pragma nounroll
    for (int k = 0; k < L1; ++k) acc += r[12 + k] * v[(n - L1 + k) * stride];
  } else {
#pragma nounroll
    for (int k = 0; k < 5; ++k) acc += r[18 + k] * v[(n - 5 + k) * stride];
  }
  return acc;
}

// Derivatives of a field stored row-major with row stride `ld` (nx for global fields, the padded
// LDS stride for staged ones).
template <bool kIn = false>
__device__ __forceinline__ double dx1(const Coefs& C, const double* v, int i, int j, int nx,
                                      int ld) {
  return op1<0, kIn>(C, v + i * ld, j, nx, 1);
}
template <bool kIn = false>
__device__ __forceinline__ double dy1(const Coefs& C, const double* v, int i, int j, int ny,
                                      int ld) {
  return op1<1, kIn>(C, v + j, i, ny, ld);
}

// M.dksideta = kron(D1y, D1x) (:806): sum over the row operator of the column-derivatives.
template <bool kIn = false>
__device__ __forceinline__ double dxy(const Coefs& C, const double* v, int i, int j, int nx,
                                      int ny, int ld) {
  double acc = 0.0;
  if (kIn || (i >= 2 && i <= ny - 3)) {
    const double* in = C.in[1];
    acc += in[0] * dx1<kIn>(C, v, i - 2, j, nx, ld);  // row order, zero centre weight skipped
    acc += in[1] * dx1<kIn>(C, v, i - 1, j, nx, ld);
    acc += in[3] * dx1<kIn>(C, v, i + 1, j, nx, ld);
    acc += in[4] * dx1<kIn>(C, v, i + 2, j, nx, ld);
    return acc;
  }
  const double* r = g_rows + 24;
  int start = 0;
  if (i == 1) r += 6;
  if (i == ny - 2) { r += 12; start = ny - 5; }
  if (i == ny - 1) { r += 18; start = ny - 5; }
#pragma nounroll
  for (int k = 0; k < 5; ++k) acc += r[k] * dx1<kIn>(C, v, start + k, j, nx, ld);
  return acc;
}

// The explicit part of Laplace_operator along one axis (:616-668): v_xx (axis = x, A = A11) or
// v_yy (axis = y, A = A22) at position `pos` of a line of length n, element k at v[k*stride].
template <bool kIn = false>
__device__ __forceinline__ double lap_axis(const double* v, int sv, const double* A, int sa,
                                           int pos, int n, double h2) {
  auto V = [&](int k) { return v[k * sv]; };
  auto a = [&](int k) { return A[k * sa]; };
  const int m = pos;
  if (kIn || (m >= 3 && m <= n - 4)) {  // interior (:617-631)
    return (4 * (a(m - 1) * (V(m - 3) - 8 * V(m - 2) + 8 * V(m) - V(m + 1)))
            - ((-a(m - 2) + 9 * a(m - 1) + 9 * a(m) - a(m + 1)) *
               (V(m - 2) - 27 * V(m - 1) + 27 * V(m) - V(m + 1)))
            + ((-a(m - 1) + 9 * a(m) + 9 * a(m + 1) - a(m + 2)) *
               (V(m - 1) - 27 * V(m) + 27 * V(m + 1) - V(m + 2)))
            - 4 * (a(m + 1) * (V(m - 1) - 8 * V(m) + 8 * V(m + 2) - V(m + 3)))) / (288 * h2);
  }
  if (m == 1) {  // next-to boundary (:635-637)
    return (a(1) * (10 * V(0) - 15 * V(1) - 4 * V(2) + 14 * V(3) - 6 * V(4) + V(5))) / (12 * h2)
           + ((-3 * V(0) - 10 * V(1) + 18 * V(2) - 6 * V(3) + V(4)) *
              (-3 * a(0) - 10 * a(1) + 18 * a(2) - 6 * a(3) + a(4))) / (144 * h2);
  }
  if (m == n - 2) {  // (:643-645)
    const int e = n - 1;
    return (a(e - 1) * (10 * V(e) - 15 * V(e - 1) - 4 * V(e - 2) + 14 * V(e - 3) - 6 * V(e - 4) +
                        V(e - 5))) / (12 * h2)
           + ((3 * V(e) + 10 * V(e - 1) - 18 * V(e - 2) + 6 * V(e - 3) - V(e - 4)) *
              (3 * a(e) + 10 * a(e - 1) - 18 * a(e - 2) + 6 * a(e - 3) - a(e - 4))) / (144 * h2);
  }
  if (m == 2) {  // next-to-next-to boundary (:653-655)
    return (a(2) * (-V(0) + 16 * V(1) - 30 * V(2) + 16 * V(3) - V(4))) / (12 * h2)
           + ((V(0) - 8 * V(1) + 8 * V(3) - V(4)) * (a(0) - 8 * a(1) + 8 * a(3) - a(4))) /
                 (144 * h2);
  }
  if (m == n - 3) {  // (:661-663)
    const int e = n - 1;
    return (a(e - 2) * (-V(e) + 16 * V(e - 1) - 30 * V(e - 2) + 16 * V(e - 3) - V(e - 4))) /
               (12 * h2)
           + ((V(e - 4) - 8 * V(e - 3) + 8 * V(e - 1) - V(e)) *
              (a(e - 4) - 8 * a(e - 3) + 8 * a(e - 1) - a(e))) / (144 * h2);
  }
  return 0.0;  // the boundary line itself stays zero before the cross term (:615)
}

// x^n for the small integer exponents of the models (n >= 0) by repeated multiplication.  The
// reference's NumPy `**` calls libm pow (correctly rounded); this differs from it by a few ulp,
// where the device pow (an extended-precision log / exp, ~100 instructions) took ~5 us of
// single-workgroup time per call site and launch.
__device__ __forceinline__ double ipow(double x, int n) {
  double r = 1.0;
  for (int k = 0; k < n; ++k) r *= x;
  return r;
}

__device__ __forceinline__ double PI(const DropParams& P, double h) {
  // disjoining pressure (:462-467)
  const double r = P.epsilon / h;
  return (P.n_exp - 1) * (P.m_exp - 1) * (ipow(r, P.m_exp) - ipow(r, P.n_exp)) /
         (2 * P.epsilon * (P.n_exp - P.m_exp));
}

__device__ __forceinline__ double pressure(const DropParams& P, double h, double hxx, double hyy) {
  return -(hxx + hyy) + PI(P, h) + P.Bo * cos(P.alpha2) * h;  // (:469-473)
}

// Visit every grid point once: the deep interior (3 <= i <= ny-4, 3 <= j <= nx-4, where every
// operator takes its 5-point interior form) first, branch-free (kIn = true), then the 3-wide
// boundary ring with the general per-position code.  Only the one wave straddling the split
// diverges; a row-major walk would put boundary columns in nearly every wave.
// Division by a run-time divisor d as one multiply-high: q = umulhi(t, ceil(2^32/d)), exact
// while t*d < 2^32 (shape_ok bounds the grid so).
struct FastDiv {
  uint32_t m;
  __device__ explicit FastDiv(uint32_t d) : m(0xFFFFFFFFu / d + 1u) {}
  __device__ int operator()(int t) const { return int(__umulhi(uint32_t(t), m)); }
};

// point u of the boundary ring: rows 0-2 and ny-3..ny-1, then columns 0-2 and nx-3..nx-1 of
// rows 3..ny-4
__device__ __forceinline__ void ring_point(int u, int nx, int ny, const FastDiv& diy,
                                           const FastDiv& dnx, int* i, int* j) {
  if (u < 6 * nx) {
    const int r = dnx(u);
    *i = r < 3 ? r : ny - 6 + r;
    *j = u - r * nx;
  } else {
    u -= 6 * nx;
    const int c = diy(u);
    *j = c < 3 ? c : nx - 6 + c;
    *i = 3 + (u - c * (ny - 6));
  }
}

template <class F>
__device__ __forceinline__ void for_points(int nx, int ny, F f) {
  const int ix = nx - 6, iy = ny - 6, nI = ix * iy, NN = nx * ny;
  const FastDiv dix(ix), diy(iy), dnx(nx);
  for (int t = threadIdx.x; t < NN; t += DB) {
    if (t < nI) {
      const int q = dix(t);
      const int i = 3 + q, j = 3 + (t - q * ix);
      f(i * nx + j, i, j, std::true_type{});
    } else {
      int i, j;
      ring_point(t - nI, nx, ny, diy, dnx, &i, &j);
      f(i * nx + j, i, j, std::false_type{});
    }
  }
}
#define FOR_POINTS(NN) \
  for_points(nx, ny, [&](const int p_, const int i_, const int j_, auto kin_)

// The stencil stages visit the interior in column strips instead: a thread takes one column j
// and kS consecutive rows i0 .. i0+kS-1 (one pass over the droplet's 85 x 55 interior with 935
// threads), loads the neighbours its points share once into registers -- the strip's window --
// and computes every point from them with the same operators in the same summation order as the
// point walk (a register array indexed by constants is what op1 / lap_axis read then).  All of a
// strip's loads precede its stores, so they issue together; then the boundary ring point-wise.
constexpr int kS = 5;

template <class F>
__device__ __forceinline__ void for_strips(int nx, int ny, F f) {
  const int ix = nx - 6, iy = ny - 6, ns = (iy + kS - 1) / kS;
  const FastDiv dix(ix);
  for (int t = threadIdx.x; t < ns * ix; t += DB) {
    const int s = dix(t);
    f(3 + kS * s, 3 + (t - s * ix), min(kS, iy - kS * s));  // (i0, j, rows of this strip)
  }
}

template <class F>
__device__ __forceinline__ void for_ring(int nx, int ny, F f) {
  const int nR = nx * ny - (nx - 6) * (ny - 6);
  const FastDiv diy(ny - 6), dnx(nx);
  for (int u = threadIdx.x; u < nR; u += DB) {
    int i, j;
    ring_point(u, nx, ny, diy, dnx, &i, &j);
    f(i * nx + j, i, j);
  }
}

// W[r][c] = v(i0 - R + r, j - CW + c): rows clamped to the grid (a short last strip computes
// rows it does not store); entries a stage never reads are dead loads the compiler drops
template <int R, int CW, int NR = kS + 2 * R>
__device__ __forceinline__ void load_window(double (&W)[NR][2 * CW + 1], const double* v, int ld,
                                            int i0, int j, int ny) {
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int row = min(i0 - R + r, ny - 1);
#pragma unroll
    for (int c = 0; c <= 2 * CW; ++c) W[r][c] = v[row * ld + j - CW + c];
  }
}

// ---------------------------------------------------------------------------- kernels
// compute_Q_spatial_ders (:696-711), J (:376) and the Laplace metric (:612-614) at grid point
// (i, j), reading q at (iq, jq) of a field with row stride ldq: the grid plane itself (iq, jq =
// i, j) or, in the interior (kIn), a strip's register window
struct MeshPt {
  double qd, qe, q2x, q2y, qxy, J, A11, A22, A12;
};
template <bool kIn>
__device__ __forceinline__ MeshPt mesh_point(const DropParams& P, const Coefs& C, const double* q,
                                             int ldq, int iq, int jq, int i, int j) {
  const int nx = P.nx, ny = P.ny;
  const bool left = !kIn && j == 0, right = !kIn && j == nx - 1;
  const bool bottom = !kIn && i == 0, top = !kIn && i == ny - 1;
  MeshPt m;
  m.qd = dx1<kIn>(C, q, iq, jq, nx, ldq);
  m.qe = dy1<kIn>(C, q, iq, jq, ny, ldq);
  if (left) m.qd = P.endl;
  if (right) m.qd = P.endr;
  if (bottom) m.qe = P.endb;
  if (top) m.qe = P.endt;
  double t = 0.0;
  if (left) t = 25 / (6 * P.dksi) * fabs(P.endl);
  if (right) t = 25 / (6 * P.dksi) * fabs(P.endr);
  m.q2x = op1<2, kIn>(C, q + iq * ldq, jq, nx, 1) + t;
  t = 0.0;
  if (top) t = 25 / (6 * P.deta) * fabs(P.endt);
  if (bottom) t = 25 / (6 * P.deta) * fabs(P.endb);
  m.q2y = op1<3, kIn>(C, q + jq, iq, ny, ldq) + t;
  m.qxy = (left || right || top || bottom) ? 0.0 : dxy<kIn>(C, q, iq, jq, nx, ny, ldq);
  m.J = m.q2x * m.q2y - m.qxy * m.qxy;
  m.A11 = (m.qxy * m.qxy + m.q2y * m.q2y) / m.J;
  m.A22 = (m.qxy * m.qxy + m.q2x * m.q2x) / m.J;
  m.A12 = -(m.qxy * (m.q2x + m.q2y)) / m.J;
  return m;
}

// all == false: only the fields the PMA iteration itself reads next (J, A12; A11 / A22 go to the
// LDS planes) -- the loop's last iteration writes the full set the caller reads afterwards
__device__ void mesh_stage(const DropParams& P, const Coefs& C, const double* q, int ldq,
                           const DropMesh& M, double* a11 = nullptr, double* a22 = nullptr,
                           bool all = true) {
  const int nx = P.nx, ny = P.ny;
  auto put = [&](int p, int i, int j, const MeshPt& m) {
    if (all) {
      M.dksi[p] = m.qd;
      M.deta[p] = m.qe;
      M.d2ksi[p] = m.q2x;
      M.d2eta[p] = m.q2y;
      M.dksideta[p] = m.qxy;
    }
    M.J[p] = m.J;
    if (all) {
      M.A11[p] = m.A11;
      M.A22[p] = m.A22;
    }
    if (a11) {
      a11[i * ldq + j] = m.A11;
      a22[i * ldq + j] = m.A22;
    }
    M.A12[p] = m.A12;
  };
  for_strips(nx, ny, [&](int i0, int j, int nr) {  // the 5 x 5 neighbourhood of each point
    double W[kS + 4][5];
    load_window<2, 2>(W, q, ldq, i0, j, ny);
#pragma unroll
    for (int s = 0; s < kS; ++s)
      if (s < nr) put((i0 + s) * nx + j, i0 + s, j, mesh_point<true>(P, C, &W[0][0], 5, s + 2, 2, 0, 0));
  });
  for_ring(nx, ny, [&](int p, int i, int j) { put(p, i, j, mesh_point<false>(P, C, q, ldq, i, j, i, j)); });
}

__global__ void __launch_bounds__(DB) drop_mesh_kernel(DropParams P, Coefs Ck, const double* q,
                                                       DropMesh M) {
  const Coefs& C = Ck;
  coef_rows_init(C);
  mesh_stage(P, C, q, P.nx, M);
}

// A row-major field with row stride ld: global fields use nx, LDS planes nx|1.
struct Plane {
  double* v;
  int ld;
  __device__ double& operator()(int i, int j) const { return v[i * ld + j]; }
};
struct CPlane {
  const double* v;
  int ld;
  __device__ CPlane(const double* v_, int ld_) : v(v_), ld(ld_) {}
  __device__ CPlane(const Plane& p) : v(p.v), ld(p.ld) {}
  __device__ double operator()(int i, int j) const { return v[i * ld + j]; }
};

template <bool kIn>
__device__ __forceinline__ double dx1(const Coefs& C, CPlane f, int i, int j, int nx) {
  return dx1<kIn>(C, f.v, i, j, nx, f.ld);
}
template <bool kIn>
__device__ __forceinline__ double dy1(const Coefs& C, CPlane f, int i, int j, int ny) {
  return dy1<kIn>(C, f.v, i, j, ny, f.ld);
}

// compute_u_spatial_ders (:713-727) first half: u_xi, u_eta with its boundary rules, incl. the
// U_dksi[Bottom] quirk (:722), as the cross-term inputs t1 = A12 u_eta, t2 = A12 u_xi.
// kRaw: residual() feeds the raw derivatives to Laplace_operator instead (:437, no rules).
template <bool kRaw = false>
__device__ void uders_stage(const DropParams& P, const Coefs& C, const DropMesh& M, CPlane u,
                            Plane t1, Plane t2) {
  const int nx = P.nx, ny = P.ny;
  for_strips(nx, ny, [&](int i0, int j, int nr) {  // interior: no boundary rules
    double W[kS + 4][5];  // (the cross of each point's 5 x 5 neighbourhood is read)
    load_window<2, 2>(W, u.v, u.ld, i0, j, ny);
    double ud[kS], ue[kS], a[kS];
#pragma unroll
    for (int s = 0; s < kS; ++s) {
      ud[s] = dx1<true>(C, &W[0][0], s + 2, 2, nx, 5);
      ue[s] = dy1<true>(C, &W[0][0], s + 2, 2, ny, 5);
      a[s] = M.A12[min(i0 + s, ny - 1) * nx + j];
    }
#pragma unroll
    for (int s = 0; s < kS; ++s) {
      if (s < nr) {
        t1(i0 + s, j) = a[s] * ue[s];
        t2(i0 + s, j) = a[s] * ud[s];
      }
    }
  });
  for_ring(nx, ny, [&](const int p, const int i, const int j) {
    double ud = dx1<false>(C, u, i, j, nx), ue = dy1<false>(C, u, i, j, ny);
    if (!kRaw) {
      if (j == 0 || j == nx - 1) ud = 0.0;
      if (i == ny - 1) ue = 0.0;
      if (i == 0) ud = 0.0;
    }
    t1(i, j) = M.A12[p] * ue;
    t2(i, j) = M.A12[p] * ud;
  });
}

// Laplace_operator (:601-681) at every point: f(p, i, j, u_xx, u_yy) with
//   u_xx = J^-1 [(A11 u_xi)_xi explicit stencil + (A12 u_eta)_xi], u_yy likewise,
// given the cross-term inputs t1 = A12 u_eta, t2 = A12 u_xi.
template <class F>
__device__ void lap_stage(const DropParams& P, const Coefs& C, const DropMesh& M, CPlane u,
                          CPlane a11, CPlane a22, CPlane t1, CPlane t2, F f) {
  const int nx = P.nx, ny = P.ny;
  for_points(nx, ny, [&](const int p, const int i, const int j, auto kin) {
    constexpr bool kIn = decltype(kin)::value;
    const double vxx = lap_axis<kIn>(u.v + i * u.ld, 1, a11.v + i * a11.ld, 1, j, nx,
                                     P.dksi * P.dksi);
    const double vyy = lap_axis<kIn>(u.v + j, u.ld, a22.v + j, a22.ld, i, ny, P.deta * P.deta);
    double tx = dx1<kIn>(C, t1, i, j, nx);
    if (j == 0 || j == nx - 1) tx = 0.0;
    double ty = dy1<kIn>(C, t2, i, j, ny);
    if (i == 0 || i == ny - 1) ty = 0.0;
    f(p, i, j, (vxx + tx) / M.J[p], (vyy + ty) / M.J[p]);
  });
}

// The shared tail of the residual / pde_rhs chains, given u (point values):
//   stage L: v_xx, v_yy (explicit + cross terms t1 = A12 u_eta, t2 = A12 u_xi) -> u_xx, u_yy, p
//   stage P: p derivatives with dp/dn = 0 -> p_x, p_y -> A, B
//   stage F: F2 = J^-1 [d2eta A_xi - dksideta A_eta - dksideta B_xi + d2ksi B_eta]
// Stage L writes the pressure to `pout`, or with `mon` set (the PMA loop) the raw monitor
// |u_xx + u_yy|^2 (:737) instead; u_xx / u_yy go to the optional point arrays uxx / uyy.
__device__ void lap_pressure_stage(const DropParams& P, const Coefs& C, const DropMesh& M,
                                   CPlane u, CPlane a11, CPlane a22, CPlane t1, CPlane t2,
                                   double* uxx, double* uyy, double* mon, Plane pout) {
  lap_stage(P, C, M, u, a11, a22, t1, t2,
            [&](const int p, const int i, const int j, const double hxx, const double hyy) {
              if (uxx) uxx[p] = hxx;
              if (uyy) uyy[p] = hyy;
              if (mon) {
                const double s = fabs(hxx + hyy);
                mon[p] = s * s;
              } else {
                pout(i, j) = pressure(P, u(i, j), hxx, hyy);
              }
            });
}

// compute_P_spatial_ders (:683-694) and the pde_rhs fluxes A, B (:452-457)
__device__ void flux_AB_stage(const DropParams& P, const Coefs& C, const DropMesh& M, CPlane pr,
                              CPlane u, Plane A, Plane B) {
  // (point-wise: in column strips this stage and the flux divergence spill registers in the
  // residual kernel, 44 -> 56 us per launch)
  const int nx = P.nx, ny = P.ny;
  const double slope = P.Bo * sin(P.alpha2) / P.epsilon2;  // (uniform: once per launch)
  for_points(nx, ny, [&](const int p, const int i, const int j, auto kin) {
    constexpr bool kIn = decltype(kin)::value;
    double pd = dx1<kIn>(C, pr, i, j, nx), pe = dy1<kIn>(C, pr, i, j, ny);
    if (j == 0 || j == nx - 1) pd = 0.0;
    if (i == 0 || i == ny - 1) pe = 0.0;
    const double pdx = (M.d2eta[p] * pd - M.dksideta[p] * pe) / M.J[p];
    const double pdy = (-M.dksideta[p] * pd + M.d2ksi[p] * pe) / M.J[p];
    const double h3 = ipow(u(i, j), 3);
    A(i, j) = (pdx - slope) * h3 / 3;
    B(i, j) = pdy * h3 / 3;
  });
}

template <bool kIn>
__device__ __forceinline__ double flux_div_point(const Coefs& C, const DropMesh& M, CPlane A,
                                                 CPlane B, int p, int i, int j, int nx, int ny) {
  return (M.d2eta[p] * dx1<kIn>(C, A, i, j, nx) - M.dksideta[p] * dy1<kIn>(C, A, i, j, ny)
          - M.dksideta[p] * dx1<kIn>(C, B, i, j, nx) + M.d2ksi[p] * dy1<kIn>(C, B, i, j, ny)) /
         M.J[p];
}

__global__ void __launch_bounds__(DB) drop_rhs_kernel(DropParams P, Coefs Ck, DropMesh M,
                                                      DropScratch S, const double* u,
                                                      double* uxx, double* uyy, double* F) {
  const Coefs& C = Ck;
  coef_rows_init(C);
  const int nx = P.nx, ny = P.ny;
  const Plane t1{S.t1, nx}, t2{S.t2, nx}, pr{S.p, nx}, A{S.A, nx}, B{S.B, nx};
  const CPlane uu(u, nx);
  uders_stage(P, C, M, uu, t1, t2);
  __syncthreads();
  // P.val = pressure(U.val, U.xx, U.yy) (:378)
  lap_pressure_stage(P, C, M, uu, CPlane(M.A11, nx), CPlane(M.A22, nx), t1, t2, uxx, uyy,
                     nullptr, pr);
  __syncthreads();
  flux_AB_stage(P, C, M, pr, uu, A, B);
  __syncthreads();
  for_points(nx, ny, [&](const int p, const int i, const int j, auto kin) {
    F[p] = flux_div_point<decltype(kin)::value>(C, M, A, B, p, i, j, nx, ny);
  });
}

// residual(U, F, dt) (:435-450) and its forward-difference JVP, one launch per evaluation.
// kLds: w stays in LDS plane L0 for the whole chain and every neighbour-read input (t1/t2, p,
// A/B) is staged in planes L1/L2; otherwise all intermediates live in global scratch.
template <bool kLds>
__global__ void __launch_bounds__(DB) drop_resid_kernel(DropParams P, Coefs Ck, DropMesh M,
                                                        DropScratch S, const double* x,
                                                        const double* y, double alpha,
                                                        const double* uval, const double* F,
                                                        double dt, int mode, const double* f0,
                                                        double sc, double* out, double* xt,
                                                        double* partial, const double* znorm2,
                                                        double omega, const double* prm) {
  const Coefs& C = Ck;
  if (prm) {  // device-side Arnoldi control: the step's parameters (a handed-back step: nothing)
    if (prm[kArnMaxNV + 3] != 0.0) return;
    alpha = prm[kArnMaxNV + 1];
    sc = prm[kArnMaxNV + 2];
  }
  if (znorm2) {  // the FD step from the device value |z|^2 (KrylovJacobian.matvec, _nonlin.py:
                 // 1505-1509, with v = z/|z|): the host's sc = omega/|v|, alpha = sc/|z|
    const double hn = sqrt(*znorm2);
    double sig = 1.0 / hn;
    if (!isfinite(sig)) sig = 1.0;
    sc = omega / (sig * hn);
    alpha = sc * sig;
  }
  coef_rows_init(C);
  const int nx = P.nx, ny = P.ny, ld = kLds ? (nx | 1) : nx;
  extern __shared__ double lds[];
  const Plane W = kLds ? Plane{lds, ld} : Plane{S.w, nx};
  const Plane L1 = kLds ? Plane{lds + ny * ld, ld} : Plane{S.t1, nx};
  const Plane L2 = kLds ? Plane{lds + 2 * ny * ld, ld} : Plane{S.t2, nx};
  const Plane gp{S.p, nx}, gB{S.B, nx};
  for_points(nx, ny, [&](const int p, const int i, const int j, auto) {
    double w = x[p];
    if (y) w = w + alpha * y[p];
    W(i, j) = w;
  });
  __syncthreads();
  uders_stage<true>(P, C, M, W, L1, L2);  // t1 -> L1, t2 -> L2
  __syncthreads();
  lap_pressure_stage(P, C, M, W, CPlane(M.A11, nx), CPlane(M.A22, nx), L1, L2, nullptr, nullptr,
                     nullptr, gp);
  __syncthreads();
  Plane pr = gp, A = {S.A, nx}, B = gB;
  if (kLds) {  // p -> L1
    for_points(nx, ny, [&](const int p, const int i, const int j, auto) { L1(i, j) = gp.v[p]; });
    __syncthreads();
    pr = L1;
    A = L2;
  }
  flux_AB_stage(P, C, M, pr, W, A, B);
  __syncthreads();
  if (kLds) {  // B -> L1 (p is dead)
    for_points(nx, ny, [&](const int p, const int i, const int j, auto) { L1(i, j) = gB.v[p]; });
    __syncthreads();
    B = L1;
  }
  double red[3] = {0.0, 0.0, 0.0};
  for_points(nx, ny, [&](const int p, const int i, const int j, auto kin) {
    const double F2 = flux_div_point<decltype(kin)::value>(C, M, A, B, p, i, j, nx, ny);
    const double w = W(i, j);
    const double R = (w - uval[p]) - dt * (F2 + F[p]) / 2;  // (:450)
    if (mode == 0) {
      out[p] = R;
      if (xt) xt[p] = w;
      red[0] += R * R;
      red[1] = nmax(red[1], fabs(R));
      red[2] = nmax(red[2], fabs(w));
    } else {
      out[p] = (R - f0[p]) / sc;
    }
  });
  if (mode == 0) {
    const double v = block_reduce<3, 1, DB>(red);
    if (threadIdx.x < 3) partial[threadIdx.x] = v;
  }
}

// ---------------------------------------------------------------------------- droplet init
// compute_U2 (:413-429) at the node coordinates of the current mesh.
__global__ void __launch_bounds__(256) drop_u2_kernel(DropParams P, DropMesh M, DropSet D,
                                                      double* u) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= P.nx * P.ny) return;
  const double xp = M.dksi[p], yp = M.deta[p];
  double r = P.epsilon;
  for (int d = 0; d < D.n; ++d) {
    const double x = D.v[d][0], y = D.v[d][1], R = D.v[d][2], V = D.v[d][3];
    const double xx = sqrt((xp - x) * (xp - x) + (yp - y) * (yp - y));
    const double psi =
        R + log((1 + exp(-2 * P.a * (xx + R))) / (1 + exp(-2 * P.a * (xx - R)))) / (2 * P.a);
    r += (1 - P.epsilon) * (4 * V * (1 - psi * psi / (R * R)) / (R * R));
  }
  u[p] = r;
}

// ---------------------------------------------------------------------------- PMA2 (MEMS)
// PMA2_nk.py residual() (:121-159) / compute_rhs_pde() (:400-413): the bilaplacian chain
//   u -> (u_xx, u_yy) = Laplace_operator(u) -> v = u_xx + u_yy -> (v_xx, v_yy) = Laplace_operator(v)
// with raw centred derivatives feeding each Laplace_operator (:133, :141).  kLds: w, v and the
// cross-term inputs live in three LDS planes; otherwise in global scratch.
template <bool kLds>
__global__ void __launch_bounds__(DB) mems_resid_kernel(DropParams P, Coefs Ck, MemsParams Mp,
                                                        DropMesh M, DropScratch S, const double* x,
                                                        const double* y, double alpha,
                                                        const double* uval, const double* cn,
                                                        int mode, const double* f0, double sc,
                                                        double* out, double* xt, double* uxx,
                                                        double* uyy, double* partial,
                                                        const double* znorm2, double omega,
                                                        const double* prm) {
  const Coefs& C = Ck;
  if (prm) {  // device-side Arnoldi control (as drop_resid_kernel)
    if (prm[kArnMaxNV + 3] != 0.0) return;
    alpha = prm[kArnMaxNV + 1];
    sc = prm[kArnMaxNV + 2];
  }
  if (znorm2) {  // the FD step from the device value |y|^2 (as drop_resid_kernel)
    const double hn = sqrt(*znorm2);
    double sig = 1.0 / hn;
    if (!isfinite(sig)) sig = 1.0;
    sc = omega / (sig * hn);
    alpha = sc * sig;
  }
  coef_rows_init(C);
  const int nx = P.nx, ny = P.ny, ld = kLds ? (nx | 1) : nx;
  extern __shared__ double lds[];
  const Plane W = kLds ? Plane{lds, ld} : Plane{S.w, nx};
  const Plane L1 = kLds ? Plane{lds + ny * ld, ld} : Plane{S.t1, nx};
  const Plane L2 = kLds ? Plane{lds + 2 * ny * ld, ld} : Plane{S.t2, nx};
  const Plane V = kLds ? W : Plane{S.p, nx};  // v = u_xx + u_yy (LDS: reuses w's plane)
  const CPlane A11(M.A11, nx), A22(M.A22, nx);
  for_points(nx, ny, [&](const int p, const int i, const int j, auto) {
    double w = x[p];
    if (y) w = w + alpha * y[p];
    W(i, j) = w;
    if (kLds) S.w[p] = w;  // read back point-wise once W's plane holds v
  });
  __syncthreads();
  uders_stage<true>(P, C, M, W, L1, L2);
  __syncthreads();
  lap_stage(P, C, M, W, A11, A22, L1, L2,
            [&](const int p, const int, const int, const double hxx, const double hyy) {
              if (mode == 2 && uxx) {
                uxx[p] = hxx;
                uyy[p] = hyy;
              }
              S.p[p] = hxx + hyy;
            });
  __syncthreads();
  if (kLds) {
    for_points(nx, ny, [&](const int p, const int i, const int j, auto) { V(i, j) = S.p[p]; });
    __syncthreads();
  }
  uders_stage<true>(P, C, M, V, L1, L2);
  __syncthreads();
  double red[3] = {0.0, 0.0, 0.0};
  if (mode == 2) red[0] = -INFINITY;
  lap_stage(P, C, M, V, A11, A22, L1, L2,
            [&](const int p, const int i, const int j, const double vxx, const double vyy) {
              const double w = S.w[p];
              const double g = 1 + w;
              double r = -Mp.lambd / (g * g) + Mp.lam_eps / ipow(g, Mp.m);
              r = r - Mp.beta2 * (vxx + vyy);
              if (i == 0 || j == 0 || i == ny - 1 || j == nx - 1) r = 0.0;  // (:157)
              if (mode == 2) {
                out[p] = r;
                red[0] = nmax(red[0], -ipow(g, 3));
                return;
              }
              const double R = (w - uval[p]) / Mp.k - (r + cn[p]) / 2;  // (:159)
              if (mode == 0) {
                out[p] = R;
                if (xt) xt[p] = w;
                red[0] += R * R;
                red[1] = nmax(red[1], fabs(R));
                red[2] = nmax(red[2], fabs(w));
              } else {
                out[p] = (R - f0[p]) / sc;
              }
            });
  if (mode == 0) {
    const double v = block_reduce<3, 1, DB>(red);
    if (threadIdx.x < 3) partial[threadIdx.x] = v;
  } else if (mode == 2) {
    const double v = block_reduce<3, 0, DB>(red);  // all-max; only red[0] is meaningful
    if (threadIdx.x == 0) partial[0] = v;
  }
}

// ---------------------------------------------------------------------------- PMA mesh loop
// loop_pma (:589-599), solve_PMA (:578-587), compute_and_smooth_monitor (:729-760) as ONE
// persistent single-workgroup kernel running all `loops` iterations on the GPU.  The orthonormal
// DCT-II / -III (scipy.fft dct / idct, norm="ortho") are dense products with precomputed DCT
// matrices (91x91 and 61x61 at the reference size).

// One pass of the 9-point monitor filter (:740-756), T -> Mo, both with row stride ld.
template <class Tf>
__device__ __forceinline__ double smooth9(Tf t, int i, int j) {
  return t(i, j) + (t(i - 1, j) + t(i + 1, j) + t(i, j - 1) + t(i, j + 1)) / 8 +
         (t(i - 1, j - 1) + t(i - 1, j + 1) + t(i + 1, j - 1) + t(i + 1, j + 1)) / 16;
}
// T has row stride ldt, Mo ldm.  J (optional): also return this thread's share of the Mackenzie
// integral sum(Mo |J|) (:757-759) over the points it wrote.
__device__ double smooth_pass(const DropParams& P, const double* T, int ldt, double* Mo, int ldm,
                              const double* J = nullptr) {
  const int nx = P.nx, ny = P.ny;
  double acc = 0.0;
  for_strips(nx, ny, [&](int i0, int j, int nr) {
    double W[kS + 2][3];
    load_window<1, 1>(W, T, ldt, i0, j, ny);
    double v[kS];
#pragma unroll
    for (int s = 0; s < kS; ++s) v[s] = smooth9([&](int a, int b) { return W[a][b]; }, s + 1, 1);
#pragma unroll
    for (int s = 0; s < kS; ++s) {
      if (s < nr) {
        Mo[(i0 + s) * ldm + j] = v[s];
        if (J) acc += v[s] * fabs(J[(i0 + s) * nx + j]);
      }
    }
  });
  for_ring(nx, ny, [&](const int p, const int i, const int j) {
    auto t = [&](int a, int b) { return T[a * ldt + b]; };
    double v;
    const bool in_i = i > 0 && i < ny - 1, in_j = j > 0 && j < nx - 1;
    if (in_i && in_j) {
      v = smooth9(t, i, j);
    } else if (in_i && j == nx - 1) {
      v = (4 * t(i, j) + 2 * t(i - 1, j) + 2 * t(i + 1, j) + 2 * t(i, j - 1) + t(i + 1, j - 1) +
           t(i - 1, j - 1)) / 12;
    } else if (in_i && j == 0) {
      v = (4 * t(i, 0) + 2 * t(i - 1, 0) + 2 * t(i + 1, 0) + 2 * t(i, 1) + t(i + 1, 1) +
           t(i - 1, 1)) / 12;
    } else if (in_j && i == ny - 1) {
      v = (4 * t(i, j) + 2 * t(i, j - 1) + 2 * t(i, j + 1) + 2 * t(i - 1, j) + t(i - 1, j + 1) +
           t(i - 1, j - 1)) / 12;
    } else if (in_j && i == 0) {
      v = (4 * t(0, j) + 2 * t(0, j - 1) + 2 * t(0, j + 1) + 2 * t(1, j) + t(1, j + 1) +
           t(1, j - 1)) / 12;
    } else if (i == 0 && j == 0) {
      v = (4 * t(0, 0) + 2 * t(0, 1) + 2 * t(1, 0) + t(1, 1)) / 9;
    } else if (i == 0) {  // j == nx-1
      v = (4 * t(0, j) + 2 * t(0, j - 1) + 2 * t(1, j) + t(1, j - 1)) / 9;
    } else if (j == 0) {  // i == ny-1
      v = (4 * t(i, 0) + 2 * t(i, 1) + 2 * t(i - 1, 0) + t(i - 1, 1)) / 9;
    } else {
      v = (4 * t(i, j) + 2 * t(i, j - 1) + 2 * t(i - 1, j) + t(i - 1, j - 1)) / 9;
    }
    Mo[i * ldm + j] = v;
    if (J) acc += v * fabs(J[p]);
  });
  return acc;
}

// Mackenzie regularisation integral sum(mon |J|) dksi deta (:757-759), broadcast to all threads.
__device__ double monitor_integral(const DropParams& P, const DropMesh& M, const double* T, int ld,
                                   double* bcast) {
  const int nx = P.nx, ny = P.ny;
  double part[1] = {0.0};
  FOR_POINTS(NN) { part[0] += T[i_ * ld + j_] * fabs(M.J[p_]); });
  const double tot = block_reduce<1, 1, DB>(part);
  if (threadIdx.x == 0) *bcast = tot * P.dksi * P.deta;
  __syncthreads();
  return *bcast;
}

// Fallback for grids whose working planes do not fit LDS: every field in global (L2) memory.
__global__ void __launch_bounds__(DB) drop_pma_kernel(DropParams P, Coefs Ck, DropMesh M,
                                                      DropScratch S, double* q, const double* uval,
                                                      const double* uxx0, const double* uyy0,
                                                      PmaTables Tb, double dtm, int loops,
                                                      int monitor) {
  const Coefs& C = Ck;
  coef_rows_init(C);
  const int nx = P.nx, ny = P.ny, NN = nx * ny;
  __shared__ double bcast;
  double* uxx = S.A;  // u_xx, u_yy of the current mesh (first iteration: the caller's)
  double* uyy = S.B;
  for (int it = 0; it < loops; ++it) {
    if (monitor == kMonGap) {
      FOR_POINTS(NN) { S.ud[p_] = 1 / ipow(1 + uval[p_], 6); });  // (PMA2_nk.py:357)
      if (it > 0) {
        mesh_stage(P, C, q, nx, M);
      }
    } else if (it > 0) {
      // compute_Q_spatial_ders, J, compute_u_spatial_ders (:595-597)
      mesh_stage(P, C, q, nx, M);
      __syncthreads();
      uders_stage(P, C, M, CPlane(uval, nx), Plane{S.t1, nx}, Plane{S.t2, nx});
      __syncthreads();
      lap_pressure_stage(P, C, M, CPlane(uval, nx), CPlane(M.A11, nx), CPlane(M.A22, nx),
                         CPlane(S.t1, nx), CPlane(S.t2, nx), uxx, uyy, S.ud, Plane{S.p, nx});
    } else {
      FOR_POINTS(NN) {
        const double s = fabs(uxx0[p_] + uyy0[p_]);  // monitor |u_xx + u_yy|^2 (:737)
        S.ud[p_] = s * s;
      });
    }
    __syncthreads();
    double* T = S.ud;
    double* Mo = S.ue;
    for (int sm = 0; sm < P.smoothing_iters; ++sm) {
      smooth_pass(P, T, nx, Mo, nx);
      __syncthreads();
      double* sw = T;
      T = Mo;
      Mo = sw;
    }
    const double integral = monitor_integral(P, M, T, nx, &bcast);
    // q_rhs = sqrt(mon |J|) / alpha (:584)
    double* X = S.p;
    FOR_POINTS(NN) { X[p_] = sqrt((T[p_] + P.C * integral) * fabs(M.J[p_])) / P.alpha; });
    __syncthreads();
    // 2-D DCT-II ortho: T1 = Cy X (along eta), T2 = T1 Cx^T (along xi) (:585)
    double* T1 = S.t1;
    FOR_POINTS(NN) {
    [[maybe_unused]] constexpr bool kIn = decltype(kin_)::value;
      const int k = i_, j = j_;
      double acc = 0.0;
      for (int i = 0; i < ny; ++i) acc += Tb.cy[k * ny + i] * X[i * nx + j];
      T1[p_] = acc;
    });
    __syncthreads();
    double* T2 = S.t2;
    FOR_POINTS(NN) {
    [[maybe_unused]] constexpr bool kIn = decltype(kin_)::value;
      const int k = i_, l = j_;
      double acc = 0.0;
      for (int j = 0; j < nx; ++j) acc += T1[k * nx + j] * Tb.cx[l * nx + j];
      T2[p_] = acc / Tb.den[p_];  // / (1 - gamma Leig) (:586)
    });
    __syncthreads();
    // inverse (DCT-III ortho): Y1 = Cy^T T2, dQ = Y1 Cx (:586-587)
    FOR_POINTS(NN) {
    [[maybe_unused]] constexpr bool kIn = decltype(kin_)::value;
      const int i = i_, l = j_;
      double acc = 0.0;
      for (int k = 0; k < ny; ++k) acc += Tb.cy[k * ny + i] * T2[k * nx + l];
      T1[p_] = acc;
    });
    __syncthreads();
    FOR_POINTS(NN) {
    [[maybe_unused]] constexpr bool kIn = decltype(kin_)::value;
      const int i = i_, j = j_;
      double acc = 0.0;
      for (int l = 0; l < nx; ++l) acc += T1[i * nx + l] * Tb.cx[l * nx + j];
      q[p_] = q[p_] + dtm * acc;  // Q.val += dt * Q.dt (:591, :599)
    });
    __syncthreads();
  }
}

// ---- LDS-resident variant.  Three LDS planes (row stride ld = nx|1, odd so that column walks
// are bank-conflict free) hold the stencil inputs of each stage and the DCT intermediates.  The
// four DCT products run on v_mfma_f64_16x16x4: the constant DCT operand streams from a global
// table already in fragment order (one coalesced 512-B load per wave and k step), the data
// operand comes from the LDS plane; one lane operand pair feeds 256 multiply-adds.
constexpr int kWaves = DB / 64;
typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr int kBatch = 4;  // k steps whose operands load together

// k steps of a K-deep product, padded to a multiple of kBatch (the tables hold zeros there)
__host__ __device__ inline int pma_ksteps(int K) { return ((K + 3) / 4 + kBatch - 1) / kBatch * kBatch; }

__device__ __forceinline__ f64x4 mfma_f64(double a, double b, f64x4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// The DCT products with the transform's first butterfly folded in: DCT-II rows are even or odd
// about the middle (C[k][N-1-n] = (-1)^k C[k][n]), so
//   forward (kInv false): frequency 2h takes s_k = x_k + x_{N-1-k}, frequency 2h+1 takes
//     d_k = x_k - x_{N-1-k}, k < ceil(N/2) (an odd N's middle entry: weight C/2 on s = 2 x_mid);
//   inverse (DCT-III): E_h, O_h sum the even / odd frequencies, h < ceil(N/2), and
//     y_h = E_h + O_h, y_{N-1-h} = E_h - O_h.
// Half the multiply-adds of the dense product.  A wave task is the even and the odd 16 x 16 tile
// of one half-index range: each loaded operand pair feeds both (forward), each E / O pair meets in
// one epilogue (inverse).  f(t, o, value): t the transformed index, o the other one.
// kConstA: transform along rows (A = table [h][k], B(k, o) = plane[k*ld + o], o < No);
// else along columns (A(o, k) = plane[o*ld + k], o < No, B = table [k][h]).
// Padded k steps have zero table entries; plane indices are clamped so they read finite data.
template <bool kConstA, bool kInv, class Fn>
__device__ __forceinline__ void dct_pair(const double* __restrict__ fe,
                                         const double* __restrict__ fo, const double* plane,
                                         int ld, int Nt, int No, Fn f) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
  const int hs = (Nt + 1) >> 1, S = pma_ksteps(hs), Ht = (hs + 15) >> 4, Ot = (No + 15) >> 4;
  for (int task = wave; task < Ht * Ot; task += kWaves) {
    const int th = task / Ot, to = task - th * Ot;
    const int h0 = 16 * th, o0 = 16 * to;
    const double* pe = fe + size_t(th) * S * 64 + lane;
    const double* po = fo + size_t(th) * S * 64 + lane;
    const int oc = min(o0 + r, No - 1);  // this lane's plane line (column or row), clamped
    const double* pl = kConstA ? plane + oc : plane + oc * ld;
    const int ks = kConstA ? ld : 1;
    f64x4 ce = {0.0, 0.0, 0.0, 0.0}, co = {0.0, 0.0, 0.0, 0.0};
    for (int s0 = 0; s0 < S; s0 += kBatch) {  // S is a multiple of kBatch (zero-padded)
      double ve[kBatch], vo[kBatch], xe[kBatch], xo[kBatch];
#pragma unroll
      for (int u = 0; u < kBatch; ++u) {
        const int k = 4 * (s0 + u) + g;
        ve[u] = pe[(s0 + u) * 64];
        vo[u] = po[(s0 + u) * 64];
        if (kInv) {
          xe[u] = pl[min(2 * k, Nt - 1) * ks];
          xo[u] = pl[min(2 * k + 1, Nt - 1) * ks];
        } else {
          const int kc = min(k, hs - 1);
          const double a = pl[kc * ks], b = pl[(Nt - 1 - kc) * ks];
          xe[u] = a + b;
          xo[u] = a - b;
        }
      }
#pragma unroll
      for (int u = 0; u < kBatch; ++u) {
        ce = kConstA ? mfma_f64(ve[u], xe[u], ce) : mfma_f64(xe[u], ve[u], ce);
        co = kConstA ? mfma_f64(vo[u], xo[u], co) : mfma_f64(xo[u], vo[u], co);
      }
    }
    // D layout: row = (lane >> 4) + 4*reg, col = lane & 15 (the half index runs along A's rows
    // when kConstA, along B's columns otherwise)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int h = kConstA ? h0 + g + 4 * v : h0 + r;
      const int o = kConstA ? o0 + r : o0 + g + 4 * v;
      if (h < hs && o < No) {
        if (kInv) {
          f(h, o, ce[v] + co[v]);
          if (Nt - 1 - h > h) f(Nt - 1 - h, o, ce[v] - co[v]);
        } else {
          f(2 * h, o, ce[v]);
          if (2 * h + 1 < Nt) f(2 * h + 1, o, co[v]);
        }
      }
    }
  }
}

__global__ void __launch_bounds__(DB) drop_pma_lds_kernel(
    DropParams P, Coefs Ck, DropMesh M, DropScratch S, double* q, const double* uval,
    const double* uxx0, const double* uyy0, PmaTables Tb, double dtm, int loops, int monitor,
    unsigned long long* tprof) {
  const double* __restrict__ den = Tb.den;
  const Coefs& C = Ck;
  coef_rows_init(C);
  const int nx = P.nx, ny = P.ny, NN = nx * ny, ld = nx | 1;
  __shared__ double bcast;
  extern __shared__ double lds[];
  double* L0 = lds;
  double* L1 = L0 + ny * ld;
  double* L2 = L1 + ny * ld;
  // optional per-stage timing (NKHIP_PMA_TIMING): thread 0 accumulates wall-clock deltas
  unsigned long long tacc[6] = {0, 0, 0, 0, 0, 0}, tlast = 0;
  auto mark = [&](int k) {
    if (tprof && threadIdx.x == 0) {
      const unsigned long long t = wall_clock64();
      if (k >= 0) tacc[k] += t - tlast;
      tlast = t;
    }
  };
  mark(-1);
  // q of iterations > 0 is in L0 already: the previous iteration's last DCT product wrote it there
  for (int it = 0; it < loops; ++it) {
    const double* T = L0;  // the monitor
    if (monitor == kMonGap) {
      if (it > 0) {  // the mesh fields (J) of the updated q
        mesh_stage(P, C, L0, ld, M);
        __syncthreads();
      }
      FOR_POINTS(NN) { L0[i_ * ld + j_] = 1 / ipow(1 + uval[p_], 6); });  // (PMA2_nk.py:357)
    } else if (it > 0) {
      // compute_Q_spatial_ders + J (:595-596) from q in L0; A11 -> L1, A22 -> L2
      mesh_stage(P, C, L0, ld, M, L1, L2, it == loops - 1);
      __syncthreads();
      mark(0);
      // compute_u_spatial_ders (:597) from u staged in L0
      FOR_POINTS(NN) { L0[i_ * ld + j_] = uval[p_]; });
      __syncthreads();
      uders_stage(P, C, M, CPlane(L0, ld), Plane{S.t1, nx}, Plane{S.t2, nx});
      __syncthreads();
      mark(1);
      // (u_xx / u_yy of the iteration's mesh are not read again: only the monitor is kept, in
      // global scratch while the three planes are busy, then in L0; reading it from there in
      // the first smoothing pass instead costs more than the copy: 19.6 against 8.7 us)
      lap_pressure_stage(P, C, M, CPlane(L0, ld), CPlane(L1, ld), CPlane(L2, ld),
                         CPlane(S.t1, nx), CPlane(S.t2, nx), nullptr, nullptr, S.ud,
                         Plane{S.p, nx});
      mark(2);
      __syncthreads();
      FOR_POINTS(NN) { L0[i_ * ld + j_] = S.ud[p_]; });
    } else {
      FOR_POINTS(NN) {
        const double s = fabs(uxx0[p_] + uyy0[p_]);  // monitor |u_xx + u_yy|^2 (:737)
        L0[i_ * ld + j_] = s * s;
      });
    }
    __syncthreads();
    // smoothing passes ping-pong L1 / L0 (an odd count ends in L1, an even one in L0); the last
    // one also sums this thread's share of the Mackenzie integral
    double part[1] = {0.0};
    for (int sm = 0; sm < P.smoothing_iters; ++sm) {
      double* Mo = (sm % 2 == 0) ? L1 : L0;
      part[0] = smooth_pass(P, T, ld, Mo, ld, sm == P.smoothing_iters - 1 ? M.J : nullptr);
      __syncthreads();
      T = Mo;
    }
    mark(3);
    if (P.smoothing_iters == 0) FOR_POINTS(NN) { part[0] += T[i_ * ld + j_] * fabs(M.J[p_]); });
    // Mackenzie regularisation integral sum(mon |J|) dksi deta (:757-759)
    {
      const double tot = block_reduce<1, 1, DB>(part);
      if (threadIdx.x == 0) bcast = tot * P.dksi * P.deta;
      __syncthreads();
    }
    const double integral = bcast;
    // q_rhs = sqrt(mon |J|) / alpha (:584) -> L2
    FOR_POINTS(NN) {
    [[maybe_unused]] constexpr bool kIn = decltype(kin_)::value;
      L2[i_ * ld + j_] = sqrt((T[i_ * ld + j_] + P.C * integral) * fabs(M.J[p_])) / P.alpha;
    });
    __syncthreads();
    mark(4);
    // DCT-II along eta: T1 = Cy X (L2 -> L0)
    dct_pair<true, false>(Tb.f[0][0], Tb.f[0][1], L2, ld, ny, nx,
                          [&](int t, int o, double v) { L0[t * ld + o] = v; });
    __syncthreads();
    // along xi: T2 = T1 Cx^T, / (1 - gamma Leig) (:585-586) (L0 -> L1)
    dct_pair<false, false>(Tb.f[1][0], Tb.f[1][1], L0, ld, nx, ny,
                           [&](int t, int o, double v) { L1[o * ld + t] = v / den[o * nx + t]; });
    __syncthreads();
    // inverse (DCT-III ortho) along eta: Y1 = Cy^T T2 (L1 -> L2)
    dct_pair<true, true>(Tb.f[2][0], Tb.f[2][1], L1, ld, ny, nx,
                         [&](int t, int o, double v) { L2[t * ld + o] = v; });
    __syncthreads();
    // along xi: dQ = Y1 Cx; Q.val += dt * Q.dt (:587, :591, :599)
    // (the new q also into L0, where the next iteration's mesh stage reads it)
    dct_pair<false, true>(Tb.f[3][0], Tb.f[3][1], L2, ld, nx, ny, [&](int t, int o, double v) {
      const double qn = q[o * nx + t] + dtm * v;
      q[o * nx + t] = qn;
      L0[o * ld + t] = qn;
    });
    __syncthreads();
    mark(5);
  }
  if (tprof && threadIdx.x == 0)
    for (int k = 0; k < 6; ++k) tprof[k] = tacc[k];
}


Coefs make_coefs(const DropParams& P) {
  // make_M's weights (:782-806): interior rows {1,-8,0,8,-1}/12h and {-1,16,-30,16,-1}/12h^2
  Coefs C{};
  const double d1[5] = {1, -8, 0, 8, -1}, d2[5] = {-1, 16, -30, 16, -1};
  C.s[0] = 12 * P.dksi;
  C.s[1] = 12 * P.deta;
  C.s[2] = 12 * (P.dksi * P.dksi);
  C.s[3] = 12 * (P.deta * P.deta);
  for (int k = 0; k < 5; ++k) {
    C.in[0][k] = d1[k] / C.s[0];
    C.in[1][k] = d1[k] / C.s[1];
    C.in[2][k] = d2[k] / C.s[2];
    C.in[3][k] = d2[k] / C.s[3];
  }
  return C;
}

// >= 7 points per side (3-wide boundary ring + interior); FastDiv exact: NN * max(nx, ny) < 2^32
bool shape_ok(const DropParams& P) {
  return P.nx >= 7 && P.ny >= 7 &&
         double(P.nx) * P.ny * (P.nx > P.ny ? P.nx : P.ny) < 4294967295.0;
}

}  // namespace

hipError_t drop_mesh_launch(const DropParams& P, const double* q, DropMesh M, hipStream_t s) {
  if (!shape_ok(P)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(drop_mesh_kernel, dim3(1), dim3(DB), 0, s, P, make_coefs(P), q, M);
  return hipGetLastError();
}

hipError_t drop_rhs_launch(const DropParams& P, const double* uval, DropMesh M, DropScratch S,
                           double* uxx, double* uyy, double* F, hipStream_t s) {
  if (!shape_ok(P)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(drop_rhs_kernel, dim3(1), dim3(DB), 0, s, P, make_coefs(P), M, S, uval, uxx,
                     uyy, F);
  return hipGetLastError();
}

hipError_t drop_resid_launch(const DropParams& P, DropMesh M, DropScratch S, const double* x,
                             const double* y, double alpha, const double* uval, const double* F,
                             double dt, int mode, const double* f0, double sc, double* out,
                             double* xt, double* partial, hipStream_t s, const double* znorm2,
                             double omega, const double* prm) {
  if (!shape_ok(P)) return hipErrorInvalidValue;
  const size_t lds = 3 * size_t(P.ny) * (P.nx | 1) * sizeof(double);
  const bool force_global = env_flag("NKHIP_DROP_GLOBAL") != 0;  // (read per launch: tests flip it)
  if (!force_global && lds <= kPmaLdsMax) {
    static const hipError_t attr = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&drop_resid_kernel<true>),
        hipFuncAttributeMaxDynamicSharedMemorySize, int(kPmaLdsMax));
    if (attr != hipSuccess) return attr;
    hipLaunchKernelGGL(drop_resid_kernel<true>, dim3(1), dim3(DB), lds, s, P, make_coefs(P), M, S,
                       x, y, alpha, uval, F, dt, mode, f0, sc, out, xt, partial, znorm2, omega, prm);
  } else {
    hipLaunchKernelGGL(drop_resid_kernel<false>, dim3(1), dim3(DB), 0, s, P, make_coefs(P), M, S,
                       x, y, alpha, uval, F, dt, mode, f0, sc, out, xt, partial, znorm2, omega, prm);
  }
  return hipGetLastError();
}

hipError_t drop_u2_launch(const DropParams& P, DropMesh M, const DropSet& drops, double* u,
                          hipStream_t s) {
  if (!shape_ok(P) || drops.n < 0 || drops.n > kMaxDrops) return hipErrorInvalidValue;
  const int n = P.nx * P.ny;
  hipLaunchKernelGGL(drop_u2_kernel, dim3((n + 255) / 256), dim3(256), 0, s, P, M, drops, u);
  return hipGetLastError();
}

hipError_t mems_resid_launch(const DropParams& P, const MemsParams& Mp, DropMesh M, DropScratch S,
                             const double* x, const double* y, double alpha, const double* uval,
                             const double* cn, int mode, const double* f0, double sc, double* out,
                             double* xt, double* uxx, double* uyy, double* partial, hipStream_t s,
                             const double* znorm2, double omega, const double* prm) {
  if (!shape_ok(P) || mode < 0 || mode > 2) return hipErrorInvalidValue;
  const size_t lds = 3 * size_t(P.ny) * (P.nx | 1) * sizeof(double);
  const bool force_global = env_flag("NKHIP_DROP_GLOBAL") != 0;  // (read per launch: tests flip it)
  if (!force_global && lds <= kPmaLdsMax) {
    static const hipError_t attr = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&mems_resid_kernel<true>),
        hipFuncAttributeMaxDynamicSharedMemorySize, int(kPmaLdsMax));
    if (attr != hipSuccess) return attr;
    hipLaunchKernelGGL(mems_resid_kernel<true>, dim3(1), dim3(DB), lds, s, P, make_coefs(P), Mp,
                       M, S, x, y, alpha, uval, cn, mode, f0, sc, out, xt, uxx, uyy, partial, znorm2,
                       omega, prm);
  } else {
    hipLaunchKernelGGL(mems_resid_kernel<false>, dim3(1), dim3(DB), 0, s, P, make_coefs(P), Mp, M,
                       S, x, y, alpha, uval, cn, mode, f0, sc, out, xt, uxx, uyy, partial, znorm2,
                       omega, prm);
  }
  return hipGetLastError();
}

// Host side: DCT matrices, the (1 - gamma Leig) divisor and the MFMA fragment tables, uploaded
// once per stepper.
namespace {
size_t frag_size(int tiles, int K) { return size_t(tiles) * pma_ksteps(K) * 64; }
// the half length of product g's transformed axis (0, 2: eta = ny; 1, 3: xi = nx) and its tables
int pma_half(const DropParams& P, int g) { return ((g % 2 ? P.nx : P.ny) + 1) / 2; }
size_t pma_frag(const DropParams& P, int g) {
  const int hs = pma_half(P, g);
  return frag_size((hs + 15) / 16, hs);
}
}  // namespace

size_t drop_pma_table_size(const DropParams& P) {
  size_t n = size_t(P.nx) * P.nx + size_t(P.ny) * P.ny + size_t(P.nx) * P.ny;
  for (int g = 0; g < 4; ++g) n += 2 * pma_frag(P, g);
  return n;
}

PmaTables drop_pma_view(const DropParams& P, const double* t) {
  PmaTables T;
  T.cx = t;
  T.cy = T.cx + size_t(P.nx) * P.nx;
  T.den = T.cy + size_t(P.ny) * P.ny;
  const double* f = T.den + size_t(P.nx) * P.ny;
  for (int g = 0; g < 4; ++g)
    for (int e = 0; e < 2; ++e) {
      T.f[g][e] = f;
      f += pma_frag(P, g);
    }
  return T;
}

std::vector<double> drop_pma_tables(const DropParams& P) {
  std::vector<double> out(drop_pma_table_size(P), 0.0);
  const PmaTables T = drop_pma_view(P, out.data());
  auto W = [](const double* p) { return const_cast<double*>(p); };
  auto dct = [](int n, double* c) {
    for (int k = 0; k < n; ++k)
      for (int m = 0; m < n; ++m)
        c[size_t(k) * n + m] =
            std::sqrt((k == 0 ? 1.0 : 2.0) / n) * std::cos(M_PI * k * (2 * m + 1) / (2.0 * n));
  };
  const int nx = P.nx, ny = P.ny;
  dct(nx, W(T.cx));
  dct(ny, W(T.cy));
  double* den = W(T.den);
  for (int i = 0; i < ny; ++i)
    for (int j = 0; j < nx; ++j) {
      // M.Leig (:829-833), including the division by dksi*deta
      const double a = 2 * std::cos(M_PI * i / (ny - 1)) - 2;
      const double b = 2 * std::cos(M_PI * j / (nx - 1)) - 2;
      const double leig = (a * 1.0 + 1.0 * b) / (P.dksi * P.deta);
      den[size_t(i) * nx + j] = 1 - P.gamma * leig;
    }
  // fragment tables; A(m, k) / B(k, n) accessors with zero padding
  auto fill_a = [](double* f, int M, int K, auto A) {
    const int S = pma_ksteps(K);
    for (int mt = 0; mt < (M + 15) / 16; ++mt)
      for (int s = 0; s < S; ++s)
        for (int l = 0; l < 64; ++l) {
          const int m = 16 * mt + (l & 15), k = 4 * s + (l >> 4);
          f[(size_t(mt) * S + s) * 64 + l] = (m < M && k < K) ? A(m, k) : 0.0;
        }
  };
  auto fill_b = [](double* f, int K, int N, auto B) {
    const int S = pma_ksteps(K);
    for (int nt = 0; nt < (N + 15) / 16; ++nt)
      for (int s = 0; s < S; ++s)
        for (int l = 0; l < 64; ++l) {
          const int k = 4 * s + (l >> 4), n = 16 * nt + (l & 15);
          f[(size_t(nt) * S + s) * 64 + l] = (k < K && n < N) ? B(k, n) : 0.0;
        }
  };
  // dct_pair's operands, half index h, k < ceil(N/2): forward even / odd rows of C (the middle
  // column of an odd N halved on the even side -- it multiplies x_mid + x_mid -- and dropped on
  // the odd side), inverse C^T by even / odd frequency
  for (int g = 0; g < 4; ++g) {
    const int N = g % 2 ? nx : ny, hs = (N + 1) / 2;
    const double* C = g % 2 ? T.cx : T.cy;
    auto c = [&](int k, int m) { return C[size_t(k) * N + m]; };
    auto ent = [&](int odd, int h, int k) -> double {
      if (g < 2) {
        if (odd) return (2 * h + 1 < N && 2 * k + 1 != N) ? c(2 * h + 1, k) : 0.0;
        return 2 * k + 1 == N ? c(2 * h, k) / 2 : c(2 * h, k);
      }
      const int fk = 2 * k + odd;
      return fk < N ? c(fk, h) : 0.0;
    };
    for (int e = 0; e < 2; ++e) {
      if (g % 2 == 0)
        fill_a(W(T.f[g][e]), hs, hs, [&](int m, int k) { return ent(e, m, k); });
      else
        fill_b(W(T.f[g][e]), hs, hs, [&](int k, int n) { return ent(e, n, k); });
    }
  }
  return out;
}

hipError_t drop_pma_launch(const DropParams& P, DropMesh M, DropScratch S, double* q,
                           const double* uval, const double* uxx0, const double* uyy0,
                           const PmaTables& T, double dtm, int loops, hipStream_t s,
                           int monitor) {
  if (!shape_ok(P) || loops < 1 || (monitor != kMonLap && monitor != kMonGap))
    return hipErrorInvalidValue;
  static unsigned long long* tprof = [] {
    unsigned long long* t = nullptr;
    if (env_flag("NKHIP_PMA_TIMING") && hipMalloc(&t, 64) != hipSuccess) t = nullptr;
    return t;
  }();
  const size_t lds = 3 * size_t(P.ny) * (P.nx | 1) * sizeof(double);
  const bool force_global = env_flag("NKHIP_DROP_GLOBAL") != 0;  // (read per launch: tests flip it)
  if (!force_global && lds <= kPmaLdsMax) {
    static const hipError_t attr = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&drop_pma_lds_kernel),
        hipFuncAttributeMaxDynamicSharedMemorySize, int(kPmaLdsMax));
    if (attr != hipSuccess) return attr;
    hipLaunchKernelGGL(drop_pma_lds_kernel, dim3(1), dim3(DB), lds, s, P, make_coefs(P), M, S, q,
                       uval, uxx0, uyy0, T, dtm, loops, monitor, tprof);
  } else {
    hipLaunchKernelGGL(drop_pma_kernel, dim3(1), dim3(DB), 0, s, P, make_coefs(P), M, S, q, uval,
                       uxx0, uyy0, T, dtm, loops, monitor);
  }
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess && tprof && !force_global) {
    // debug: per-stage wall-clock (100 MHz) of this launch, to stderr
    unsigned long long h[6];
    if (hipMemcpyAsync(h, tprof, sizeof h, hipMemcpyDeviceToHost, s) == hipSuccess &&
        hipStreamSynchronize(s) == hipSuccess)
      std::fprintf(stderr,
                   "pma us/loop: mesh %.2f uders %.2f lap %.2f smooth+integral %.2f rhs %.2f "
                   "dct %.2f\n",
                   h[0] / 100.0 / loops, h[1] / 100.0 / loops, h[2] / 100.0 / loops,
                   h[3] / 100.0 / loops, h[4] / 100.0 / loops, h[5] / 100.0 / loops);
  }
  return e;
}

}  // namespace nk

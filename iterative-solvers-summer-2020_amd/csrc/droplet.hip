// Droplet (python_work/droplet.py) device kernels -- see droplet.h.
//
// Each launch is ONE workgroup of 1024 threads walking the 5551-point grid stage by stage
// (workgroup barriers between stages; intermediate fields in L2-resident scratch).  Formulas and
// their association order follow the reference line by line (cited per function); derivative
// matrices of make_M (droplet.py:778-833) are applied matrix-free with their exact coefficients
// (integer weights divided by 12*h or 12*h^2, as the reference builds them).
#include <cmath>
#include <vector>

#include "droplet.h"
#include "nk_device.h"

namespace nk {
namespace {

constexpr int DB = 1024;

// One 1-D derivative operator (a kron factor of make_M): interior weights at offsets -2..2 and
// explicit rows for the two outermost points at each end.
struct Op1 {
  double in[5];
  double r0[6], r1[6], rm2[6], rm1[6];  // rows 0, 1, n-2, n-1
  int n0, n1, nm2, nm1;                 // entries in those rows (rows n-2/n-1 end at column n-1)
};

struct Coefs {
  Op1 d1x, d1y, d2x, d2y;
};

Op1 make_d1(double h) {
  // dksiCentre / detaCentre factor (:795-806)
  Op1 o{};
  const double s = 12 * h;
  const double in[5] = {1, -8, 0, 8, -1};
  const double r0[5] = {-25, 48, -36, 16, -3}, r1[5] = {-3, -10, 18, -6, 1};
  const double rm2[5] = {-1, 6, -18, 10, 3}, rm1[5] = {3, -16, 36, -48, 25};
  for (int k = 0; k < 5; ++k) {
    o.in[k] = in[k] / s;
    o.r0[k] = r0[k] / s;
    o.r1[k] = r1[k] / s;
    o.rm2[k] = rm2[k] / s;
    o.rm1[k] = rm1[k] / s;
  }
  o.n0 = o.n1 = o.nm2 = o.nm1 = 5;
  return o;
}

Op1 make_d2(double h2) {
  // d2ksi / d2eta factor (:782-793)
  Op1 o{};
  const double s = 12 * h2;
  const double in[5] = {-1, 16, -30, 16, -1};
  const double r0[5] = {-415.0 / 6, 96, -36, 32.0 / 3, -1.5};
  const double r1[6] = {10, -15, -4, 14, -6, 1};
  const double rm2[6] = {1, -6, 14, -4, -15, 10};
  const double rm1[5] = {-1.5, 32.0 / 3, -36, 96, -415.0 / 6};
  for (int k = 0; k < 5; ++k) {
    o.in[k] = in[k] / s;
    o.r0[k] = r0[k] / s;
    o.rm1[k] = rm1[k] / s;
  }
  for (int k = 0; k < 6; ++k) {
    o.r1[k] = r1[k] / s;
    o.rm2[k] = rm2[k] / s;
  }
  o.n0 = 5;
  o.n1 = 6;
  o.nm2 = 6;
  o.nm1 = 5;
  return o;
}

// Apply a 1-D operator at position `pos` of an axis of length n; element k of the axis is
// v[k*stride].
__device__ __forceinline__ double op1(const Op1& o, const double* v, int pos, int n, int stride) {
  double acc = 0.0;
  if (pos >= 2 && pos <= n - 3) {
    acc = o.in[0] * v[(pos - 2) * stride] + o.in[1] * v[(pos - 1) * stride];
    if (o.in[2] != 0.0) acc += o.in[2] * v[pos * stride];
    acc += o.in[3] * v[(pos + 1) * stride] + o.in[4] * v[(pos + 2) * stride];
    return acc;
  }
  if (pos == 0) {
    for (int k = 0; k < o.n0; ++k) acc += o.r0[k] * v[k * stride];
  } else if (pos == 1) {
    for (int k = 0; k < o.n1; ++k) acc += o.r1[k] * v[k * stride];
  } else if (pos == n - 2) {
    for (int k = 0; k < o.nm2; ++k) acc += o.rm2[k] * v[(n - o.nm2 + k) * stride];
  } else {
    for (int k = 0; k < o.nm1; ++k) acc += o.rm1[k] * v[(n - o.nm1 + k) * stride];
  }
  return acc;
}

__device__ __forceinline__ double dx1(const Coefs& C, const double* v, int i, int j, int nx) {
  return op1(C.d1x, v + i * nx, j, nx, 1);
}
__device__ __forceinline__ double dy1(const Coefs& C, const double* v, int i, int j, int nx,
                                      int ny) {
  return op1(C.d1y, v + j, i, ny, nx);
}

// M.dksideta = kron(D1y, D1x) (:806): sum over the row operator of the column-derivatives.
__device__ __forceinline__ double dxy(const Coefs& C, const double* v, int i, int j, int nx,
                                      int ny) {
  const Op1& o = C.d1y;
  double acc = 0.0;
  if (i >= 2 && i <= ny - 3) {
    for (int k = -2; k <= 2; ++k)
      if (o.in[k + 2] != 0.0) acc += o.in[k + 2] * dx1(C, v, i + k, j, nx);
    return acc;
  }
  const double* w;
  int cnt, start;
  if (i == 0) { w = o.r0; cnt = o.n0; start = 0; }
  else if (i == 1) { w = o.r1; cnt = o.n1; start = 0; }
  else if (i == ny - 2) { w = o.rm2; cnt = o.nm2; start = ny - o.nm2; }
  else { w = o.rm1; cnt = o.nm1; start = ny - o.nm1; }
  for (int k = 0; k < cnt; ++k) acc += w[k] * dx1(C, v, start + k, j, nx);
  return acc;
}

// The explicit part of Laplace_operator along one axis (:616-668): v_xx (axis = x, A = A11) or
// v_yy (axis = y, A = A22) at position `pos` of a line of length n, element k at v[k*stride].
__device__ __forceinline__ double lap_axis(const double* v, const double* A, int pos, int n,
                                           int s, double h2) {
  auto V = [&](int k) { return v[k * s]; };
  auto a = [&](int k) { return A[k * s]; };
  const int m = pos;
  if (m >= 3 && m <= n - 4) {  // interior (:617-631)
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

__device__ __forceinline__ double PI(const DropParams& P, double h) {
  // disjoining pressure (:462-467)
  const double r = P.epsilon / h;
  return (P.n_exp - 1) * (P.m_exp - 1) * (pow(r, double(P.m_exp)) - pow(r, double(P.n_exp))) /
         (2 * P.epsilon * (P.n_exp - P.m_exp));
}

__device__ __forceinline__ double pressure(const DropParams& P, double h, double hxx, double hyy) {
  return -(hxx + hyy) + PI(P, h) + P.Bo * cos(P.alpha2) * h;  // (:469-473)
}

#define FOR_POINTS(NN)                                                     \
  for (int p_ = threadIdx.x; p_ < (NN); p_ += DB)                          \
    if (const int i_ = p_ / nx, j_ = p_ - i_ * nx; true)

// ---------------------------------------------------------------------------- kernels
__device__ void mesh_stage(const DropParams& P, const Coefs& C, const double* q, const DropMesh& M) {
  const int nx = P.nx, ny = P.ny, NN = nx * ny;
  // compute_Q_spatial_ders (:696-711), J (:376) and the Laplace metric (:612-614): point-wise
  FOR_POINTS(NN) {
    const int p = p_, i = i_, j = j_;
    const bool left = j == 0, right = j == nx - 1, bottom = i == 0, top = i == ny - 1;
    double qd = dx1(C, q, i, j, nx), qe = dy1(C, q, i, j, nx, ny);
    if (left) qd = P.endl;
    if (right) qd = P.endr;
    if (bottom) qe = P.endb;
    if (top) qe = P.endt;
    double t = 0.0;
    if (left) t = 25 / (6 * P.dksi) * fabs(P.endl);
    if (right) t = 25 / (6 * P.dksi) * fabs(P.endr);
    const double q2x = op1(C.d2x, q + i * nx, j, nx, 1) + t;
    t = 0.0;
    if (top) t = 25 / (6 * P.deta) * fabs(P.endt);
    if (bottom) t = 25 / (6 * P.deta) * fabs(P.endb);
    const double q2y = op1(C.d2y, q + j, i, ny, nx) + t;
    const double qxy = (left || right || top || bottom) ? 0.0 : dxy(C, q, i, j, nx, ny);
    const double J = q2x * q2y - qxy * qxy;
    M.dksi[p] = qd;
    M.deta[p] = qe;
    M.d2ksi[p] = q2x;
    M.d2eta[p] = q2y;
    M.dksideta[p] = qxy;
    M.J[p] = J;
    M.A11[p] = (qxy * qxy + q2y * q2y) / J;
    M.A22[p] = (qxy * qxy + q2x * q2x) / J;
    M.A12[p] = -(qxy * (q2x + q2y)) / J;
  }
}

__global__ void __launch_bounds__(DB) drop_mesh_kernel(DropParams P, Coefs C, const double* q,
                                                       DropMesh M) {
  mesh_stage(P, C, q, M);
}

// compute_u_spatial_ders (:713-727) first half: u_xi, u_eta with its boundary rules, incl. the
// U_dksi[Bottom] quirk (:722), as the cross-term inputs t1 = A12 u_eta, t2 = A12 u_xi.
__device__ void uders_stage(const DropParams& P, const Coefs& C, const DropMesh& M,
                            const DropScratch& S, const double* u) {
  const int nx = P.nx, ny = P.ny, NN = nx * ny;
  FOR_POINTS(NN) {
    const int p = p_, i = i_, j = j_;
    double ud = dx1(C, u, i, j, nx), ue = dy1(C, u, i, j, nx, ny);
    if (j == 0 || j == nx - 1) ud = 0.0;
    if (i == ny - 1) ue = 0.0;
    if (i == 0) ud = 0.0;
    S.t1[p] = M.A12[p] * ue;
    S.t2[p] = M.A12[p] * ud;
  }
}

// The shared tail of the residual / pde_rhs chains, given u (point values) in `u`:
//   stage L: v_xx, v_yy (explicit + cross terms t1 = A12 u_eta, t2 = A12 u_xi) -> u_xx, u_yy, p
//   stage P: p derivatives with dp/dn = 0 -> p_x, p_y -> A, B
//   stage F: F2 = J^-1 [d2eta A_xi - dksideta A_eta - dksideta B_xi + d2ksi B_eta]
// The caller has filled S.ud / S.ue (u derivatives with its own boundary rules), S.t1, S.t2.
__device__ void lap_pressure_stage(const DropParams& P, const Coefs& C, const DropMesh& M,
                                   const DropScratch& S, const double* u, double* uxx,
                                   double* uyy) {
  const int nx = P.nx, ny = P.ny, NN = nx * ny;
  FOR_POINTS(NN) {
    const int p = p_, i = i_, j = j_;
    const double vxx = lap_axis(u + i * nx, M.A11 + i * nx, j, nx, 1, P.dksi * P.dksi);
    const double vyy = lap_axis(u + j, M.A22 + j, i, ny, nx, P.deta * P.deta);
    double tx = dx1(C, S.t1, i, j, nx);
    if (j == 0 || j == nx - 1) tx = 0.0;
    double ty = dy1(C, S.t2, i, j, nx, ny);
    if (i == 0 || i == ny - 1) ty = 0.0;
    const double hxx = (vxx + tx) / M.J[p];
    const double hyy = (vyy + ty) / M.J[p];
    if (uxx) uxx[p] = hxx;
    if (uyy) uyy[p] = hyy;
    S.p[p] = pressure(P, u[p], hxx, hyy);
  }
}

__device__ void flux_AB_stage(const DropParams& P, const Coefs& C, const DropMesh& M,
                              const DropScratch& S, const double* u) {
  const int nx = P.nx, ny = P.ny, NN = nx * ny;
  FOR_POINTS(NN) {
    const int p = p_, i = i_, j = j_;
    double pd = dx1(C, S.p, i, j, nx), pe = dy1(C, S.p, i, j, nx, ny);
    if (j == 0 || j == nx - 1) pd = 0.0;
    if (i == 0 || i == ny - 1) pe = 0.0;
    const double pdx = (M.d2eta[p] * pd - M.dksideta[p] * pe) / M.J[p];
    const double pdy = (-M.dksideta[p] * pd + M.d2ksi[p] * pe) / M.J[p];
    const double h3 = pow(u[p], 3.0);
    S.A[p] = (pdx - P.Bo * sin(P.alpha2) / P.epsilon2) * h3 / 3;
    S.B[p] = pdy * h3 / 3;
  }
}

__device__ __forceinline__ double flux_div_point(const Coefs& C, const DropMesh& M,
                                                 const DropScratch& S, int p, int i, int j,
                                                 int nx, int ny) {
  return (M.d2eta[p] * dx1(C, S.A, i, j, nx) - M.dksideta[p] * dy1(C, S.A, i, j, nx, ny)
          - M.dksideta[p] * dx1(C, S.B, i, j, nx) + M.d2ksi[p] * dy1(C, S.B, i, j, nx, ny)) /
         M.J[p];
}

__global__ void __launch_bounds__(DB) drop_rhs_kernel(DropParams P, Coefs C, DropMesh M,
                                                      DropScratch S, const double* u,
                                                      double* uxx, double* uyy, double* F) {
  const int nx = P.nx, ny = P.ny, NN = nx * ny;
  uders_stage(P, C, M, S, u);
  __syncthreads();
  lap_pressure_stage(P, C, M, S, u, uxx, uyy);  // P.val = pressure(U.val, U.xx, U.yy) (:378)
  __syncthreads();
  flux_AB_stage(P, C, M, S, u);  // compute_P_spatial_ders (:683-694), pde_rhs A, B (:456-457)
  __syncthreads();
  FOR_POINTS(NN) { F[p_] = flux_div_point(C, M, S, p_, i_, j_, nx, ny); }
}

__global__ void __launch_bounds__(DB) drop_resid_kernel(DropParams P, Coefs C, DropMesh M,
                                                        DropScratch S, const double* x,
                                                        const double* y, double alpha,
                                                        const double* uval, const double* F,
                                                        double dt, int mode, const double* f0,
                                                        double sc, double* out, double* xt,
                                                        double* partial) {
  const int nx = P.nx, ny = P.ny, NN = nx * ny;
  FOR_POINTS(NN) {
    double w = x[p_];
    if (y) w = w + alpha * y[p_];
    S.w[p_] = w;
  }
  __syncthreads();
  // residual() feeds the raw derivatives to Laplace_operator (:437, no boundary rules)
  FOR_POINTS(NN) {
    const int p = p_, i = i_, j = j_;
    const double ud = dx1(C, S.w, i, j, nx), ue = dy1(C, S.w, i, j, nx, ny);
    S.t1[p] = M.A12[p] * ue;
    S.t2[p] = M.A12[p] * ud;
  }
  __syncthreads();
  lap_pressure_stage(P, C, M, S, S.w, nullptr, nullptr);
  __syncthreads();
  flux_AB_stage(P, C, M, S, S.w);
  __syncthreads();
  double red[3] = {0.0, 0.0, 0.0};
  FOR_POINTS(NN) {
    const int p = p_;
    const double F2 = flux_div_point(C, M, S, p, i_, j_, nx, ny);
    const double w = S.w[p];
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
  }
  if (mode == 0) {
    const double v = block_reduce<3, 1, DB>(red);
    if (threadIdx.x < 3) partial[threadIdx.x] = v;
  }
}

// ---------------------------------------------------------------------------- PMA mesh loop
// loop_pma (:589-599), solve_PMA (:578-587), compute_and_smooth_monitor (:729-760) as ONE
// persistent single-workgroup kernel running all `loops` iterations on the GPU.  The orthonormal
// DCT-II / -III (scipy.fft dct / idct, norm="ortho") are dense products with precomputed DCT
// matrices (91x91 and 61x61 at the reference size).
__global__ void __launch_bounds__(DB) drop_pma_kernel(DropParams P, Coefs C, DropMesh M, DropScratch S,
                                                      double* q, const double* uval,
                                                      const double* uxx0, const double* uyy0,
                                                      const double* Cx, const double* Cy,
                                                      const double* den, double dtm, int loops) {
  const int nx = P.nx, ny = P.ny, NN = nx * ny;
  __shared__ double bcast;
  double* uxx = S.A;  // u_xx, u_yy of the current mesh (first iteration: the caller's)
  double* uyy = S.B;
  for (int it = 0; it < loops; ++it) {
    if (it > 0) {
      // compute_Q_spatial_ders, J, compute_u_spatial_ders (:595-597)
      mesh_stage(P, C, q, M);
      __syncthreads();
      uders_stage(P, C, M, S, uval);
      __syncthreads();
      lap_pressure_stage(P, C, M, S, uval, uxx, uyy);
      __syncthreads();
    }
    const double* lx = it > 0 ? uxx : uxx0;
    const double* ly = it > 0 ? uyy : uyy0;
    // monitor |u_xx + u_yy|^2 (:737), then smoothing_iters passes of the 9-point filter (:740-759)
    double* T = S.ud;
    double* Mo = S.ue;
    for (int p = threadIdx.x; p < NN; p += DB) {
      const double s = fabs(lx[p] + ly[p]);
      T[p] = s * s;
    }
    __syncthreads();
    for (int sm = 0; sm < P.smoothing_iters; ++sm) {
      for (int p = threadIdx.x; p < NN; p += DB) {
        const int i = p / nx, j = p - i * nx;
        auto t = [&](int a, int b) { return T[a * nx + b]; };
        double v;
        const bool in_i = i > 0 && i < ny - 1, in_j = j > 0 && j < nx - 1;
        if (in_i && in_j) {
          v = t(i, j) + (t(i - 1, j) + t(i + 1, j) + t(i, j - 1) + t(i, j + 1)) / 8 +
              (t(i - 1, j - 1) + t(i - 1, j + 1) + t(i + 1, j - 1) + t(i + 1, j + 1)) / 16;
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
        Mo[p] = v;
      }
      __syncthreads();
      double* sw = T;
      T = Mo;
      Mo = sw;
    }
    // Mackenzie regularisation: mon += C * sum(mon |J|) dksi deta (:757-759)
    double part[1] = {0.0};
    for (int p = threadIdx.x; p < NN; p += DB) part[0] += T[p] * fabs(M.J[p]);
    const double tot = block_reduce<1, 1, DB>(part);
    if (threadIdx.x == 0) bcast = tot * P.dksi * P.deta;
    __syncthreads();
    const double integral = bcast;
    // q_rhs = sqrt(mon |J|) / alpha (:584)
    double* X = S.p;
    for (int p = threadIdx.x; p < NN; p += DB) {
      const double mon = T[p] + P.C * integral;
      X[p] = sqrt(mon * fabs(M.J[p])) / P.alpha;
    }
    __syncthreads();
    // 2-D DCT-II ortho: T1 = Cy X (along eta), T2 = T1 Cx^T (along xi) (:585)
    double* T1 = S.t1;
    for (int p = threadIdx.x; p < NN; p += DB) {
      const int k = p / nx, j = p - k * nx;
      double acc = 0.0;
      for (int i = 0; i < ny; ++i) acc += Cy[k * ny + i] * X[i * nx + j];
      T1[p] = acc;
    }
    __syncthreads();
    double* T2 = S.t2;
    for (int p = threadIdx.x; p < NN; p += DB) {
      const int k = p / nx, l = p - k * nx;
      double acc = 0.0;
      for (int j = 0; j < nx; ++j) acc += T1[k * nx + j] * Cx[l * nx + j];
      T2[p] = acc / den[p];  // / (1 - gamma Leig) (:586)
    }
    __syncthreads();
    // inverse (DCT-III ortho): Y1 = Cy^T T2, dQ = Y1 Cx (:586-587)
    for (int p = threadIdx.x; p < NN; p += DB) {
      const int i = p / nx, l = p - i * nx;
      double acc = 0.0;
      for (int k = 0; k < ny; ++k) acc += Cy[k * ny + i] * T2[k * nx + l];
      T1[p] = acc;
    }
    __syncthreads();
    for (int p = threadIdx.x; p < NN; p += DB) {
      const int i = p / nx, j = p - i * nx;
      double acc = 0.0;
      for (int l = 0; l < nx; ++l) acc += T1[i * nx + l] * Cx[l * nx + j];
      q[p] = q[p] + dtm * acc;  // Q.val += dt * Q.dt (:591, :599)
    }
    __syncthreads();
  }
}


Coefs make_coefs(const DropParams& P) {
  Coefs C;
  C.d1x = make_d1(P.dksi);
  C.d1y = make_d1(P.deta);
  C.d2x = make_d2(P.dksi * P.dksi);
  C.d2y = make_d2(P.deta * P.deta);
  return C;
}

bool shape_ok(const DropParams& P) { return P.nx >= 7 && P.ny >= 7; }

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
                             double* xt, double* partial, hipStream_t s) {
  if (!shape_ok(P)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(drop_resid_kernel, dim3(1), dim3(DB), 0, s, P, make_coefs(P), M, S, x, y,
                     alpha, uval, F, dt, mode, f0, sc, out, xt, partial);
  return hipGetLastError();
}

// Host side: DCT matrices and the (1 - gamma Leig) divisor, uploaded once per stepper.
void drop_pma_tables(const DropParams& P, std::vector<double>* cx, std::vector<double>* cy,
                     std::vector<double>* den) {
  auto dct = [](int n, std::vector<double>* c) {
    c->assign(size_t(n) * n, 0.0);
    for (int k = 0; k < n; ++k)
      for (int m = 0; m < n; ++m)
        (*c)[size_t(k) * n + m] =
            std::sqrt((k == 0 ? 1.0 : 2.0) / n) * std::cos(M_PI * k * (2 * m + 1) / (2.0 * n));
  };
  dct(P.nx, cx);
  dct(P.ny, cy);
  den->assign(size_t(P.nx) * P.ny, 0.0);
  for (int i = 0; i < P.ny; ++i)
    for (int j = 0; j < P.nx; ++j) {
      // M.Leig (:829-833), including the division by dksi*deta
      const double a = 2 * std::cos(M_PI * i / (P.ny - 1)) - 2;
      const double b = 2 * std::cos(M_PI * j / (P.nx - 1)) - 2;
      const double leig = (a * 1.0 + 1.0 * b) / (P.dksi * P.deta);
      (*den)[size_t(i) * P.nx + j] = 1 - P.gamma * leig;
    }
}

hipError_t drop_pma_launch(const DropParams& P, DropMesh M, DropScratch S, double* q,
                           const double* uval, const double* uxx0, const double* uyy0,
                           const double* Cx, const double* Cy, const double* den, double dtm,
                           int loops, hipStream_t s) {
  if (P.nx < 7 || P.ny < 7 || loops < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(drop_pma_kernel, dim3(1), dim3(DB), 0, s, P, make_coefs(P), M, S, q, uval, uxx0,
                     uyy0, Cx, Cy, den, dtm, loops);
  return hipGetLastError();
}

}  // namespace nk

// Thin-film droplet (python_work/droplet.py) on a mapped 2-D mesh: device kernels.
//
// The grid is small (91 x 61 = 5551 points in the reference, config 3), so every operator chain
// runs as ONE single-workgroup kernel whose stages are separated by workgroup barriers, with the
// intermediate fields in L2-resident scratch: one launch per residual evaluation instead of the
// reference's 10 sparse mat-vecs and ~60 NumPy passes (droplet.py:435-450).
//
// Layout: u[i*nx + j], i = eta row (ny), j = xi column (nx); Left/Right = columns 0/nx-1,
// Bottom/Top = rows 0/ny-1 (make_Ibdy, droplet.py:762-776).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace nk {

struct DropParams {
  int nx, ny;
  double dksi, deta;
  double endl, endr, endb, endt;  // domain limits (droplet.py:32-33)
  double epsilon;                 // precursor film (:24)
  int n_exp, m_exp;               // disjoining-pressure exponents (:48-49)
  double Bo, alpha2, epsilon2;    // Bond number, inclination, Ho/Lo (:47,50-51)
  double alpha, gamma, C;         // PMA: adaption speed, smoothing, Mackenzie constant (:40-42)
  int smoothing_iters;            // (:31)
  double a;                       // droplet profile sharpness of G/G2 (:24)
};

// Per-time-step fields of the mesh potential Q (compute_Q_spatial_ders :696-711, J :376) and
// the Laplace metric coefficients A11, A22, A12 (:612-614).
struct DropMesh {
  double *d2ksi, *d2eta, *dksideta, *J, *A11, *A22, *A12;
  double *dksi, *deta;  // Q_xi, Q_eta = the physical node coordinates x, y
};

// Scratch fields of the staged kernels (8 arrays of nx*ny doubles).
struct DropScratch {
  double *w, *ud, *ue, *t1, *t2, *p, *A, *B;
};

// Q -> DropMesh (one single-workgroup launch).
hipError_t drop_mesh_launch(const DropParams& P, const double* q, DropMesh M, hipStream_t s);

// Old-time quantities of evolve_with_PDE (:371-381): U.xx, U.yy (Laplacian with the
// compute_u_spatial_ders boundary rules, incl. the U_dksi[Bottom] quirk :722) and the CN term
// F = pde_rhs(U.val, U.xx, U.yy).
hipError_t drop_rhs_launch(const DropParams& P, const double* uval, DropMesh M, DropScratch S,
                           double* uxx, double* uyy, double* F, hipStream_t s);

// residual(w, F, dt) (:435-450) at w = x + alpha*y (y may be null).
//   mode 0: out = R(w); also xt <- w (if non-null) and partial[0..2] = sum R^2, max|R|, max|w|
//   mode 1: out = (R(w) - f0) / sc  (the finite-difference JVP of KrylovJacobian.matvec)
// znorm2 (optional, device): y is a raw basis vector whose |y|^2 is there; the kernel takes
// sc = omega / |v|, alpha = sc / |y| (v = y / |y|) from it instead of the arguments.
hipError_t drop_resid_launch(const DropParams& P, DropMesh M, DropScratch S, const double* x,
                             const double* y, double alpha, const double* uval, const double* F,
                             double dt, int mode, const double* f0, double sc, double* out,
                             double* xt, double* partial, hipStream_t s,
                             const double* znorm2 = nullptr, double omega = 0.0,
                             const double* prm = nullptr);
// prm (both residual launches; device-side Arnoldi control, nk_kernels.h kCtlPrm): alpha and
// the FD step sc from the control's parameter block (entries kArnMaxNV + 1, + 2); a step the
// control handed back (entry kArnMaxNV + 3) does nothing.

// compute_U2 (:413-423): u = eps + sum_d (1-eps) H2(G2(|x - x_d|, R_d), R_d, V_d) at the node
// coordinates x = (M.dksi, M.deta); `drops` holds ndrops (x, y, R, V) quadruples (by value).
constexpr int kMaxDrops = 8;
struct DropSet {
  double v[kMaxDrops][4];
  int n;
};
hipError_t drop_u2_launch(const DropParams& P, DropMesh M, const DropSet& drops, double* u,
                          hipStream_t s);

// PMA2 (python_work/PMA2_nk.py) physics on the same mapped mesh (:121-159, :400-413):
//   new_rhs(u) = -lambda/(1+u)^2 + lambda eps^(m-2)/(1+u)^m - beta^2 Lap(Lap u), 0 on the boundary
//   residual(u) = (u - U.val)/k - (new_rhs(u) + CN_term)/2
struct MemsParams {
  double lambd;    // lambda (:30)
  double lam_eps;  // lambda * eps^(m-2), evaluated on the host as the reference does
  double beta2;    // beta*beta
  double k;        // the global dt = k used by residual() (:51)
  int m;
  int pad_;
};

// mode 0: out = residual(x + alpha y), xt = x + alpha y, partial[0..2] = (sum R^2, max|R|, max|x|)
// mode 1: out = (residual(x + alpha y) - f0)/sc                          (forward-difference JVP)
// mode 2: out = new_rhs(x) (CN_term), uxx/uyy = Laplace_operator(x) (compute_u_spatial_ders),
//         partial[0] = max(-(1+x)^3), i.e. -compute_g() (:437-441)
hipError_t mems_resid_launch(const DropParams& P, const MemsParams& Mp, DropMesh M, DropScratch S,
                             const double* x, const double* y, double alpha, const double* uval,
                             const double* cn, int mode, const double* f0, double sc, double* out,
                             double* xt, double* uxx, double* uyy, double* partial, hipStream_t s,
                             const double* znorm2 = nullptr, double omega = 0.0,
                             const double* prm = nullptr);

// Device tables of the PMA solve (solve_PMA, :578-587): orthonormal DCT-II matrices Cx (nx*nx),
// Cy (ny*ny), den = 1 - gamma*Leig (ny*nx), and the operands of the four DCT products of the
// MFMA path with the transform's first butterfly folded in (droplet.hip dct_pair), in
// v_mfma_f64_16x16x4 fragment order (zero-padded to 16-wide tiles and 4-deep k steps), half
// index h < ceil(N/2), N the transformed length, C its DCT-II matrix:
//   f[0]: A = even / odd rows of Cy (T1 = Cy X)     f[1]: B, the same of Cx (T2 = T1 Cx^T)
//   f[2]: A = Cy^T by even / odd frequency (Y1)     f[3]: B, the same of Cx (dQ = Y1 Cx)
// f[g][0] even part, f[g][1] odd part.  A fragments: [t][s][lane] = A[16t + (lane&15)][4s +
// (lane>>4)]; B fragments: [t][s][lane] = B[4s + (lane>>4)][16t + (lane&15)].
struct PmaTables {
  const double *cx, *cy, *den;
  const double* f[4][2];
};
size_t drop_pma_table_size(const DropParams& P);
std::vector<double> drop_pma_tables(const DropParams& P);
PmaTables drop_pma_view(const DropParams& P, const double* packed);

// The PMA mesh loop loop_pma(dtm, loops) (:589-599) in one persistent single-workgroup launch.
// The first iteration uses the caller's u_xx, u_yy (and the mesh fields in M); q is updated in
// place.  Monitor (compute_and_smooth_monitor): kMonLap = |u_xx + u_yy|^2 (droplet.py:737,
// PMA2_nk.py:361 for eps > 0, p = 2); kMonGap = 1/(1+u)^6 from uval (PMA2_nk.py:357, eps = 0).
enum { kMonLap = 0, kMonGap = 1 };
hipError_t drop_pma_launch(const DropParams& P, DropMesh M, DropScratch S, double* q,
                           const double* uval, const double* uxx0, const double* uyy0,
                           const PmaTables& T, double dtm, int loops, hipStream_t s,
                           int monitor = kMonLap);

}  // namespace nk

// Swift-Hohenberg stepper problem and generic callback problem (see sh_problem.h).
#include "sh_problem.h"

#include <cmath>

namespace nk {

// ============================================================================================
// SHProblem
// ============================================================================================
SHProblem::SHProblem(Engine& E, int64_t ny, int64_t nx, int64_t ny_global, SHCoef c, int jvp_mode)
    : E_(E), ny_(ny), nx_(nx), ny_g_(ny_global), c_(c), jvp_mode_(jvp_mode) {
  if (hipMalloc(reinterpret_cast<void**>(&B_), sizeof(double) * Engine::pad(ny * nx)) !=
      hipSuccess) {
    B_ = nullptr;
    status_ = NK_ENOMEM;
    return;
  }
  if (dist()) {
    if (ny < 2) {
      status_ = NK_EINVAL;  // a 2-row halo must come from one neighbour
      return;
    }
    double* h = nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&h), sizeof(double) * 16 * nx) != hipSuccess) {
      status_ = NK_ENOMEM;
      return;
    }
    hx_ = h;
    hz_ = h + 4 * nx;
    hd_ = h + 8 * nx;
    hu_ = h + 12 * nx;
  }
}

SHProblem::~SHProblem() {
  if (B_) hipFree(B_);
  if (hx_) hipFree(hx_);
}

Field SHProblem::field(const double* p, const double* halo) const {
  if (!dist()) return periodic(p);
  return Field{p, halo, halo + 2 * nx_};
}

int SHProblem::halo(const double* v, double* h) {
  if (!dist()) return NK_OK;
  return E_.launch(K_HALO, 2.0 * 4 * 8 * nx_,
                   [&] {
                     return E_.comm->halo(v, h, h + 2 * nx_, ny_, nx_, E_.s) == NK_OK
                                ? hipSuccess
                                : hipErrorUnknown;
                   }) == NK_OK
             ? NK_OK
             : NK_ECOMM;
}

int SHProblem::prepare(const double* u_prev) {
  int rc = halo(u_prev, hu_);
  if (rc) return rc;
  StencilArgs A;
  A.ny = ny_;
  A.nx = nx_;
  A.a = field(u_prev, hu_);
  A.c = c_;
  A.out0 = B_;
  return E_.launch(K_BOLD, stencil_bytes_per_point(SMode::BOLD, false) * ny_ * nx_,
                   [&] { return stencil_launch(SMode::BOLD, A, E_.s, nullptr); });
}

int SHProblem::set_x0(const double* x0) { return halo(x0, hx_); }
int SHProblem::set_dir(const double* d) { return halo(d, hd_); }

int SHProblem::eval(const double* x, const double* p, double alpha, double* xt, double* F,
                    double* G, double red[3]) {
  StencilArgs A;
  A.ny = ny_;
  A.nx = nx_;
  A.a = field(x, hx_);
  A.b = (p == x) ? field(x, hx_) : field(p, hd_);
  A.alpha = alpha;
  A.p0 = B_;
  A.out0 = F;
  A.out1 = G;
  A.out2 = xt;
  A.c = c_;
  A.partial = E_.partial();
  int64_t nblk = 0;
  int rc = E_.launch(K_TRIAL, stencil_bytes_per_point(SMode::TRIAL, xt != nullptr) * ny_ * nx_,
                     [&] { return stencil_launch(SMode::TRIAL, A, E_.s, &nblk); });
  if (rc) return rc;
  return E_.reduce(nblk, 1, 3, red);
}

int SHProblem::jvp(const double* x0, const double* G0, const double* z, double zs, double sc,
                   double* w) {
  int rc = halo(z, hz_);
  if (rc) return rc;
  StencilArgs A;
  A.ny = ny_;
  A.nx = nx_;
  A.c = c_;
  A.out0 = w;
  if (jvp_mode_ == NK_JVP_ANALYTIC) {
    A.a = field(z, hz_);
    A.alpha = zs;
    A.p0 = x0;
    return E_.launch(K_AJVP, stencil_bytes_per_point(SMode::AJVP, false) * ny_ * nx_,
                     [&] { return stencil_launch(SMode::AJVP, A, E_.s, nullptr); });
  }
  A.a = field(x0, hx_);
  A.b = field(z, hz_);
  A.alpha = sc * zs;
  A.p0 = G0;
  A.sc = sc;
  return E_.launch(K_FDJVP, stencil_bytes_per_point(SMode::FDJVP, false) * ny_ * nx_,
                   [&] { return stencil_launch(SMode::FDJVP, A, E_.s, nullptr); });
}

int SHProblem::jvp_dev(const double* x0, const double* G0, const double* z, const double* znorm2,
                       double omega, double* w) {
  int rc = halo(z, hz_);
  if (rc) return rc;
  StencilArgs A;
  A.ny = ny_;
  A.nx = nx_;
  A.c = c_;
  A.out0 = w;
  A.znorm2 = znorm2;
  A.omega = omega;
  if (jvp_mode_ == NK_JVP_ANALYTIC) {
    A.a = field(z, hz_);
    A.p0 = x0;
    return E_.launch(K_AJVP, stencil_bytes_per_point(SMode::AJVP, false) * ny_ * nx_,
                     [&] { return stencil_launch(SMode::AJVP, A, E_.s, nullptr); });
  }
  A.a = field(x0, hx_);
  A.b = field(z, hz_);
  A.p0 = G0;
  return E_.launch(K_FDJVP, stencil_bytes_per_point(SMode::FDJVP, false) * ny_ * nx_,
                   [&] { return stencil_launch(SMode::FDJVP, A, E_.s, nullptr); });
}

// ============================================================================================
// CallbackProblem
// ============================================================================================
CallbackProblem::CallbackProblem(Engine& E, nk_residual_fn F, void* ctx, double* tmp, double* tmp2)
    : E_(E), F_(F), ctx_(ctx), tmp_(tmp), tmp2_(tmp2) {}

int CallbackProblem::norms(double* v, double* sum2, double* vmax) {
  VecList none;
  int64_t nblk = 0;
  int rc = E_.launch(K_COMBO, 16.0 * E_.n, [&] {
    return combo_launch(tmp2_, v, 1.0, none, 0, E_.n, E_.partial(), E_.s, &nblk);
  });
  if (rc) return rc;
  double red[2];
  rc = E_.reduce(nblk, 1, 2, red);
  *sum2 = red[0];
  *vmax = red[1];
  return rc;
}

int CallbackProblem::eval(const double* x, const double* p, double alpha, double* xt, double* F,
                          double* G, double red[3]) {
  const int64_t n = E_.n;
  const double* xe = x;
  if (xt || alpha != 0.0) {
    double* dst = xt ? xt : tmp_;
    int rc = E_.launch(K_AXPBY, 24.0 * n,
                       [&] { return axpby_launch(1.0, x, alpha, p, dst, n, E_.s); });
    if (rc) return rc;
    xe = dst;
  }
  int rc = E_.launch(K_USERF, 0.0, [&] {
    return F_(ctx_, xe, F, n) == 0 ? hipSuccess : hipErrorUnknown;
  });
  if (rc) return rc;
  double s2 = 0, fm = 0, xs = 0, xm = 0;
  rc = norms(F, &s2, &fm);
  if (!rc) rc = norms(const_cast<double*>(xe), &xs, &xm);
  if (rc) return rc;
  red[0] = s2;
  red[1] = fm;
  red[2] = xm;
  if (G != F) rc = E_.copy(G, F, n);
  return rc;
}

int CallbackProblem::jvp(const double* x0, const double* G0, const double* z, double zs, double sc,
                         double* w) {
  const int64_t n = E_.n;
  int rc = E_.launch(K_AXPBY, 24.0 * n,
                     [&] { return axpby_launch(1.0, x0, sc * zs, z, tmp_, n, E_.s); });
  if (rc) return rc;
  rc = E_.launch(K_USERF, 0.0, [&] {
    return F_(ctx_, tmp_, w, n) == 0 ? hipSuccess : hipErrorUnknown;
  });
  if (rc) return rc;
  return E_.launch(K_AXPBY, 24.0 * n, [&] { return fddiff_launch(w, G0, sc, n, E_.s); });
}

}  // namespace nk

// sh_linearised.py (:48-56) on the GPU: the semi-implicit step's SPD system solved by conjugate
// gradients with the operator applied matrix-free by the 13-point stencil (SMode::LINOP, which
// also forms the new search direction p = r + beta p_old on the fly and the fused p.Ap), plus a
// fused x/r update with r.r: two passes (88 B/point) and two scalar read-backs per iteration.
#include "shlin.h"

#include <cmath>

namespace nk {

ShLinStepper::ShLinStepper(int64_t ny, int64_t nx, double h, double r, double g, double k,
                           double rtol, int64_t maxiter, hipStream_t s, bool profile)
    : E(ny * nx, nullptr, s, profile, stencil_partial_slots(ny, nx)), ny_(ny), nx_(nx), g_(g),
      k_(k), rtol_(rtol), maxiter_(maxiter) {
  c_ = sh_coef(h, r, k, g);
  status_ = E.alloc(8, &v_);
}

int ShLinStepper::linop(const double* a, const double* b, double beta, const double* d,
                        double theta, double* w, double* out, int64_t* nblk) {
  StencilArgs A;
  A.ny = ny_;
  A.nx = nx_;
  A.a = Field{a, nullptr, nullptr};
  A.b = Field{b, nullptr, nullptr};
  A.alpha = beta;
  A.p0 = d;
  A.out0 = out;
  A.out2 = w;
  A.c = c_;
  A.theta = theta;
  A.partial = E.partial();
  return E.launch(K_TRIAL, stencil_bytes_per_point(SMode::LINOP, false) * E.n,
                  [&] { return stencil_launch(SMode::LINOP, A, E.s, nblk); });
}

int ShLinStepper::step(const double* U, const double* Uo, double* Unew, ShLinStats* st) {
  if (status_) return status_;
  const int64_t n = E.n;
  double *x = v_[0], *r = v_[1], *p = v_[2], *pn = v_[3], *q = v_[4], *d = v_[5], *zero = v_[6],
         *b = v_[7];
  int64_t nblk = 0;
  double red[3];
  int rc = E.launch(K_AXPBY, 24.0 * n, [&] { return shlin_diag_launch(U, Uo, k_, g_, d, n, E.s); });
  // b = (I + L k/2) U  (the zero vector stands in for D)
  if (!rc) rc = linop(U, U, 0.0, zero, -k_ / 2, pn, b, &nblk);
  // |b|^2 (combo rewrites b unchanged and sums its squares)
  VecList none{};
  if (!rc) rc = E.launch(K_COMBO, 16.0 * n, [&] {
    return combo_launch(b, b, 1.0, none, 0, n, E.partial(), E.s, &nblk);
  });
  if (!rc) rc = E.reduce(nblk, 1, 2, red);
  if (rc) return rc;
  const double bnorm = std::sqrt(red[0]);
  // warm start x = U: r = b - A U
  if (!rc) rc = E.copy(x, U, n);
  if (!rc) rc = linop(U, U, 0.0, d, k_ / 2, pn, q, &nblk);
  VecList mq{};
  mq.p[0] = q;
  mq.c[0] = -1.0;
  if (!rc) rc = E.launch(K_COMBO, 24.0 * n, [&] {
    return combo_launch(r, b, 1.0, mq, 1, n, E.partial(), E.s, &nblk);
  });
  if (!rc) rc = E.reduce(nblk, 1, 2, red);
  if (rc) return rc;
  double rr = red[0];
  const double stop = rtol_ * bnorm;
  double beta = 0.0;
  int64_t it = 0;
  while (std::sqrt(rr) > stop && it < maxiter_) {
    // p' = r + beta p; q = A p'; p'.q
    rc = linop(r, it == 0 ? r : p, beta, d, k_ / 2, pn, q, &nblk);
    if (!rc) rc = E.reduce(nblk, 1, 3, red);
    if (rc) return rc;
    const double pq = red[0];
    if (!(pq > 0.0)) return NK_NONFINITE;  // not SPD (g k U dominated) or non-finite data
    const double alpha = rr / pq;
    rc = E.launch(K_AXPBY, 48.0 * n, [&] {
      return cg_update_launch(x, r, pn, q, alpha, n, E.partial(), E.s, &nblk);
    });
    if (!rc) rc = E.reduce(nblk, 1, 1, red);
    if (rc) return rc;
    beta = red[0] / rr;
    rr = red[0];
    std::swap(p, pn);
    ++it;
  }
  rc = E.copy(Unew, x, n);
  if (!rc) rc = E.sync();
  if (st) {
    st->iters = it;
    st->relres = bnorm > 0 ? std::sqrt(rr) / bnorm : std::sqrt(rr);
  }
  if (rc) return rc;
  return std::isfinite(rr) ? (std::sqrt(rr) <= stop ? NK_OK : NK_NO_CONVERGENCE) : NK_NONFINITE;
}

}  // namespace nk

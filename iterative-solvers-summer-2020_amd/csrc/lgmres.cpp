// LGMRES inner solve of the Newton-Krylov core: scipy/sparse/linalg/_isolve/lgmres.py:120-230
// (x0 = 0, maxiter = 1, M = identity, prepend_outer_v = True, store_outer_Av = False) around the
// FGMRES Arnoldi process of scipy/sparse/linalg/_isolve/_gcrotmk.py:14-180.
//
// Device/host split per Arnoldi step j (one host synchronisation per step):
//   host   h_j from the multi-dot of step j:  (I + L) h = V^T w_j  (inverse compact-WY MGS)
//   device combo_j:  v_{j+1} = w_j - V h_j,  |v_{j+1}|^2          -> device slot
//   device JVP_{j+1}(v_{j+1}) with its step taken from that device slot, then multi-dot_{j+1}
//   sync   host finishes step j (Givens QR of the Hessenberg column, residual test).
// When step j turns out to be the last one, the JVP/multi-dot issued for j+1 are discarded.
#include <cfloat>
#include <cmath>
#include <cstring>

#include "nk_solver.h"

namespace nk {

namespace {
constexpr double kEps = DBL_EPSILON;
}

int NewtonKrylov::issue_step(int j, int n_o, const double* sig, const double* rn, bool dev_scale) {
  const int64_t n = E_.n;
  const double* z;
  double zsig, zrn;
  if (j < n_o) {  // augmentation vectors first (_gcrotmk.py:107-110)
    const int slot = (ohead_ + j) % int(outer_.size());
    z = outer_[slot];
    zsig = osig_[slot];
    zrn = orn_[slot];
  } else if (j == n_o) {  // then v0 (:111-113)
    z = V_[0];
    zsig = sig[0];
    zrn = rn[0];
  } else {  // then the newest basis vector (:117-118)
    z = V_[j];
    zsig = dev_scale ? 0.0 : sig[j];
    zrn = dev_scale ? 0.0 : rn[j];
  }
  zp_[j] = z;
  zs_[j] = zsig;  // fixed up by the caller once sig[j] is known (dev_scale)
  double* w = V_[j + 1];
  int rc;
  if (dev_scale) {
    rc = P_.jvp_dev(X_, G0_, z, E_.dres(Engine::kSlotCombo), omega_, w);
    st_->njvp += 1;
  } else {
    const double nv = zsig * zrn;  // |z|_2 of the normalised vector (KrylovJacobian.matvec)
    if (nv == 0.0) {
      rc = E_.launch(K_COPY, 8.0 * n,
                     [&] { return hipMemsetAsync(w, 0, sizeof(double) * n, E_.s); });
    } else {
      rc = P_.jvp(X_, G0_, z, zsig, omega_ / nv, w);
      st_->njvp += 1;
    }
  }
  if (rc) return rc;
  st_->n_arnoldi += 1;
  // one pass: c_i = w.v_i (i <= j), Gram row v_j.v_i (i < j), |w|^2
  VecList P;
  for (int i = 0; i <= j; ++i) P.p[i] = V_[i];
  int64_t nblk = 0;
  const double* g = (j > 0) ? V_[j] : nullptr;
  rc = E_.launch(K_MDOT, 8.0 * n * (j + 2),
                 [&] { return mdot_launch(w, g, P, j + 1, n, E_.partial(), E_.s, &nblk); });
  if (rc) return rc;
  const int np = j + 1;
  return E_.reduce_async(nblk, 2 * np + 1, 2 * np + 1, Engine::kSlotMdot);
}

int NewtonKrylov::lgmres(double tol, double* dnorm, double* dmax, double** dvec) {
  *dnorm = 0.0;
  *dmax = 0.0;
  *dvec = nullptr;
  const double b_norm = fx_norm_;
  if (!std::isfinite(b_norm)) return NK_BAD_RHS;  // lgmres.py:125-126
  if (b_norm == 0.0) return NK_OK;                // x = b = 0  -> zero step
  const double atol = std::max(0.0, tol * b_norm);
  const double r_norm = b_norm;  // r_outer = matvec(0) - b = -b (matvec(0) short-circuits)
  if (r_norm <= std::max(atol, tol * b_norm)) return NK_OK;
  const double ptol = std::min(1.0, std::max(atol, tol * b_norm) / r_norm);

  const int n_o = ocount_;
  const int m = o_.inner_m + n_o;
  const int64_t n = E_.n;
  V_[0] = Fx_;  // v0 = b / |b|, kept raw with scale 1/|b|
  double sig[kMaxVec + 2], rn[kMaxVec + 2];
  sig[0] = 1.0 / b_norm;
  rn[0] = b_norm;
  static thread_local double R[kMaxVec + 1][kMaxVec + 1];
  static thread_local double gram[kMaxVec + 1][kMaxVec + 1];
  double cs[kMaxVec + 1], sn[kMaxVec + 1], gv[kMaxVec + 2], hcur[kMaxVec + 2], h[kMaxVec + 1];
  double red[2 * kMaxVec + 2];
  for (int i = 0; i < kMaxVec + 2; ++i) gv[i] = 0.0;
  gv[0] = 1.0;
  int j = 0;
  bool breakdown = false;
  bool pending = false;  // a speculative JVP/multi-dot for step j+1 is in flight
  int rc = issue_step(0, n_o, sig, rn, false);
  if (!rc) rc = E_.sync();
  if (rc) return rc;
  for (j = 0; j < m; ++j) {
    // -- results of the multi-dot of step j
    const int np = j + 1;
    std::memcpy(red, E_.hres(Engine::kSlotMdot), sizeof(double) * (2 * np + 1));
    const double ww = red[2 * np];
    if (!std::isfinite(ww)) return NK_NONFINITE;  // _nonlin.py:1511-1512
    const double w_norm = std::sqrt(ww);
    for (int i = 0; i < j; ++i) gram[j][i] = sig[j] * sig[i] * red[np + i];
    // MGS coefficients from the Gram matrix: (I + L) h = V^T w (inverse compact WY form)
    for (int i = 0; i <= j; ++i) {
      double acc = sig[i] * red[i];
      for (int k = 0; k < i; ++k) acc -= gram[i][k] * h[k];
      h[i] = acc;
    }
    // -- v_{j+1} = w - V h and |v_{j+1}|^2 in one pass
    VecList U;
    for (int i = 0; i <= j; ++i) {
      U.p[i] = V_[i];
      U.c[i] = -h[i] * sig[i];
    }
    double* w = V_[j + 1];
    int64_t nblk = 0;
    rc = E_.launch(K_COMBO, 8.0 * n * (j + 3), [&] {
      return combo_launch(w, w, 1.0, U, j + 1, n, E_.partial(), E_.s, &nblk);
    });
    // only |v_{j+1}|^2 is used (a non-finite v shows up in it): one sum, one all-reduce on N GPUs
    if (!rc) rc = E_.reduce_async(nblk, 1, 1, Engine::kSlotCombo);
    if (rc) return rc;
    // -- speculatively start step j+1 when its direction is v_{j+1} (device-side JVP scale)
    const bool more = j + 1 < m;
    pending = more && (j + 1 > n_o) && P_.has_dev_scale();
    if (pending) {
      rc = issue_step(j + 1, n_o, sig, rn, true);
      if (rc) return rc;
    }
    rc = E_.sync();
    if (rc) return rc;
    const double hn = std::sqrt(E_.hres(Engine::kSlotCombo)[0]);
    for (int i = 0; i <= j; ++i) hcur[i] = h[i];
    hcur[j + 1] = hn;
    const double alpha = 1.0 / hn;
    sig[j + 1] = std::isfinite(alpha) ? alpha : 1.0;  // scipy leaves w unscaled then
    rn[j + 1] = hn;
    if (pending) zs_[j + 1] = sig[j + 1];
    if (!(hn > kEps * w_norm)) breakdown = true;
    // -- Givens update of the Hessenberg QR (qr_insert, _gcrotmk.py:146-158)
    for (int i = 0; i < j; ++i) {
      const double t = cs[i] * hcur[i] + sn[i] * hcur[i + 1];
      hcur[i + 1] = -sn[i] * hcur[i] + cs[i] * hcur[i + 1];
      hcur[i] = t;
    }
    detail::givens(hcur[j], hcur[j + 1], &cs[j], &sn[j]);
    hcur[j] = cs[j] * hcur[j] + sn[j] * hcur[j + 1];
    for (int i = 0; i <= j; ++i) R[i][j] = hcur[i];
    gv[j + 1] = -sn[j] * gv[j];
    gv[j] = cs[j] * gv[j];
    const double res = std::fabs(gv[j + 1]);
    if (res < ptol || breakdown) break;
    if (more && !pending) {
      rc = issue_step(j + 1, n_o, sig, rn, false);
      if (!rc) rc = E_.sync();
      if (rc) return rc;
    }
    pending = false;
  }
  if (pending) {  // the step issued for j+1 is not part of the Arnoldi process
    st_->njvp -= 1;
    st_->n_arnoldi -= 1;
  }
  if (j == m) j = m - 1;
  if (!std::isfinite(R[j][j])) return NK_OK;  // LinAlgError -> lgmres returns x = 0
  double y[kMaxVec + 1];
  detail::lstsq_upper(R, j + 1, gv, y);
  for (int i = 0; i <= j; ++i) {
    y[i] *= b_norm;  // y *= inner_res_0
    if (!std::isfinite(y[i])) return NK_OK;
  }
  // -- dx = sum_i y_i z_i into the next outer slot (the oldest one if the ring is full; the
  //    combination reads each element before writing it, so in-place is safe)
  const int K = int(outer_.size());
  const int slot = (o_.outer_k > 0 && ocount_ < o_.outer_k) ? (ohead_ + ocount_) % K : ohead_;
  VecList Z;
  for (int i = 0; i <= j; ++i) {
    Z.p[i] = zp_[i];
    Z.c[i] = y[i] * zs_[i];
  }
  int64_t nblk = 0;
  double* d = outer_[slot];
  rc = E_.launch(K_COMBO, 8.0 * n * (j + 2), [&] {
    return combo_launch(d, nullptr, 0.0, Z, j + 1, n, E_.partial(), E_.s, &nblk);
  });
  if (rc) return rc;
  double r2[2];
  rc = E_.reduce(nblk, 1, 2, r2);
  if (rc) return rc;
  const double nx = std::sqrt(r2[0]);
  if (nx > 0 && o_.outer_k > 0) {
    osig_[slot] = 1.0 / nx;
    orn_[slot] = nx;
    if (ocount_ < o_.outer_k)
      ++ocount_;
    else
      ohead_ = (ohead_ + 1) % K;
  }
  *dnorm = nx;
  *dmax = r2[1];
  *dvec = d;
  return NK_OK;
}

}  // namespace nk

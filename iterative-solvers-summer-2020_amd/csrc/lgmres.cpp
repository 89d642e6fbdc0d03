// LGMRES inner solve of the Newton-Krylov core: scipy/sparse/linalg/_isolve/lgmres.py:120-230
// (x0 = 0, maxiter = 1, M = identity, prepend_outer_v = True, store_outer_Av = False) around the
// FGMRES Arnoldi process of scipy/sparse/linalg/_isolve/_gcrotmk.py:14-180.
//
// Device/host split per Arnoldi step j -- one host synchronisation and ONE reduction (one
// all-reduce on N GPUs) per step:
//   host   h_j from the multi-dot of step j:  (I + L) h = V^T w_j  (inverse compact-WY MGS)
//   device combo_j:  v_{j+1} = tau w_j - V h_j  (no reduction)
//   device JVP_{j+1} of v_{j+1} / |v_{j+1}|_est, with |v_{j+1}|_est^2 = |w_j|^2 - |h_j|^2 (the
//          Pythagoras identity of the Gram-Schmidt step, exact in exact arithmetic)
//   device multi-dot_{j+1}: V^T w_{j+1}, the Gram row of v_{j+1} INCLUDING |v_{j+1}|^2, |w_{j+1}|^2
//   sync   host finishes step j with the exact |v_{j+1}| from that Gram diagonal (Givens QR of the
//          Hessenberg column, residual test) and rescales w_{j+1} by tau = |v|_est / |v|: the JVP
//          was applied to a vector of norm 1 +- rounding, as in KrylovJacobian.matvec, so
//          tau * w_{j+1} = J v_{j+1} with the exactly normalised v_{j+1}.
// When |v_{j+1}| << |w_j| the estimate cancels (|v|/|w| < 1e-6): that step reduces the exact
// norm before the JVP (its in-kernel scale), as does the last step.  When step j turns out to be
// the last one, the JVP/multi-dot issued for j+1 are discarded (not counted).
// NKHIP_LAGNORM=0 disables the lagged norm (every step reduces |v_{j+1}| first); so does a
// problem that must not evaluate a discarded JVP (a user callback: scipy's exact F-call count).
//
// Device-side control (device_steps, arnctl.hip): once a fused step applies J to the new basis
// vector itself, the same per-step arithmetic runs in a one-wave kernel between the fused
// launches and the host only queues launches ahead of it; the kernel hands the step that ends
// the process (or that needs a path it does not take) back to this loop.  NKHIP_DEVCTL=1/0
// forces it on/off (default: on with a communicator, see devctl_enabled).
#include <algorithm>
#include <atomic>
#include <cstddef>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "nk_solver.h"
#include "peer_dev.h"

namespace nk {

namespace {
constexpr double kEps = DBL_EPSILON;
constexpr double kLagMinRatio2 = 1e-12;  // (|v|_est / |w|)^2 below which the estimate is not used

// Default: on with a communicator, where the host path waits for a stream synchronisation after
// every all-reduce; off on one GPU, where polling the pinned result slots already costs only the
// ~6-12 us between two launches and the device path measured 0.5-0.9 % slower (its entry and
// hand-back launches per LGMRES call outweigh the ~5 us it saves per step).  Read per call.
bool devctl_enabled(bool multi) {
  const char* v = std::getenv("NKHIP_DEVCTL");
  if (v && v[0] == '0') return false;
  if (v && v[0] == '1') return true;
  return multi;
}

bool lag_enabled() {
  static const bool on = [] {
    const char* v = std::getenv("NKHIP_LAGNORM");
    return !(v && v[0] == '0');
  }();
  return on;
}
}  // namespace

int NewtonKrylov::issue_step(int j, const double* z, double zs, double znorm, bool dev_scale,
                             bool have_w) {
  const int64_t n = E_.n;
  zp_[j] = z;
  hS_->zs[j] = zs;  // provisional when the exact scale of z is only known later
  double* w = V_[j + 1];
  int rc;
  if (have_w) {  // the speculative JVP of the line search computed it (NewtonKrylov::line_search)
    rc = NK_OK;
    st_->njvp += 1;
  } else if (dev_scale) {  // z = raw basis vector whose |z|^2 the combo left in device memory
    rc = P_.jvp_dev(X_, G0_, z, E_.dres(Engine::kSlotCombo), omega_, w);
    st_->njvp += 1;
  } else if (znorm == 0.0) {  // KrylovJacobian.matvec: a zero vector maps to zero, no F call
    rc = E_.launch(K_COPY, 8.0 * n,
                   [&] { return hipMemsetAsync(w, 0, sizeof(double) * n, E_.s); });
    if (!rc) rc = P_.publish_edges(w);  // (not a stencil output: its edges, its pushed rows)
  } else {  // sc = omega / |v| with v = zs z (_nonlin.py:1505-1507)
    rc = P_.jvp(X_, G0_, z, zs, omega_ / znorm, w);
    st_->njvp += 1;
  }
  if (rc) return rc;  // (w enters the update of the next fused step: the JVP wrote its edges)
  st_->n_arnoldi += 1;
  // one pass: c_i = w.v_i (i <= j), Gram row v_j.v_i (i <= j, the diagonal is |v_j|^2), |w|^2
  VecList P;
  for (int i = 0; i <= j; ++i) P.p[i] = V_[i];
  int64_t nblk = 0;
  const double* g = (j > 0) ? V_[j] : nullptr;
  rc = E_.launch(K_MDOT, 8.0 * n * (j + 2),
                 [&] { return mdot_launch(w, g, P, j + 1, n, E_.partial(), E_.s, &nblk); });
  if (rc) return rc;
  const int np = j + 1;
  return E_.reduce_async(nblk, 2 * np + 1, 2 * np + 1, Engine::slot_mdot(j));
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
  const int K = int(outer_.size());
  const bool lag = lag_enabled() && P_.may_speculate();
  const bool devctl = lag && devctl_enabled(E_.comm != nullptr || P_.prefers_devctl());
  V_[0] = Fx_;  // v0 = b / |b|, kept raw with scale 1/|b|
  // the loop state (shared with the device-side control: nk_kernels.h ArnCtlState)
  ArnCtlState& S = *hS_;
  S.m = m;
  S.halt = 0;
  S.steps = 0;
  S.ptol = ptol;
  S.omega = omega_;
  S.lag_ratio2 = kLagMinRatio2;
  double* const sig = S.sig;
  double* const rn = S.rn;
  double* const sig_est = S.sig_est;
  double* const wnorm = S.wnorm;
  double* const zs_ = S.zs;
  double* const h = S.h;
  sig[0] = 1.0 / b_norm;
  rn[0] = b_norm;
  double hcur[kMaxVec + 2];
  double red[2 * kMaxVec + 2];
  for (int i = 0; i < kMaxVec + 2; ++i) S.gv[i] = 0.0;
  S.gv[0] = 1.0;

  // input of step j whose scale is known on the host: the augmentation vectors first
  // (_gcrotmk.py:107-110), then v0 (:111-113), then the newest basis vector (:117-118)
  auto input = [&](int j, const double** z, double* zs, double* zn) {
    if (j < n_o) {
      const int slot = (ohead_ + j) % K;
      *z = outer_[slot];
      *zs = osig_[slot];
      *zn = osig_[slot] * orn_[slot];
    } else {
      *z = V_[j > n_o ? j : 0];
      const int q = j > n_o ? j : 0;
      *zs = sig[q];
      *zn = sig[q] * rn[q];
    }
  };
  // Step i is complete once hn = |v_{i+1}| (raw) is known: Hessenberg column i, Givens update of
  // its QR (qr_insert, _gcrotmk.py:146-158), residual test (:165).  True when the process stops.
  // (arnctl.hip restates this for the device-side control.)
  auto finish = [&](int i, double hn) -> bool {
    for (int k = 0; k <= i; ++k) hcur[k] = h[k];
    hcur[i + 1] = hn;
    const double alpha = 1.0 / hn;
    sig[i + 1] = std::isfinite(alpha) ? alpha : 1.0;  // scipy leaves w unscaled then
    rn[i + 1] = hn;
    const bool breakdown = !(hn > kEps * wnorm[i]);
    for (int k = 0; k < i; ++k) {
      const double t = S.cs[k] * hcur[k] + S.sn[k] * hcur[k + 1];
      hcur[k + 1] = -S.sn[k] * hcur[k] + S.cs[k] * hcur[k + 1];
      hcur[k] = t;
    }
    detail::givens(hcur[i], hcur[i + 1], &S.cs[i], &S.sn[i]);
    hcur[i] = S.cs[i] * hcur[i] + S.sn[i] * hcur[i + 1];
    for (int k = 0; k <= i; ++k) S.R[k][i] = hcur[k];
    S.gv[i + 1] = -S.sn[i] * S.gv[i];
    S.gv[i] = S.cs[i] * S.gv[i];
    return std::fabs(S.gv[i + 1]) < ptol || breakdown;
  };

  int rc;
  {
    const double* z;
    double zs, zn;
    input(0, &z, &zs, &zn);
    // the line search's speculative JVP applied J to this same input at this same point (the
    // accepted trial's pool vectors are the iterate and its G now)
    const bool have = spec_.valid && n_o > 0 && z == spec_.z && zs == spec_.zs &&
                      zn == spec_.zn && V_[1] == spec_.w && X_ == spec_.x && G0_ == spec_.g;
    spec_.valid = false;
    rc = issue_step(0, z, zs, zn, false, have);
  }
  sig_est[0] = 0.0;
  if (!rc) rc = E_.sync();
  if (rc) return rc;
  int j = 0, last = 0;
  bool hn_pending = false;  // step j-1 still waits for |v_j| (Gram diagonal of multi-dot j)
  for (;;) {
    // -- results of the multi-dot of step j
    const int np = j + 1;
    std::memcpy(red, E_.hres(Engine::slot_mdot(j)), sizeof(double) * (2 * np + 1));
    double tau = 1.0;
    if (hn_pending) {
      hn_pending = false;
      if (finish(j - 1, std::sqrt(red[np + j]))) {  // step j's JVP/multi-dot are not part of it
        st_->njvp -= 1;
        st_->n_arnoldi -= 1;
        last = j - 1;
        break;
      }
      if (sig_est[j] > 0.0) {  // JVP_j saw v_j scaled by sig_est instead of the exact sig
        tau = sig[j] / sig_est[j];
        zs_[j] = sig[j];
      }
    }
    const double ww = tau * tau * red[2 * np];
    if (!std::isfinite(ww)) return NK_NONFINITE;  // _nonlin.py:1511-1512
    wnorm[j] = std::sqrt(ww);
    for (int i = 0; i < j; ++i) S.gram[j][i] = sig[j] * sig[i] * red[np + i];
    // MGS coefficients from the Gram matrix: (I + L) h = V^T w (inverse compact WY form)
    double hh = 0.0;
    for (int i = 0; i <= j; ++i) {
      double acc = tau * sig[i] * red[i];
      for (int k = 0; k < i; ++k) acc -= S.gram[i][k] * h[k];
      h[i] = acc;
      hh += acc * acc;
    }
    VecList U;
    for (int i = 0; i <= j; ++i) {
      U.p[i] = V_[i];
      U.c[i] = -h[i] * sig[i];
    }
    double* w = V_[j + 1];
    const bool more = j + 1 < m;
    const bool next_is_v = more && (j + 1 > n_o);  // step j+1 applies J to v_{j+1} itself
    const double est = ww - hh;                    // |v_{j+1}|^2 = |w|^2 - |h|^2
    const bool lag_step = more && lag && (!next_is_v || est > kLagMinRatio2 * ww);
    int64_t nblk = 0;
    if (lag_step && P_.has_fused(j + 1)) {
      // -- fused: v_{j+1} = tau w - V h, JVP_{j+1} and multi-dot_{j+1} in one pass over V
      //    (arnoldi.hip).  v_{j+1} lands in the spare vector, which then takes V_[j+1]'s place.
      const double* z = nullptr;
      double zs, zn;
      if (next_is_v) {
        const double e = std::sqrt(est);
        zs = 1.0 / e;
        zn = zs * e;
      } else {
        input(j + 1, &z, &zs, &zn);
      }
      if (zn != 0.0) {  // a zero augmentation vector maps to zero without an F call: unfused path
        const double* Vp[kMaxVec];
        double cc[kMaxVec];
        for (int i = 0; i <= j; ++i) {
          Vp[i] = V_[i];
          cc[i] = U.c[i];
        }
        int64_t nw = 0;
        double* vout = Sv_;
        rc = P_.fused_step(Vp, cc, j + 1, w, tau, X_, G0_, z, zs, omega_ / zn, vout, V_[j + 2],
                           &nw, nullptr);
        if (rc) return rc;
        Sv_ = V_[j + 1];
        V_[j + 1] = vout;
        zp_[j + 1] = next_is_v ? vout : z;
        zs_[j + 1] = zs;
        sig_est[j + 1] = next_is_v ? zs : 0.0;
        st_->njvp += 1;
        st_->n_arnoldi += 1;
        const int np1 = j + 2;
        rc = E_.reduce_async(nw, 2 * np1 + 1, 2 * np1 + 1, Engine::slot_mdot(j + 1));
        if (rc) return rc;
        hn_pending = true;
        ++j;
        if (devctl && next_is_v) {  // the following steps: device-side control
          S.j = j;
          S.hn_pending = 1;
          rc = device_steps();
          j = S.j;
          hn_pending = S.hn_pending != 0;
        } else {
          rc = E_.wait_results(Engine::slot_mdot(j), 2 * np1 + 1);
        }
        if (rc) return rc;
        continue;
      }
    }
    if (lag_step) {
      // -- v_{j+1} = tau w - V h (no reduction), then step j+1 right away
      const EdgeOut eo = P_.edge_out(w);  // v_{j+1}, a basis vector of later fused steps
      rc = E_.launch(K_COMBO, 8.0 * n * (j + 3), [&] {
        return combo_launch(w, w, tau, U, j + 1, n, nullptr, E_.s, &nblk, eo);
      });
      if (!rc) rc = P_.publish_edges(w, eo.E != nullptr);
      if (rc) return rc;
      const double* z;
      double zs, zn;
      if (next_is_v) {
        const double e = std::sqrt(est);
        z = w;
        zs = 1.0 / e;
        zn = zs * e;
        sig_est[j + 1] = zs;
      } else {
        input(j + 1, &z, &zs, &zn);
        sig_est[j + 1] = 0.0;
      }
      rc = issue_step(j + 1, z, zs, zn, false);
      if (rc) return rc;
      hn_pending = true;
      ++j;
      if (devctl && next_is_v && P_.has_jvp_prm() && zn != 0.0) {
        // the following steps under device-side control, unfused (update, JVP, multi-dot and
        // the reduction + control per step, no host round trip)
        S.j = j;
        S.hn_pending = 1;
        rc = device_steps();
        j = S.j;
        hn_pending = S.hn_pending != 0;
        if (rc) return rc;
        continue;
      }
      rc = E_.sync();
      if (rc) return rc;
      continue;
    }
    // -- v_{j+1} = tau w - V h and its exact |v_{j+1}|^2 before the next JVP
    // v_{j+1}'s edge array (written by the combination) and pushed edge rows, before the
    // all-reduce below orders them
    const EdgeOut eo = P_.edge_out(w);
    rc = E_.launch(K_COMBO, 8.0 * n * (j + 3), [&] {
      return combo_launch(w, w, tau, U, j + 1, n, E_.partial(), E_.s, &nblk, eo);
    });
    if (!rc) rc = P_.publish_edges(w, eo.E != nullptr);
    // only |v_{j+1}|^2 is used (a non-finite v shows up in it): one sum, one all-reduce on N GPUs
    if (!rc) rc = E_.reduce_async(nblk, 1, 1, Engine::kSlotCombo);
    if (rc) return rc;
    // speculatively start step j+1 with its scale taken from the device norm
    const bool spec = next_is_v && P_.has_dev_scale() && P_.may_speculate();
    if (spec) {
      rc = issue_step(j + 1, w, 0.0, 0.0, true);
      if (rc) return rc;
    }
    rc = E_.sync();
    if (rc) return rc;
    const bool stop = finish(j, std::sqrt(E_.hres(Engine::kSlotCombo)[0]));
    if (spec) zs_[j + 1] = sig[j + 1];
    if (stop || !more) {
      if (spec) {  // the step issued for j+1 is not part of the Arnoldi process
        st_->njvp -= 1;
        st_->n_arnoldi -= 1;
      }
      last = j;
      break;
    }
    if (!spec) {
      const double* z;
      double zs, zn;
      input(j + 1, &z, &zs, &zn);
      rc = issue_step(j + 1, z, zs, zn, false);
      if (!rc) rc = E_.sync();
      if (rc) return rc;
    }
    sig_est[j + 1] = 0.0;
    ++j;
  }
  j = last;
  if (!std::isfinite(S.R[j][j])) return NK_OK;  // LinAlgError -> lgmres returns x = 0
  double y[kMaxVec + 1];
  detail::lstsq_upper(S.R, j + 1, S.gv, y);
  for (int i = 0; i <= j; ++i) {
    y[i] *= b_norm;  // y *= inner_res_0
    if (!std::isfinite(y[i])) return NK_OK;
  }
  // -- dx = sum_i y_i z_i into the next outer slot (the oldest one if the ring is full; the
  //    combination reads each element before writing it, so in-place is safe)
  const int slot = (o_.outer_k > 0 && ocount_ < o_.outer_k) ? (ohead_ + ocount_) % K : ohead_;
  VecList Z;
  for (int i = 0; i <= j; ++i) {
    Z.p[i] = zp_[i];
    Z.c[i] = y[i] * zs_[i];
  }
  int64_t nblk = 0;
  double* d = outer_[slot];
  // d: the line search's direction and the newest augmentation vector (z of later fused steps):
  // its edge array (written by the combination), and on pushed-halo slabs its edge rows, before
  // the all-reduce below
  const EdgeOut eo = P_.edge_out(d);
  rc = E_.launch(K_COMBO, 8.0 * n * (j + 2), [&] {
    return combo_launch(d, nullptr, 0.0, Z, j + 1, n, E_.partial(), E_.s, &nblk, eo);
  });
  if (!rc) rc = P_.publish_edges(d, eo.E != nullptr);
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

int NewtonKrylov::device_steps() {
  ArnCtlState& S = *hS_;
  const int t0 = S.j;
  // the largest basis length the device issues fused steps for (every length up to it runs fused)
  int nvmax = t0;
  while (nvmax + 1 < S.m && nvmax + 1 <= kArnMaxNV &&
         (P_.has_fused(nvmax + 1) || P_.has_jvp_prm()))
    ++nvmax;
  if (nvmax < t0 + 1) return E_.wait_results(Engine::slot_mdot(t0), 2 * (t0 + 1) + 1);
  S.nv_max = nvmax;
  S.halt = 0;
  S.steps = 0;
  S.arrive = 0;
  S.done = 0;
  volatile uint32_t* st = status_;
  for (int t = t0; t < S.m && t < kMaxVec + 2; ++t) st[t] = 0;
  std::atomic_thread_fence(std::memory_order_release);
  // the state the control reads -- everything before R, and the Gram rows of the earlier steps
  // -- is copied from hS_ by the first control launch itself (arn_ctl_launch upload_rows = t0).
  // From here the device writes every committed value into hS_ as well (no read-back).

  const bool one = E_.comm == nullptr;  // no all-reduce: the reduction carries the control
  struct Rot {
    double* spare;
    double* v;
    bool fused;
    bool unfused;  // an unfused device step (update in place, JVP, multi-dot): nothing to rotate
    bool ctl;      // the step queued a reduction + control launch (not the fused launch's tail)
    bool red;      // ... and a separate reduction before it (the generic all-reduce path)
  };
  Rot rot[kMaxVec + 2];
  double cc[kMaxVec] = {};  // the launch arguments the parameter block overrides
  // the tail's wait bound, read per run of device steps (NKHIP_PEER_TIMEOUT_S may change between
  // runs: bench legs, tests)
  const uint64_t wait_ticks = device_wait_ticks();
  // the control of step t on the (all-reduced) multi-dot results in its slot
  // the control of step t on the (all-reduced) multi-dot results in its slot; `copy`: the
  // results also to the host slot (the all-reduce path leaves out its own D2H copy)
  auto control = [&](int t, bool copy, int upload_rows = -1) {
    const int slot = Engine::slot_mdot(t);
    return E_.launch(K_CTL, 0.0, [&] {
      return arn_ctl_launch(dS_, hS_, E_.dres(slot), copy ? E_.hres_mut(slot) : nullptr, prm_,
                            status_, t, E_.s, upload_rows);
    });
  };
  // the fused step nv = t + 1 with the parameters control t writes, its reduction into the slot
  // of step t + 1 and the control of step t + 1
  auto issue = [&](int t) -> int {
    rot[t] = Rot{Sv_, V_[t + 1], false, false, true, false};
    const int nval = 2 * (t + 2) + 1;
    const int slot = Engine::slot_mdot(t + 1);
    if (!P_.has_fused(t + 1)) {
      // unfused: v_{t+1} = tau w + sum c_i V_i in place of w = V_[t+1] (coefficients from the
      // parameter block), w' = J v_{t+1} -> V_[t+2], then the multi-dot of w' and v_{t+1}
      // against V_0..V_{t+1} -- the fused kernel's result layout, so the same reduction + control
      const int64_t n = E_.n;
      double* w = V_[t + 1];
      VecList U;
      for (int i = 0; i <= t; ++i) U.p[i] = V_[i];
      int rc = E_.launch(K_COMBO, 8.0 * n * (t + 3),
                         [&] { return combo_prm_launch(w, w, prm_, U, t + 1, n, E_.s); });
      if (!rc) rc = P_.jvp_prm(X_, G0_, w, prm_, V_[t + 2]);
      if (rc) return rc;
      zp_[t + 1] = w;
      rot[t].unfused = true;
      VecList Pm;
      for (int i = 0; i <= t + 1; ++i) Pm.p[i] = V_[i];
      int64_t nb = 0;
      rc = E_.launch(K_MDOT, 8.0 * n * (t + 4), [&] {
        return mdot_launch(V_[t + 2], w, Pm, t + 2, n, E_.partial(), E_.s, &nb);
      });
      if (rc) return rc;
      if (one)
        return E_.launch(K_CTL, 8.0 * nb * nval, [&] {
          return arn_reduce_ctl_launch(E_.partial(), nb, nval, E_.dres_mut(slot),
                                       E_.hres_mut(slot), dS_, hS_, prm_, status_, t + 1, E_.s);
        });
      rot[t].red = true;
      rc = E_.reduce_async(nb, nval, nval, slot, false);
      return rc ? rc : control(t + 1, true);
    }
    const double* Vp[kMaxVec];
    for (int i = 0; i <= t; ++i) Vp[i] = V_[i];
    double* vout = Sv_;
    int64_t nw = 0;
    // peer-memory slabs: the all-reduce runs inside a kernel (the fused launch's tail, or the
    // reduction + all-reduce + control launch after it)
    PeerArgs pa;
    const bool have_pa = !one && peer_fuse_enabled() && E_.comm->take_allreduce(&pa, nval);
    // the reduction + control in the fused launch's last blocks (NKHIP_ARN_TAIL=1; default: a
    // launch of their own after it).  Ranks sharing one GPU keep the separate launch: with 8
    // processes on one GPU, fused launches whose tails wait for the other ranks' all-reduce
    // contributions stalled until the peer wait timed out (4 ranks ran), so the all-reduce inside
    // a fused launch is kept to one rank per GPU (NKHIP_ARN_TAIL=2 forces it: tests).
    ArnTail tl;
    const char* te = std::getenv("NKHIP_ARN_TAIL");
    const bool tail_env = te && (te[0] == '1' || te[0] == '2');
    const bool want_tail = tail_env && (one || (have_pa && ((te && te[0] == '2') ||
                                                            !E_.comm->group_shares_device())));
    if (want_tail) {
      tl.S = dS_;
      tl.H = hS_;
      tl.result = E_.dres_mut(slot);
      tl.result_host = E_.hres_mut(slot);
      tl.prm = prm_;
      tl.status = status_;
      tl.t = t + 1;
      tl.nval = nval;
      tl.peer = !one;
      const uint64_t ticks = wait_ticks;
      tl.wait_ticks = ticks;
      if (have_pa) tl.pa = pa;
      // NKHIP_ARN_TAIL_TIMEOUT_S (read per launch): a shorter bound for the tail's waits -- its
      // own blocks' arrival and the peer all-reduce inside it (bench.py's pushed_tail leg, so a
      // stalled variant costs seconds, not the comparison)
      if (const char* e = std::getenv("NKHIP_ARN_TAIL_TIMEOUT_S")) {
        const double sec = std::atof(e);
        if (sec > 0) {
          const uint64_t t = uint64_t(double(ticks) * sec / device_wait_seconds());
          tl.wait_ticks = std::min(tl.wait_ticks, t);
          if (have_pa) tl.pa.wait_ticks = std::min(tl.pa.wait_ticks, t);
        }
      }
    }
    bool tail_used = false;
    int rc = P_.fused_step(Vp, cc, t + 1, V_[t + 1], 1.0, X_, G0_, nullptr, 1.0, 1.0, vout,
                           V_[t + 2], &nw, prm_, want_tail ? &tl : nullptr, &tail_used);
    if (rc) return rc;
    Sv_ = V_[t + 1];
    V_[t + 1] = vout;
    zp_[t + 1] = vout;
    rot[t].fused = true;
    if (tail_used) {
      rot[t].ctl = false;
      return NK_OK;
    }
    if (one)
      return E_.launch(K_CTL, 8.0 * nw * nval, [&] {
        return arn_reduce_ctl_launch(E_.partial(), nw, nval, E_.dres_mut(slot),
                                     E_.hres_mut(slot), dS_, hS_, prm_, status_, t + 1, E_.s);
      });
    if (have_pa)  // reduction, all-reduce and control in one launch
      return E_.launch(K_CTL, 8.0 * nw * nval, [&] {
        return arn_reduce_allreduce_ctl_launch(E_.partial(), nw, nval, E_.dres_mut(slot),
                                               E_.hres_mut(slot), pa, dS_, hS_, prm_, status_,
                                               t + 1, E_.s);
      });
    rot[t].red = true;
    rc = E_.reduce_async(nw, nval, nval, slot, false);
    return rc ? rc : control(t + 1, true);
  };
  // one fused step queued beyond the one whose control is awaited, so the stream never waits
  // for the host; a step handed back leaves at most one launch pair behind that does nothing
  // step t0's results came through the host's reduce_async; this launch uploads the state
  int rc = control(t0, false, t0);
  int next = t0;  // the next fused step to queue
  if (!rc) rc = issue(next++);
  int t = t0;
  while (!rc) {
    const uint32_t v = E_.wait_flag(status_ + t);
    if (v != 1) {
      // the control of step t never ran: a collective before it failed (a peer aborted or a
      // wait timed out: the communicator says so) or a HIP error
      if (v != 2) rc = (E_.comm && E_.comm->failed()) ? NK_ECOMM : NK_EHIP;
      break;
    }
    st_->njvp += 1;  // step t's fused step is part of the process
    st_->n_arnoldi += 1;
    st_->n_device_steps += 1;
    ++t;
    if (next == t && next + 1 <= nvmax) rc = issue(next++);
  }
  // step t was handed back: the fused steps queued from t on do nothing; undo their rotations
  int voided = 0, voided_unfused = 0, voided_ctl = 0, voided_red = 0;
  for (int u = next - 1; u >= t; --u) {
    voided_ctl += rot[u].ctl ? 1 : 0;
    voided_red += rot[u].red ? 1 : 0;
    if (rot[u].unfused) {  // its update and JVP saw the halt: V_[u+1], V_[u+2] untouched
      ++voided_unfused;
      continue;
    }
    if (!rot[u].fused) continue;
    Sv_ = rot[u].spare;
    V_[u + 1] = rot[u].v;
    ++voided;
  }
  // ... and their launches did no work: out of the kernel profile (the fused launches, and the
  // reduction + control launches each of those steps queued behind it)
  P_.void_fused_steps(voided);
  E_.void_last(K_CTL, voided_ctl);
  E_.void_last(K_COMBO, voided_unfused);
  E_.void_last(K_USERF, voided_unfused);
  E_.void_last(K_MDOT, voided_unfused);
  E_.void_last(K_REDUCE, voided_red);
  if (rc) return rc;
  // The voided reduction of slot_mdot(t + 1) may still write that pinned host slot after the
  // host resumes; drain the stream here so no later poll of the slot can meet a stale write
  // (one synchronisation per hand-back, i.e. per LGMRES call).
  if (voided > 0 && (rc = E_.sync()) != NK_OK) return rc;
  if (S.j != t || S.halt != 1 + t) return NK_EHIP;
  S.halt = 0;
  return NK_OK;
}

}  // namespace nk

// Droplet time-stepper (python_work/droplet.py evolve_with_PDE, :360-411) on the GPU: the mesh and
// old-time fields, the Newton-Krylov solve of residual(u, F, dt_n) (:383) through the shared
// NewtonKrylov core, and (droplet_pma.hip) the parabolic Monge-Ampere mesh loop (:589-599).
#include "droplet_problem.h"

#include <cmath>

namespace nk {

DropletProblem::DropletProblem(Engine& E, const DropParams& P) : E_(E), P_(P) {
  const int64_t n = int64_t(P.nx) * P.ny;
  const int64_t np = Engine::pad(n);
  const int nf = 9 + 8 + 8;  // mesh, scratch, state
  if (hipMalloc(reinterpret_cast<void**>(&pool_), sizeof(double) * np * nf) != hipSuccess) {
    pool_ = nullptr;
    status_ = NK_ENOMEM;
    return;
  }
  hipMemsetAsync(pool_, 0, sizeof(double) * np * nf, E_.s);
  double* q = pool_;
  auto take = [&]() {
    double* r = q;
    q += np;
    return r;
  };
  M_.d2ksi = take();
  M_.d2eta = take();
  M_.dksideta = take();
  M_.J = take();
  M_.A11 = take();
  M_.A22 = take();
  M_.A12 = take();
  M_.dksi = take();
  M_.deta = take();
  S_.w = take();
  S_.ud = take();
  S_.ue = take();
  S_.t1 = take();
  S_.t2 = take();
  S_.p = take();
  S_.A = take();
  S_.B = take();
  uval = take();
  unew = take();
  qval = take();
  F = take();
  uxx = take();
  uyy = take();
  tmp = take();
  tmp2 = take();
}

DropletProblem::~DropletProblem() {
  if (pool_) hipFree(pool_);
}

int DropletProblem::prepare() {
  int rc = E_.launch(K_USERF, 0.0, [&] { return drop_mesh_launch(P_, qval, M_, E_.s); });
  if (rc) return rc;
  return E_.launch(K_USERF, 0.0,
                   [&] { return drop_rhs_launch(P_, uval, M_, S_, uxx, uyy, F, E_.s); });
}

int DropletProblem::eval(const double* x, const double* p, double alpha, double* xt, double* Fo,
                         double* G, double red[3]) {
  int rc = E_.launch(K_USERF, 0.0, [&] {
    return drop_resid_launch(P_, M_, S_, x, (alpha != 0.0) ? p : nullptr, alpha, uval, F, dt_, 0,
                             nullptr, 1.0, Fo, xt, E_.partial(), E_.s);
  });
  if (rc) return rc;
  rc = E_.reduce(1, 1, 3, red);
  if (rc) return rc;
  if (G != Fo) rc = E_.copy(G, Fo, n_global());
  return rc;
}

int DropletProblem::jvp(const double* x0, const double* G0, const double* z, double zs, double sc,
                        double* w) {
  return E_.launch(K_USERF, 0.0, [&] {
    return drop_resid_launch(P_, M_, S_, x0, z, sc * zs, uval, F, dt_, 1, G0, sc, w, nullptr,
                             nullptr, E_.s);
  });
}

int DropletProblem::jvp_dev(const double* x0, const double* G0, const double* z,
                            const double* znorm2, double omega, double* w) {
  return E_.launch(K_USERF, 0.0, [&] {
    return drop_resid_launch(P_, M_, S_, x0, z, 0.0, uval, F, dt_, 1, G0, 1.0, w, nullptr, nullptr,
                             E_.s, znorm2, omega);
  });
}

int DropletProblem::jvp_prm(const double* x0, const double* G0, const double* z,
                            const double* prm, double* w) {
  return E_.launch(K_USERF, 0.0, [&] {
    return drop_resid_launch(P_, M_, S_, x0, z, 0.0, uval, F, dt_, 1, G0, 1.0, w, nullptr, nullptr,
                             E_.s, nullptr, 0.0, prm);
  });
}

// ============================================================================================
// DropletStepper
// ============================================================================================
DropletStepper::DropletStepper(const DropParams& Pp, const nk_opts& o, hipStream_t s)
    : opts(o), E(int64_t(Pp.nx) * Pp.ny, nullptr, s, o.profile != 0, 16), P(E, Pp) {
  if (P.status()) {
    status_ = P.status();
    return;
  }
  NK_ = std::make_unique<NewtonKrylov>(E, P, opts);
  if (NK_->status()) {
    status_ = NK_->status();
    return;
  }
  const std::vector<double> tab = drop_pma_tables(Pp);
  if (hipMalloc(reinterpret_cast<void**>(&tables_), sizeof(double) * tab.size()) != hipSuccess) {
    tables_ = nullptr;
    status_ = NK_ENOMEM;
    return;
  }
  hipMemcpyAsync(tables_, tab.data(), sizeof(double) * tab.size(), hipMemcpyHostToDevice, s);
  status_ = E.sync();
}

DropletStepper::~DropletStepper() {
  if (E.s) hipStreamSynchronize(E.s);
  if (tables_) hipFree(tables_);
}

int DropletStepper::set_state(const double* U, const double* Q) {
  int rc = E.copy(P.unew, U, E.n);
  if (!rc) rc = E.copy(P.uval, U, E.n);
  if (!rc) rc = E.copy(P.qval, Q, E.n);
  return rc ? rc : E.sync();
}

int DropletStepper::get_state(double* U, double* Q) {
  int rc = U ? E.copy(U, P.unew, E.n) : NK_OK;
  if (!rc && Q) rc = E.copy(Q, P.qval, E.n);
  return rc ? rc : E.sync();
}

int DropletStepper::prepare() { return P.prepare(); }

int DropletStepper::residual(const double* u, double dt, double* R) {
  P.set_dt(dt);
  double red[3];
  return P.eval(u, u, 0.0, nullptr, R, R, red);
}

int DropletStepper::solve(double dt, double* U, nk_stats* st) {
  P.set_dt(dt);
  return NK_->solve(P.uval, U, st);
}

int DropletStepper::pma(double dtm, int loops) {
  const DropParams& Pp = P.params();
  return E.launch(K_USERF, 0.0, [&] {
    return drop_pma_launch(Pp, P.mesh(), P.scratch(), P.qval, P.uval, P.uxx, P.uyy,
                           drop_pma_view(Pp, tables_), dtm, loops, E.s);
  });
}

int DropletStepper::step(double dt, double dtm, int loops, nk_stats* st, double* dt_used) {
  const double dt_n = dt * scale;  // :369
  int rc = E.copy(P.uval, P.unew, E.n);  // U.val = U.new.copy() (:370)
  if (!rc) rc = prepare();                // :372-381
  if (rc) return rc;
  rc = solve(dt_n, P.unew, st);  // :383 (a NoConvergence aborts the reference's run)
  if (rc) return rc;
  if (loops > 0) rc = pma(dtm, loops);  // :384
  if (rc) return rc;
  // scale += exp(-10 |U.new - U.val|_2) (:411)
  VecList D;
  D.p[0] = P.uval;
  D.c[0] = -1.0;
  int64_t nblk = 0;
  rc = E.launch(K_COMBO, 24.0 * E.n, [&] {
    return combo_launch(P.tmp, P.unew, 1.0, D, 1, E.n, E.partial(), E.s, &nblk);
  });
  double r2[2];
  if (!rc) rc = E.reduce(nblk, 1, 2, r2);
  if (rc) return rc;
  scale += std::exp(-10 * std::sqrt(r2[0]));
  if (dt_used) *dt_used = dt_n;
  return NK_OK;
}

int DropletStepper::init_coalescing(int vsteps, const DropSet& drops, double dtm, int loops) {
  DropSet arg = drops;
  for (int i = 1; i <= vsteps; ++i) {
    int rc = E.copy(P.uval, P.unew, E.n);  // U.val = U.new.copy() (:158)
    if (!rc) rc = prepare();                // mesh fields, J, U.xx/U.yy (:160-163)
    for (int d = 0; d < drops.n; ++d) arg.v[d][3] = drops.v[d][3] * i / vsteps;  // :165-166
    if (!rc) rc = E.launch(K_USERF, 0.0, [&] {
      return drop_u2_launch(P.params(), P.mesh(), arg, P.unew, E.s);  // :167
    });
    if (!rc && loops > 0) rc = pma(dtm, loops);  // :169
    if (rc) return rc;
  }
  const int rc = E.copy(P.uval, P.unew, E.n);  // :185
  return rc ? rc : E.sync();
}

int DropletStepper::field(int which, double* out) {
  const DropMesh& M = P.mesh();
  const double* src[] = {M.d2ksi, M.d2eta, M.dksideta, M.J, M.A11, M.A22, M.A12, M.dksi, M.deta,
                         P.F, P.uxx, P.uyy, P.uval, P.unew, P.qval};
  if (which < 0 || which >= int(sizeof(src) / sizeof(src[0]))) return NK_EINVAL;
  int rc = E.copy(out, src[which], E.n);
  return rc ? rc : E.sync();
}

}  // namespace nk

// PMA2 (python_work/PMA2_nk.py) MEMS time-stepper: the mesh fields, CN_term and the adaptive dt
// (:80-94), one parabolic Monge-Ampere mesh step (solve_PMA + Q.val += dt*Q.dt, :91/:100) and the
// Newton-Krylov solve of residual(u) (:97) through the shared NewtonKrylov core.
#include "mems_problem.h"

namespace nk {

int MemsProblem::prepare(double* g) {
  int rc = E_.launch(K_USERF, 0.0, [&] { return drop_mesh_launch(P_, qval, M_, E_.s); });
  if (rc) return rc;
  rc = E_.launch(K_USERF, 0.0, [&] {
    return mems_resid_launch(P_, Mp_, M_, S_, uval, nullptr, 0.0, uval, nullptr, 2, nullptr, 1.0,
                             F, nullptr, uxx, uyy, E_.partial(), E_.s);
  });
  if (rc) return rc;
  double red[3];
  rc = E_.reduce(1, 0, 1, red);
  if (!rc && g) *g = -red[0];
  return rc;
}

int MemsProblem::eval(const double* x, const double* p, double alpha, double* xt, double* Fo,
                      double* G, double red[3]) {
  int rc = E_.launch(K_USERF, 0.0, [&] {
    return mems_resid_launch(P_, Mp_, M_, S_, x, (alpha != 0.0) ? p : nullptr, alpha, uval, F, 0,
                             nullptr, 1.0, Fo, xt, nullptr, nullptr, E_.partial(), E_.s);
  });
  if (rc) return rc;
  rc = E_.reduce(1, 1, 3, red);
  if (rc) return rc;
  if (G != Fo) rc = E_.copy(G, Fo, n_global());
  return rc;
}

int MemsProblem::jvp(const double* x0, const double* G0, const double* z, double zs, double sc,
                     double* w) {
  return E_.launch(K_USERF, 0.0, [&] {
    return mems_resid_launch(P_, Mp_, M_, S_, x0, z, sc * zs, uval, F, 1, G0, sc, w, nullptr,
                             nullptr, nullptr, nullptr, E_.s);
  });
}

int MemsProblem::jvp_dev(const double* x0, const double* G0, const double* z,
                         const double* znorm2, double omega, double* w) {
  return E_.launch(K_USERF, 0.0, [&] {
    return mems_resid_launch(P_, Mp_, M_, S_, x0, z, 0.0, uval, F, 1, G0, 1.0, w, nullptr, nullptr,
                             nullptr, nullptr, E_.s, znorm2, omega);
  });
}

int MemsProblem::jvp_prm(const double* x0, const double* G0, const double* z, const double* prm,
                         double* w) {
  return E_.launch(K_USERF, 0.0, [&] {
    return mems_resid_launch(P_, Mp_, M_, S_, x0, z, 0.0, uval, F, 1, G0, 1.0, w, nullptr, nullptr,
                             nullptr, nullptr, E_.s, nullptr, 0.0, prm);
  });
}

MemsStepper::MemsStepper(const DropParams& Pp, const MemsParams& Mp, double epsilon,
                         const nk_opts& o, hipStream_t s)
    : opts(o), E(int64_t(Pp.nx) * Pp.ny, nullptr, s, o.profile != 0, 16), P(E, Pp, Mp),
      epsilon_(epsilon) {
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

MemsStepper::~MemsStepper() {
  if (E.s) hipStreamSynchronize(E.s);
  if (tables_) hipFree(tables_);
}

int MemsStepper::set_state(const double* U, const double* Q) {
  int rc = E.copy(P.unew, U, E.n);
  if (!rc) rc = E.copy(P.uval, U, E.n);
  if (!rc) rc = E.copy(P.qval, Q, E.n);
  return rc ? rc : E.sync();
}

int MemsStepper::get_state(double* U, double* Q) {
  int rc = U ? E.copy(U, P.unew, E.n) : NK_OK;
  if (!rc && Q) rc = E.copy(Q, P.qval, E.n);
  return rc ? rc : E.sync();
}

int MemsStepper::prepare(double* dt) {
  double g = 1.0;
  const int rc = P.prepare(&g);
  // compute_g (:437-441): min((1+u)^3) for eps == 0, else 1; dt = g*k moves mesh and clock only
  if (!rc && dt) *dt = (epsilon_ == 0.0 ? g : 1.0) * P.k();
  return rc;
}

int MemsStepper::residual(const double* u, double* R) {
  double red[3];
  return P.eval(u, u, 0.0, nullptr, R, R, red);
}

int MemsStepper::solve(double* U, nk_stats* st) { return NK_->solve(P.uval, U, st); }

int MemsStepper::pma(double dt) {
  const DropParams& Pp = P.params();
  return E.launch(K_USERF, 0.0, [&] {
    return drop_pma_launch(Pp, P.mesh(), P.scratch(), P.qval, P.uval, P.uxx, P.uyy,
                           drop_pma_view(Pp, tables_), dt, 1, E.s,
                           epsilon_ == 0.0 ? kMonGap : kMonLap);
  });
}

int MemsStepper::step(nk_stats* st, double* dt_used) {
  int rc = E.copy(P.uval, P.unew, E.n);  // U.val = U.new.copy() (:80)
  double dt = 0.0;
  if (!rc) rc = prepare(&dt);  // :83-94
  if (!rc) rc = solve(P.unew, st);  // :97 (NoConvergence aborts the reference's run)
  // solve_PMA's Q.dt depends only on U.val and the mesh of this step, so computing it after the
  // solve and applying Q.val += dt*Q.dt (:100) in the same launch is the reference's order
  if (!rc) rc = pma(dt);
  if (rc) return rc;
  time += dt;  // :103
  if (dt_used) *dt_used = dt;
  return NK_OK;
}

int MemsStepper::field(int which, double* out) {
  const DropMesh& M = P.mesh();
  const double* src[] = {M.d2ksi, M.d2eta, M.dksideta, M.J, M.A11, M.A22, M.A12, M.dksi, M.deta,
                         P.F, P.uxx, P.uyy, P.uval, P.unew, P.qval};
  if (which < 0 || which >= int(sizeof(src) / sizeof(src[0]))) return NK_EINVAL;
  int rc = E.copy(out, src[which], E.n);
  return rc ? rc : E.sync();
}

}  // namespace nk

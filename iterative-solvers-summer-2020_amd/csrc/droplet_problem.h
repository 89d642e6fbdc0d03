// Droplet problem for the Newton-Krylov core (see droplet_problem.cpp).
#pragma once

#include <memory>

#include "droplet.h"
#include "nk_solver.h"

namespace nk {

class DropletProblem : public Problem {
 public:
  DropletProblem(Engine& E, const DropParams& P);
  ~DropletProblem() override;
  int status() const { return status_; }
  int64_t n_global() const override { return int64_t(P_.nx) * P_.ny; }
  void set_dt(double dt) { dt_ = dt; }
  // mesh fields from qval, then U.xx, U.yy, F from uval (evolve_with_PDE :372-381)
  int prepare();
  int eval(const double* x, const double* p, double alpha, double* xt, double* F, double* G,
           double red[3]) override;
  int jvp(const double* x0, const double* G0, const double* z, double zs, double sc,
          double* w) override;
  // the FD step from the device norm of the raw basis vector: no host round trip between the
  // update of step j and the JVP of step j+1 (which the solver then issues speculatively)
  bool has_dev_scale() const override { return true; }
  int jvp_dev(const double* x0, const double* G0, const double* z, const double* znorm2,
              double omega, double* w) override;
  // the LGMRES inner loop under device-side control (no host round trip per Arnoldi step): each
  // step is a 5551-point single-workgroup residual plus small Krylov launches, latency-bound
  bool has_jvp_prm() const override { return true; }
  int jvp_prm(const double* x0, const double* G0, const double* z, const double* prm,
              double* w) override;
  bool prefers_devctl() const override { return true; }
  const DropMesh& mesh() const { return M_; }
  const DropScratch& scratch() const { return S_; }
  const DropParams& params() const { return P_; }
  double dt() const { return dt_; }

  // state and per-step fields (device, nx*ny each)
  double *uval = nullptr, *unew = nullptr, *qval = nullptr, *F = nullptr, *uxx = nullptr,
         *uyy = nullptr, *tmp = nullptr, *tmp2 = nullptr;

 protected:
  Engine& E_;
  DropParams P_;
  DropMesh M_{};
  DropScratch S_{};
  double* pool_ = nullptr;
  double dt_ = 0.0;
  int status_ = NK_OK;
};

// evolve_with_PDE (:360-411) one step at a time: state (U.new, Q.val), the adaptive-dt scale,
// the Newton-Krylov solver and the PMA tables.
class DropletStepper {
 public:
  DropletStepper(const DropParams& P, const nk_opts& o, hipStream_t s);
  ~DropletStepper();
  int status() const { return status_; }
  int set_state(const double* U, const double* Q);
  int get_state(double* U, double* Q);
  int prepare();                                             // :371-381 for the current state
  int residual(const double* u, double dt, double* R);       // :435-450
  int solve(double dt, double* U, nk_stats* st);             // :383 at the prepared mesh
  int pma(double dtm, int loops);                            // :384 / :589-599
  int step(double dt, double dtm, int loops, nk_stats* st, double* dt_used);  // :369-411
  // initialise_coalescing_droplets (:132-189) from the current state
  int init_coalescing(int vsteps, const DropSet& drops, double dtm, int loops);
  int field(int which, double* out);
  double scale = 1.0;
  nk_opts opts;
  Engine E;
  DropletProblem P;

 private:
  std::unique_ptr<NewtonKrylov> NK_;
  double* tables_ = nullptr;  // PMA DCT tables (drop_pma_tables)
  int status_ = NK_OK;
};

}  // namespace nk

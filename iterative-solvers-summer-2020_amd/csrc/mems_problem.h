// PMA2 (python_work/PMA2_nk.py) MEMS moving-mesh time-stepper on the GPU (see mems_problem.cpp).
#pragma once

#include <memory>

#include "droplet_problem.h"

namespace nk {

// The residual of PMA2_nk.py (:121-159) on the droplet's mesh/scratch storage: F holds CN_term.
class MemsProblem final : public DropletProblem {
 public:
  MemsProblem(Engine& E, const DropParams& P, const MemsParams& Mp)
      : DropletProblem(E, P), Mp_(Mp) {}
  // mesh fields from qval; U.xx, U.yy, CN_term from uval; g = min((1+u)^3) (:80-91, :100)
  int prepare(double* g);
  double k() const { return Mp_.k; }
  int eval(const double* x, const double* p, double alpha, double* xt, double* F, double* G,
           double red[3]) override;
  int jvp(const double* x0, const double* G0, const double* z, double zs, double sc,
          double* w) override;
  int jvp_dev(const double* x0, const double* G0, const double* z, const double* znorm2,
              double omega, double* w) override;
  int jvp_prm(const double* x0, const double* G0, const double* z, const double* prm,
              double* w) override;

 private:
  MemsParams Mp_;
};

// main()'s loop body (:77-106) one step at a time.
class MemsStepper {
 public:
  MemsStepper(const DropParams& P, const MemsParams& Mp, double epsilon, const nk_opts& o,
              hipStream_t s);
  ~MemsStepper();
  int status() const { return status_; }
  int set_state(const double* U, const double* Q);
  int get_state(double* U, double* Q);
  int prepare(double* dt);                           // :80-88 (+ CN_term, :94)
  int residual(const double* u, double* R);          // :121-159 at the prepared state
  int solve(double* U, nk_stats* st);                // :97
  int pma(double dt);                                // solve_PMA (:91) + Q.val += dt*Q.dt (:100)
  int step(nk_stats* st, double* dt_used);           // :77-103
  int field(int which, double* out);
  double time = 0.0;
  nk_opts opts;
  Engine E;
  MemsProblem P;

 private:
  std::unique_ptr<NewtonKrylov> NK_;
  double* tables_ = nullptr;
  double epsilon_;
  int status_ = NK_OK;
};

}  // namespace nk

// Semi-implicit Swift-Hohenberg stepper of python_work/sh_linearised.py (see shlin.cpp).
#pragma once

#include <vector>

#include "nk_solver.h"

namespace nk {

struct ShLinStats {
  int64_t iters = 0;     // CG iterations of the last step
  double relres = 0.0;   // |b - A x| / |b| at exit
};

// U[s+1] = solve(I + D - L k/2, (I + L k/2) U[s]), D = diag((5U[s] - U[s-1])^2 k/16 - g k U[s])
// (sh_linearised.py:48-56).  The reference factorises the sparse matrix (spsolve); here the
// matrix is never formed: it is symmetric positive definite whenever 1 + min(D) > k r/2
// (always for g = 0), so a matrix-free conjugate-gradient solve on the 13-point stencil replaces
// the direct solve, warm-started from U[s] and run to a relative residual of rtol.
class ShLinStepper {
 public:
  ShLinStepper(int64_t ny, int64_t nx, double h, double r, double g, double k, double rtol,
               int64_t maxiter, hipStream_t s, bool profile);
  int status() const { return status_; }
  int step(const double* U, const double* Uo, double* Unew, ShLinStats* st);
  Engine E;

 private:
  int linop(const double* a, const double* b, double beta, const double* d, double theta,
            double* w, double* out, int64_t* nblk);
  int64_t ny_, nx_;
  double g_, k_, rtol_;
  int64_t maxiter_;
  SHCoef c_{};
  std::vector<double*> v_;
  int status_ = NK_OK;
};

}  // namespace nk

/*
 * TEST INFRASTRUCTURE ONLY -- a plain-C restatement of the Swift-Hohenberg hot-path arithmetic of
 * /root/reference/python_work/sh_scipy_nk.py (C++ twin: cpp_work/.../main.cpp), used by the CPU
 * tests (ctypes) and built with AddressSanitizer + UndefinedBehaviorSanitizer by check_main.c
 * ("race detection / sanitizers").  Nothing in the product links it.
 *
 * Grids are row-major u[i*nx + j] (i = y row, j = x column), periodic in both directions, as the
 * reference's Lap blocks fix (sh_scipy_nk.py:34-35).
 */
#include "sh_oracle.h"

#include <stdlib.h>

static int64_t wrap(int64_t i, int64_t n) {
  const int64_t r = i % n;
  return r < 0 ? r + n : r;
}

/* y = Lap v: e (v[i+-1, j] + v[i, j+-1] - 4 v[i, j]), e = 1/h^2 (sh_scipy_nk.py:32-35;
 * main.cpp:38-71) */
void sho_lap5(const double* v, double* y, int64_t ny, int64_t nx, double e) {
  for (int64_t i = 0; i < ny; ++i)
    for (int64_t j = 0; j < nx; ++j) {
      const double s = v[wrap(i - 1, ny) * nx + j] + v[wrap(i + 1, ny) * nx + j] +
                       v[i * nx + wrap(j - 1, nx)] + v[i * nx + wrap(j + 1, nx)];
      y[i * nx + j] = e * (s - 4.0 * v[i * nx + j]);
    }
}

/* y = L v with L = -Lap*Lap - 2*Lap + (r-1)*I built as the reference builds it: two
 * applications of Lap (sh_scipy_nk.py:38-39; main.cpp:78-81), NOT the closed-form 13-point
 * coefficients the kernels use -- so agreement is an independent check of those coefficients. */
int sho_sh13(const double* v, double* y, int64_t ny, int64_t nx, double h, double r) {
  const double e = 1.0 / (h * h);
  const size_t n = (size_t)(ny * nx);
  double* l1 = (double*)malloc(sizeof(double) * n);
  double* l2 = (double*)malloc(sizeof(double) * n);
  if (!l1 || !l2) {
    free(l1);
    free(l2);
    return -1;
  }
  sho_lap5(v, l1, ny, nx, e);
  sho_lap5(l1, l2, ny, nx, e);
  for (size_t p = 0; p < n; ++p) y[p] = -l2[p] - 2.0 * l1[p] + (r - 1.0) * v[p];
  free(l1);
  free(l2);
  return 0;
}

/* F(u) = (u - Uo)/k - (L u + g u^2 - u^3 + L Uo + g Uo^2 - Uo^3)/2 with the reference's
 * association (sh_scipy_nk.py:47-49; main.cpp:19-32) */
int sho_residual(const double* u, const double* uo, double* F, int64_t ny, int64_t nx, double h,
                 double r, double k, double g) {
  const size_t n = (size_t)(ny * nx);
  double* Lu = (double*)malloc(sizeof(double) * n);
  double* Luo = (double*)malloc(sizeof(double) * n);
  int rc = (!Lu || !Luo) ? -1 : 0;
  if (!rc) rc = sho_sh13(u, Lu, ny, nx, h, r);
  if (!rc) rc = sho_sh13(uo, Luo, ny, nx, h, r);
  if (!rc)
    for (size_t p = 0; p < n; ++p) {
      const double uu = u[p] * u[p], oo = uo[p] * uo[p];
      F[p] = (u[p] - uo[p]) / k - (Lu[p] + g * uu - u[p] * uu + Luo[p] + g * oo - uo[p] * oo) / 2;
    }
  free(Lu);
  free(Luo);
  return rc;
}

/* KrylovJacobian.matvec's difference quotient (scipy/optimize/_nonlin.py:1505-1509) on this
 * residual in the closed form the fused Arnoldi kernel evaluates (csrc/arnoldi.hip centre()):
 * (alpha/sc) [z/k - (L z + z (g (2 x0 + t) - (3 x0 (x0 + t) + t^2)))/2], t = alpha z */
int sho_fd_closed(const double* x0, const double* z, double alpha, double sc, double* w,
                  int64_t ny, int64_t nx, double h, double r, double k, double g) {
  const size_t n = (size_t)(ny * nx);
  double* Lz = (double*)malloc(sizeof(double) * n);
  if (!Lz) return -1;
  int rc = sho_sh13(z, Lz, ny, nx, h, r);
  if (!rc)
    for (size_t p = 0; p < n; ++p) {
      const double t = alpha * z[p];
      const double D = g * (2.0 * x0[p] + t) - (3.0 * x0[p] * (x0[p] + t) + t * t);
      w[p] = (alpha / sc) * (z[p] / k - (Lz[p] + z[p] * D) / 2);
    }
  free(Lz);
  return rc;
}

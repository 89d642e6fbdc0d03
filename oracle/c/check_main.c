/*
 * TEST INFRASTRUCTURE ONLY -- self-check of the C restatement under AddressSanitizer and
 * UndefinedBehaviorSanitizer (built by oracle/c/Makefile's `asan` target, run by
 * tests/test_oracle_c.py).  On odd, rectangular and tiny periodic grids it compares
 *   * L v (two applications of Lap, the reference's construction) with a direct 13-point
 *     stencil of the closed-form coefficients (centre -20e^2+8e+r-1, axial+-1 8e^2-2e,
 *     diagonal -2e^2, axial+-2 -e^2);
 *   * the closed-form FD quotient with SciPy's two-evaluation quotient (G(x0 + a z) - G(x0))/sc
 *     in long double;
 * and exits non-zero on a mismatch (or on any sanitizer report).
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "sh_oracle.h"

static int64_t wrapi(int64_t i, int64_t n) {
  const int64_t r = i % n;
  return r < 0 ? r + n : r;
}

static double rnd(unsigned* s) {
  *s = *s * 1664525u + 1013904223u;
  return ((*s >> 8) / 16777216.0) * 2.0 - 1.0;
}

static long double G(long double w, long double Lw, double k, double g) {
  return w / k - (Lw + g * w * w - w * w * w) / 2;
}

static int check(int64_t ny, int64_t nx, double h, double r, double k, double g, unsigned seed) {
  const size_t n = (size_t)(ny * nx);
  double *v = malloc(sizeof(double) * n), *x0 = malloc(sizeof(double) * n);
  double *y = malloc(sizeof(double) * n), *w = malloc(sizeof(double) * n);
  double *xp = malloc(sizeof(double) * n), *Lx = malloc(sizeof(double) * n);
  double *Lxp = malloc(sizeof(double) * n);
  int bad = 0;
  if (!v || !x0 || !y || !w || !xp || !Lx || !Lxp) return 1;
  for (size_t p = 0; p < n; ++p) {
    v[p] = rnd(&seed);
    x0[p] = rnd(&seed);
  }
  const double e = 1.0 / (h * h);
  const double c0 = -20.0 * e * e + 8.0 * e + r - 1.0, c1 = 8.0 * e * e - 2.0 * e;
  const double c2 = -2.0 * e * e, c3 = -e * e;
  if (sho_sh13(v, y, ny, nx, h, r)) return 1;
  double worst = 0.0, scale = 0.0;
  for (int64_t i = 0; i < ny; ++i)
    for (int64_t j = 0; j < nx; ++j) {
#define V(a, b) v[wrapi(i + (a), ny) * nx + wrapi(j + (b), nx)]
      const double d = c0 * V(0, 0) + c1 * (V(1, 0) + V(-1, 0) + V(0, 1) + V(0, -1)) +
                       c2 * (V(1, 1) + V(1, -1) + V(-1, 1) + V(-1, -1)) +
                       c3 * (V(2, 0) + V(-2, 0) + V(0, 2) + V(0, -2));
#undef V
      worst = fmax(worst, fabs(d - y[i * nx + j]));
      scale = fmax(scale, fabs(d));
    }
  if (worst > 1e-12 * fmax(scale, 1.0)) {
    fprintf(stderr, "L %lldx%lld: two-Lap vs 13-point differ by %g (scale %g)\n", (long long)ny,
            (long long)nx, worst, scale);
    bad = 1;
  }
  const double alpha = 1e-3, sc = 0.5;
  if (sho_fd_closed(x0, v, alpha, sc, w, ny, nx, h, r, k, g)) return 1;
  for (size_t p = 0; p < n; ++p) xp[p] = x0[p] + alpha * v[p];
  if (sho_sh13(x0, Lx, ny, nx, h, r) || sho_sh13(xp, Lxp, ny, nx, h, r)) return 1;
  worst = 0.0;
  scale = 0.0;
  for (size_t p = 0; p < n; ++p) {
    const long double q = (G(xp[p], Lxp[p], k, g) - G(x0[p], Lx[p], k, g)) / sc;
    worst = fmax(worst, fabs((double)(q - w[p])));
    scale = fmax(scale, fabs(w[p]));
  }
  /* the two-evaluation form cancels ~1/alpha digits: compare to that rounding level */
  if (worst > 1e-9 * fmax(scale, 1.0)) {
    fprintf(stderr, "FD %lldx%lld: closed form vs two evaluations differ by %g (scale %g)\n",
            (long long)ny, (long long)nx, worst, scale);
    bad = 1;
  }
  free(v);
  free(x0);
  free(y);
  free(w);
  free(xp);
  free(Lx);
  free(Lxp);
  return bad;
}

int main(void) {
  const int64_t shapes[][2] = {{61, 61}, {5, 5}, {3, 7}, {1, 1}, {2, 9}, {64, 48}, {17, 128}};
  int bad = 0;
  for (size_t s = 0; s < sizeof(shapes) / sizeof(shapes[0]); ++s)
    bad |= check(shapes[s][0], shapes[s][1], 40.0 / 64.0, 0.01, 0.2, 1.0, 2020u + (unsigned)s);
  printf("%s\n", bad ? "MISMATCH" : "ok");
  return bad;
}

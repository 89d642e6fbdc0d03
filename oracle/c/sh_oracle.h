/* TEST INFRASTRUCTURE ONLY -- see sh_oracle.c. */
#ifndef SH_ORACLE_H
#define SH_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
void sho_lap5(const double* v, double* y, int64_t ny, int64_t nx, double e);
int sho_sh13(const double* v, double* y, int64_t ny, int64_t nx, double h, double r);
int sho_residual(const double* u, const double* uo, double* F, int64_t ny, int64_t nx, double h,
                 double r, double k, double g);
int sho_fd_closed(const double* x0, const double* z, double alpha, double sc, double* w,
                  int64_t ny, int64_t nx, double h, double r, double k, double g);
#ifdef __cplusplus
}
#endif
#endif

// The C++ twin's time loop (cpp_work/NewtonKrylov_Implementation/Project1/main.cpp:93-107)
// written against include/nkhip.h exactly as INTEGRATION.md section 3 shows it: nk_sh_create ->
// nk_sh_step (in place, U = nonlin_solve(residual, Uo, ...)) -> nk_sh_destroy, device buffers from
// hipMalloc, no Python.  tests/test_gpu_capi.py drives it on the reference's N = 5, d = 2 geometry
// (main.cpp:3-12) against the nk_n5_d2_tight fixture.
//
//   sh_step N d r k g f_tol nsteps in.bin out.bin
//     in.bin: N*N doubles (U0, row-major); out.bin: nsteps*N*N doubles (U after each step)
//     stdout: one line per step "step <s> nit <nit> nfev <nfev> njvp <njvp>"
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "nkhip.h"

int main(int argc, char** argv) {
  if (argc != 10) {
    std::fprintf(stderr, "usage: %s N d r k g f_tol nsteps in.bin out.bin\n", argv[0]);
    return 2;
  }
  const int64_t N = std::atoll(argv[1]);
  const double d = std::atof(argv[2]), r = std::atof(argv[3]), k = std::atof(argv[4]),
               g = std::atof(argv[5]), f_tol = std::atof(argv[6]);
  const int nsteps = std::atoi(argv[7]);
  const size_t n = size_t(N * N);
  std::vector<double> U(n);
  std::FILE* fi = std::fopen(argv[8], "rb");
  if (!fi || std::fread(U.data(), sizeof(double), n, fi) != n) {
    std::fprintf(stderr, "cannot read %s\n", argv[8]);
    return 2;
  }
  std::fclose(fi);

  double* U_dev = nullptr;
  if (hipMalloc(reinterpret_cast<void**>(&U_dev), n * sizeof(double)) != hipSuccess ||
      hipMemcpy(U_dev, U.data(), n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) {
    std::fprintf(stderr, "hip setup failed\n");
    return 3;
  }
  nk_opts o;
  nk_opts_default(&o);
  o.f_tol = f_tol;  // main.cpp:104 passes 6e-6; the fixture's solve is tighter
  nk_sh* sh = nullptr;
  int rc = nk_sh_create(&sh, N, N, N, d / double(N), r, k, g, &o, /*comm=*/nullptr,
                        /*stream=*/nullptr);
  if (rc != NK_OK) {
    std::fprintf(stderr, "nk_sh_create: %s\n", nk_status_string(rc));
    return 4;
  }
  std::vector<double> traj;
  for (int s = 0; s < nsteps; ++s) {  // main.cpp:94
    nk_stats st;
    rc = nk_sh_step(sh, U_dev, U_dev, &st);  // Uo = U; U = nonlin_solve(residual, Uo, ...)
    if (rc != NK_OK) {
      std::fprintf(stderr, "nk_sh_step: %s\n", nk_status_string(rc));
      return 5;
    }
    if (hipMemcpy(U.data(), U_dev, n * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
      return 3;
    traj.insert(traj.end(), U.begin(), U.end());
    std::printf("step %d nit %lld nfev %lld njvp %lld\n", s + 1, static_cast<long long>(st.nit),
                static_cast<long long>(st.nfev), static_cast<long long>(st.njvp));
  }
  nk_sh_destroy(sh);
  (void)hipFree(U_dev);
  std::FILE* fo = std::fopen(argv[9], "wb");
  if (!fo || std::fwrite(traj.data(), sizeof(double), traj.size(), fo) != traj.size()) return 2;
  std::fclose(fo);
  return 0;
}

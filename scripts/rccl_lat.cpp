// RCCL latency probe on one GPU (world size 1): self send/recv of a 2-row halo (the slab
// exchange of csrc/comm.cpp), and in-place all-reduces of 1 and 83 doubles (the per-Arnoldi-step
// reductions).  Build: hipcc --offload-arch=gfx950 -O2 scripts/rccl_lat.cpp -lrccl -o /tmp/rccl_lat
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>

#define CK(x)                                                         \
  do {                                                                \
    if ((x) != 0) {                                                   \
      std::printf("fail %s line %d\n", #x, __LINE__);                \
      return 1;                                                       \
    }                                                                 \
  } while (0)

int main() {
  ncclUniqueId id;
  CK(ncclGetUniqueId(&id));
  ncclComm_t c;
  CK(ncclCommInitRank(&c, 1, id, 0));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const size_t nx = 4096, cnt = 2 * nx;
  double *v, *lo, *hi, *r;
  CK(hipMalloc(&v, 8 * nx * 64));
  CK(hipMalloc(&lo, 8 * cnt));
  CK(hipMalloc(&hi, 8 * cnt));
  CK(hipMalloc(&r, 8 * 128));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto halo = [&]() {
    ncclGroupStart();
    ncclSend(v + 62 * nx, cnt, ncclDouble, 0, c, s);
    ncclSend(v, cnt, ncclDouble, 0, c, s);
    ncclRecv(lo, cnt, ncclDouble, 0, c, s);
    ncclRecv(hi, cnt, ncclDouble, 0, c, s);
    ncclGroupEnd();
  };
  for (int w = 0; w < 20; ++w) halo();
  const int it = 200;
  CK(hipEventRecord(a, s));
  for (int i = 0; i < it; ++i) halo();
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  std::printf("self halo send/recv 2x%zu doubles: %.1f us\n", cnt, 1e3 * ms / it);
  for (int n : {1, 83}) {
    for (int w = 0; w < 20; ++w) ncclAllReduce(r, r, n, ncclDouble, ncclSum, c, s);
    CK(hipEventRecord(a, s));
    for (int i = 0; i < it; ++i) ncclAllReduce(r, r, n, ncclDouble, ncclSum, c, s);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    std::printf("allreduce %d doubles: %.1f us\n", n, 1e3 * ms / it);
  }
  ncclCommDestroy(c);
  return 0;
}

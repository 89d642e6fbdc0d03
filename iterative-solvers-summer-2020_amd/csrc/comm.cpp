// Communicators for the row-slab decomposition (see comm.h).
#include "comm.h"

#include <rccl/rccl.h>

#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <vector>

#include "../../include/nkhip.h"

namespace nk {
namespace {

// ------------------------------------------------------------------------------------------
// RCCL: one process per GPU.  Halo = grouped ncclSend/ncclRecv with the ring neighbours on the
// solver's stream; reductions = ncclAllReduce in place on the device result vector.
// ------------------------------------------------------------------------------------------
struct RcclComm final : nk_comm {
  ncclComm_t c = nullptr;
  int r = 0, p = 1;
  double* bar = nullptr;  // barrier scratch, allocated on first use
  bool aborted = false;
  ~RcclComm() override {
    if (c) ncclCommDestroy(c);  // an aborted communicator was released in abort()
    if (bar) hipFree(bar);
  }
  int rank() const override { return r; }
  int size() const override { return p; }

  int allreduce(double* dev, int nsum, int nv, hipStream_t s) override {
    if (aborted) return NK_ECOMM;
    if (nsum > 0 && ncclAllReduce(dev, dev, size_t(nsum), ncclDouble, ncclSum, c, s) != ncclSuccess)
      return NK_ECOMM;
    if (nv > nsum &&
        ncclAllReduce(dev + nsum, dev + nsum, size_t(nv - nsum), ncclDouble, ncclMax, c, s) !=
            ncclSuccess)
      return NK_ECOMM;
    return NK_OK;
  }

  int halo(const double* v, double* lo, double* hi, int64_t ny, int64_t nx,
           hipStream_t s) override {
    const int prev = (r - 1 + p) % p, next = (r + 1) % p;
    const size_t cnt = size_t(2 * nx);
    // Sends to one peer are matched in posting order, so with p == 2 (prev == next) the
    // neighbour's first receive (its lo) gets our last rows and its second (its hi) our first.
    if (aborted) return NK_ECOMM;
    if (ncclGroupStart() != ncclSuccess) return NK_ECOMM;
    // every call inside the group is checked; the group is closed in any case
    ncclResult_t e = ncclSend(v + (ny - 2) * nx, cnt, ncclDouble, next, c, s);
    if (e == ncclSuccess) e = ncclSend(v, cnt, ncclDouble, prev, c, s);
    if (e == ncclSuccess) e = ncclRecv(lo, cnt, ncclDouble, prev, c, s);
    if (e == ncclSuccess) e = ncclRecv(hi, cnt, ncclDouble, next, c, s);
    const ncclResult_t g = ncclGroupEnd();
    if (e != ncclSuccess || g != ncclSuccess) {
      std::fprintf(stderr, "nkhip: RCCL halo failed: %s\n",
                   ncclGetErrorString(e != ncclSuccess ? e : g));
      return NK_ECOMM;
    }
    return NK_OK;
  }

  int barrier(hipStream_t s) override {
    if (aborted) return NK_ECOMM;
    if (!bar && hipMalloc(reinterpret_cast<void**>(&bar), sizeof(double)) != hipSuccess) {
      bar = nullptr;
      return NK_EHIP;
    }
    if (hipMemsetAsync(bar, 0, sizeof(double), s) != hipSuccess) return NK_EHIP;
    if (ncclAllReduce(bar, bar, 1, ncclDouble, ncclSum, c, s) != ncclSuccess) return NK_ECOMM;
    return hipStreamSynchronize(s) == hipSuccess ? NK_OK : NK_EHIP;
  }

  // Aborts this rank's communicator at once (ncclCommAbort releases its enqueued RCCL work and
  // its resources); every later call of this rank returns NK_ECOMM.  Peer PROCESSES are not
  // told: a peer blocked in a collective with this rank is released by its own failure handling
  // (the launcher / torch.distributed watchdog), not by this call (nkhip.h nk_comm_abort).
  void abort() override {
    if (aborted) return;
    aborted = true;
    if (c) {
      ncclCommAbort(c);
      c = nullptr;
    }
  }
};

// ------------------------------------------------------------------------------------------
// Loopback: `p` slabs on one device, each driven by its own host thread.  Halos are D2D copies
// from the neighbour's slab after a host barrier; reductions are combined on the host in rank
// order (deterministic).  Used to test the slab decomposition on a single GPU.
// ------------------------------------------------------------------------------------------
struct LoopShared {
  int p;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  int64_t gen = 0;
  std::vector<const double*> vptr;
  std::vector<int64_t> vny;
  std::vector<std::vector<double>> vals;
  bool aborted = false;
  explicit LoopShared(int np) : p(np), vptr(np), vny(np), vals(np) {}
  // false once any rank has aborted the group (then nobody waits for the missing rank)
  bool wait() {
    std::unique_lock<std::mutex> lk(m);
    if (aborted) return false;
    const int64_t g = gen;
    if (++arrived == p) {
      arrived = 0;
      ++gen;
      cv.notify_all();
      return true;
    }
    cv.wait(lk, [&] { return gen != g || aborted; });
    return gen != g;
  }
  void abort() {
    std::lock_guard<std::mutex> lk(m);
    aborted = true;
    cv.notify_all();
  }
};

struct LoopComm final : nk_comm {
  std::shared_ptr<LoopShared> sh;
  int r = 0;
  int rank() const override { return r; }
  int size() const override { return sh->p; }
  bool shares_device() const override { return true; }

  int allreduce(double* dev, int nsum, int nv, hipStream_t s) override {
    std::vector<double> host(nv);
    if (hipMemcpyAsync(host.data(), dev, sizeof(double) * nv, hipMemcpyDeviceToHost, s) !=
            hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
      sh->abort();
      return NK_EHIP;
    }
    sh->vals[r] = host;
    if (!sh->wait()) return NK_ECOMM;
    for (int k = 0; k < nv; ++k) {
      double acc = sh->vals[0][k];
      for (int q = 1; q < sh->p; ++q) {
        const double v = sh->vals[q][k];
        if (k < nsum)
          acc += v;
        else if (acc == acc && (v != v || v > acc))
          acc = v;
      }
      host[k] = acc;
    }
    if (!sh->wait()) return NK_ECOMM;
    if (hipMemcpyAsync(dev, host.data(), sizeof(double) * nv, hipMemcpyHostToDevice, s) !=
            hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return NK_EHIP;
    return NK_OK;
  }

  int halo(const double* v, double* lo, double* hi, int64_t ny, int64_t nx,
           hipStream_t s) override {
    const int p = sh->p, prev = (r - 1 + p) % p, next = (r + 1) % p;
    if (hipStreamSynchronize(s) != hipSuccess) {
      sh->abort();
      return NK_EHIP;
    }
    sh->vptr[r] = v;
    sh->vny[r] = ny;
    if (!sh->wait()) return NK_ECOMM;
    const size_t bytes = sizeof(double) * size_t(2 * nx);
    hipError_t e = hipMemcpyAsync(lo, sh->vptr[prev] + (sh->vny[prev] - 2) * nx, bytes,
                                  hipMemcpyDeviceToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(hi, sh->vptr[next], bytes, hipMemcpyDeviceToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    // nobody may overwrite its slab before every neighbour has copied
    if (!sh->wait()) return NK_ECOMM;
    if (e != hipSuccess) {
      sh->abort();
      return NK_EHIP;
    }
    return NK_OK;
  }

  int barrier(hipStream_t s) override {
    if (hipStreamSynchronize(s) != hipSuccess) {
      sh->abort();
      return NK_EHIP;
    }
    return sh->wait() ? NK_OK : NK_ECOMM;
  }

  void abort() override { sh->abort(); }
};

}  // namespace

int comm_unique_id_bytes() { return int(sizeof(ncclUniqueId)); }

int comm_get_unique_id(void* out) {
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return NK_ECOMM;
  std::memcpy(out, &id, sizeof(id));
  return NK_OK;
}

int comm_create_rccl(nk_comm** out, const void* uid, int rank, int nranks) {
  if (!out || !uid || nranks < 1 || rank < 0 || rank >= nranks) return NK_EINVAL;
  auto c = std::make_unique<RcclComm>();
  ncclUniqueId id;
  std::memcpy(&id, uid, sizeof(id));
  const ncclResult_t e = ncclCommInitRank(&c->c, nranks, id, rank);
  if (e != ncclSuccess) {
    std::fprintf(stderr, "nkhip: ncclCommInitRank failed: %s\n", ncclGetErrorString(e));
    c->c = nullptr;
    return NK_ECOMM;
  }
  c->r = rank;
  c->p = nranks;
  *out = c.release();
  return NK_OK;
}

int comm_create_loopback(nk_comm** out, int nranks) {
  if (!out || nranks < 1) return NK_EINVAL;
  auto sh = std::make_shared<LoopShared>(nranks);
  for (int q = 0; q < nranks; ++q) {
    auto c = new LoopComm();
    c->sh = sh;
    c->r = q;
    out[q] = c;
  }
  return NK_OK;
}

}  // namespace nk

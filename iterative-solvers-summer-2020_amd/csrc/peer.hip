// Peer-memory communicator for the row-slab decomposition (one process per GPU, xGMI).
//
// The slab path's collectives are tiny and latency-bound: per Arnoldi step one 2-row halo of
// 2 x nx doubles per neighbour and one all-reduce of 2 nv + 3 doubles (SURVEY.md section 5:
// "latency dominates, not the 153 GB/s link rate").  Through RCCL each costs a library call, its
// proxy/kernels and their own synchronisation (measured at world size 1: grouped send/recv
// 25 us).  Here every rank exports ONE fine-grained device buffer (IPC handle
// exchanged once through any side channel, e.g. torch.distributed); afterwards a collective is
// one small kernel on the solver's stream that writes straight into the peers' buffers over
// xGMI and waits for their tagged flags in its own:
//
//   halo       each block writes its columns of rows 0, 1 into the previous rank's "hi" staging
//              rows and rows ny-2, ny-1 into the next rank's "lo" staging rows; the last block to
//              arrive publishes both flags (release, system scope); every block then waits for
//              the two flags of its own buffer and copies its staging rows into lo / hi.  With
//              two ranks (prev == next) the two directions land in different staging rows, so
//              no posting order matters (the RCCL path needed one, comm.cpp).
//   allreduce  one block writes the rank's values into slot [rank] of every rank's buffer, then
//              a flag per rank; it waits for all flags of its own buffer and combines the slots
//              in rank order (sum, or NaN-propagating max), so every rank computes bitwise the
//              same result.
//
// Tags: each collective kind has its own counter, advanced identically on every rank (all ranks
// issue the same collectives in the same order).  Slots and flags are double-buffered by tag
// parity: a rank can only be one collective ahead of any peer (each collective waits for every
// peer's contribution to the previous one), so parity t & 1 is never overwritten before it was
// read.  A wait is bounded: after NKHIP_PEER_TIMEOUT_S (20 s) of wall-clock time, or once any rank aborted the group (its abort word is
// written into every peer's buffer), the kernel sets the rank's error word (pinned host memory)
// and returns; the host turns that into NK_ECOMM (Engine::sync), so peers blocked in a
// collective with a failed rank return instead of hanging (nkhip.h nk_comm_abort).
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <random>
#include <vector>

#include "../../include/nkhip.h"
#include "comm.h"
#include "nk_device.h"
#include "nk_kernels.h"
#include "peer_dev.h"

namespace nk {
namespace {

// host (optional, pinned): the result is written there too (Engine::reduce_async's host slot)
__global__ void __launch_bounds__(kRedMax) peer_allreduce_kernel(const PeerArgs a, double* dev,
                                                                 double* host, int nsum, int nv) {
  const int t = threadIdx.x;
  const int par = int(a.tag & 1);
  const double v = (t < nv) ? dev[t] : 0.0;
  if (t < nv)
    for (int q = 0; q < a.P; ++q) red_slot(a.base[q], a.P, par, a.rank)[t] = v;
  __threadfence_system();
  __syncthreads();
  if (t < a.P)
    __hip_atomic_store(red_flag(a.base[t], par, a.rank), a.tag, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  __shared__ int ok;
  if (t == 0) ok = 1;
  __syncthreads();
  if (t < a.P && !wait_tag(a, red_flag(a.base[a.rank], par, t))) ok = 0;
  __syncthreads();
  if (!ok) return;
  __threadfence_system();
  if (t < nv) {
    char* mine = a.base[a.rank];
    double acc = red_slot(mine, a.P, par, 0)[t];
    for (int q = 1; q < a.P; ++q) {
      const double x = red_slot(mine, a.P, par, q)[t];
      acc = (t < nsum) ? acc + x : nmax(acc, x);
    }
    dev[t] = acc;
    if (host) host[t] = acc;
  }
}

__global__ void __launch_bounds__(kHaloBlock) peer_halo_kernel(const PeerArgs a, const double* v,
                                                               double* lo, double* hi, int64_t ny,
                                                               int64_t nx) {
  const int par = int(a.tag & 1);
  const int prev = (a.rank - 1 + a.P) % a.P, next = (a.rank + 1) % a.P;
  // a grid of at most kHaloMaxBlocks blocks (peer_dev.h: it must fit the GPU as a whole)
  const int64_t step = int64_t(gridDim.x) * kHaloBlock;
  for (int64_t c = int64_t(blockIdx.x) * kHaloBlock + threadIdx.x; c < nx; c += step) {
    // my first rows are the previous rank's "hi", my last rows the next rank's "lo"
    stage(a.base[prev], a.P, a.max_nx, par, 1, 0)[c] = v[c];
    stage(a.base[prev], a.P, a.max_nx, par, 1, 1)[c] = v[nx + c];
    stage(a.base[next], a.P, a.max_nx, par, 0, 0)[c] = v[(ny - 2) * nx + c];
    stage(a.base[next], a.P, a.max_nx, par, 0, 1)[c] = v[(ny - 1) * nx + c];
  }
  peer_halo_finish(a, nx, lo, hi);
}

// Pushed halo rows (arnoldi.hip): v's rows 0, 1 -> rows 2, 3 of the previous rank's slot, rows
// ny-2, ny-1 -> rows 0, 1 of the next rank's slot, written through (store_sys8) and drained.
// Nothing waits.
__global__ void __launch_bounds__(kHaloBlock) push_rows_kernel(const double* v, double* pp,
                                                              double* pn, int64_t ny, int64_t nx,
                                                              int64_t ld) {
  const int t = blockIdx.y;
  const int64_t row = (t < 2) ? t : ny - 4 + t;
  double* dst = (t < 2) ? pp + (2 + t) * ld : pn + (t - 2) * ld;
  const int64_t step = int64_t(gridDim.x) * kHaloBlock;
  for (int64_t j = int64_t(blockIdx.x) * kHaloBlock + threadIdx.x; j < nx; j += step)
    store_sys8(dst + j, v[row * nx + j]);
  drain_stores();
}

// what a rank publishes about its buffer (nk_comm_peer_handle_bytes bytes)
struct PeerBlob {
  hipIpcMemHandle_t ipc;
  uint64_t ptr;  // the buffer in the owner's address space (used only by the owner itself)
  uint64_t nonce;  // random per process: with the pid, tells "this process" apart across pid
                   // namespaces and hosts
  int32_t pid, bus, dev, domain;
  int64_t bytes;
};

uint64_t process_nonce() {
  static const uint64_t v = [] {
    std::random_device rd;
    uint64_t x = (uint64_t(rd()) << 32) ^ rd();
    return x ? x : 1;
  }();
  return v;
}

uint64_t wait_ticks() { return device_wait_ticks(); }
}  // namespace

double device_wait_seconds() {
  const char* e = std::getenv("NKHIP_PEER_TIMEOUT_S");
  const double s = (e && *e) ? std::atof(e) : 20.0;
  return (s > 0) ? s : 20.0;
}

uint64_t device_wait_ticks() {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0)
    khz = 100000;  // the 100 MHz constant clock of CDNA3/4
  return uint64_t(device_wait_seconds() * 1e3 * double(khz));
}

namespace {

struct PeerComm final : nk_comm {
  int r = 0, p = 1;
  int64_t max_nx = 0;
  char* local = nullptr;  // this rank's exported, fine-grained buffer
  int64_t bytes = 0;
  std::vector<char*> base;
  std::vector<bool> opened;  // base[q] came from hipIpcOpenMemHandle
  uint32_t* counter = nullptr;
  int* err = nullptr;  // pinned host
  hipStream_t side = nullptr;  // abort writes (never queued behind a spinning collective)
  uint64_t red_tag = 0, halo_tag = 0;
  uint64_t ticks = 0;  // wait bound (wait_ticks)
  const void* slot_owner = nullptr;  // the stepper holding the halo slots
  bool connected = false, same_dev = false, any_shared = false, aborted = false;
  PeerBlob blob{};

  ~PeerComm() override {
    for (int q = 0; q < int(base.size()); ++q)
      if (opened[q]) (void)hipIpcCloseMemHandle(base[q]);
    if (local) (void)hipFree(local);
    if (counter) (void)hipFree(counter);
    if (err) (void)hipHostFree(err);
    if (side) (void)hipStreamDestroy(side);
  }
  int rank() const override { return r; }
  int size() const override { return p; }
  bool shares_device() const override { return same_dev; }
  bool group_shares_device() const override { return any_shared; }
  bool failed() const override {
    return aborted || (err && __atomic_load_n(err, __ATOMIC_ACQUIRE) != 0);
  }

  PeerArgs args(uint64_t tag) const {
    PeerArgs a;
    for (int q = 0; q < kMaxPeers; ++q) a.base[q] = q < p ? base[q] : nullptr;
    a.P = p;
    a.rank = r;
    a.max_nx = max_nx;
    a.tag = tag;
    a.counter = counter;
    a.err = err;
    a.wait_ticks = ticks;
    return a;
  }

  int allreduce(double* dev, int nsum, int nv, hipStream_t s) override {
    return allreduce_host(dev, nullptr, nsum, nv, s);
  }
  int allreduce_host(double* dev, double* host, int nsum, int nv, hipStream_t s) override {
    if (!connected || failed()) return NK_ECOMM;
    if (nv <= 0) return NK_OK;
    if (nv > kRedMax) return NK_EINVAL;
    hipLaunchKernelGGL(peer_allreduce_kernel, dim3(1), dim3(kRedMax), 0, s, args(++red_tag), dev,
                       host, nsum, nv);
    return hipGetLastError() == hipSuccess ? NK_OK : NK_EHIP;
  }
  bool allreduce_writes_host() const override { return true; }

  bool take_allreduce(PeerArgs* out, int nv) override {
    if (!connected || failed() || nv < 1 || nv > kRedMax) return false;
    *out = args(++red_tag);
    return true;
  }
  bool claim_slots(const void* owner, nk_halo_slots* out) override {
    if (!connected || !owner || (slot_owner && slot_owner != owner)) return false;
    slot_owner = owner;
    const int prev = (r - 1 + p) % p, next = (r + 1) % p;
    const int64_t off = off_slots(p, max_nx);
    out->mine = reinterpret_cast<double*>(base[r] + off);
    out->prev = reinterpret_cast<double*>(base[prev] + off);
    out->next = reinterpret_cast<double*>(base[next] + off);
    out->ld = max_nx;
    out->count = kHaloSlots;
    return true;
  }
  uint64_t epoch() const override { return red_tag; }
  void release_slots(const void* owner) override {
    if (slot_owner == owner) slot_owner = nullptr;
  }
  bool take_halo(PeerArgs* out, int64_t nx) override {
    if (!connected || failed() || nx > max_nx) return false;
    *out = args(++halo_tag);
    return true;
  }

  int halo(const double* v, double* lo, double* hi, int64_t ny, int64_t nx,
           hipStream_t s) override {
    if (!connected || failed()) return NK_ECOMM;
    if (nx > max_nx || ny < 2) return NK_EINVAL;
    hipLaunchKernelGGL(peer_halo_kernel, dim3(unsigned(halo_blocks(nx))), dim3(kHaloBlock), 0, s,
                       args(++halo_tag), v, lo, hi, ny, nx);
    return hipGetLastError() == hipSuccess ? NK_OK : NK_EHIP;
  }

  int barrier(hipStream_t s) override {
    if (!connected || failed()) return NK_ECOMM;
    double* d = nullptr;
    if (hipMallocAsync(reinterpret_cast<void**>(&d), sizeof(double), s) != hipSuccess)
      return NK_EHIP;
    int rc = hipMemsetAsync(d, 0, sizeof(double), s) == hipSuccess ? allreduce(d, 1, 1, s) : NK_EHIP;
    (void)hipFreeAsync(d, s);
    if (rc) return rc;
    if (hipStreamSynchronize(s) != hipSuccess) return NK_EHIP;
    return failed() ? NK_ECOMM : NK_OK;
  }

  // The group failed: every rank's kernels waiting in a collective leave with the error word
  // set -- this rank's at once, the peers' through the abort word written into their buffers.
  void abort() override {
    if (aborted) return;
    aborted = true;
    if (!side) return;
    static const uint64_t one = 1;
    for (int q = 0; q < int(base.size()); ++q)
      if (base[q])
        (void)hipMemcpyAsync(base[q] + kOffAbort, &one, sizeof(one), hipMemcpyHostToDevice, side);
    (void)hipStreamSynchronize(side);
    (void)hipGetLastError();
  }
};

}  // namespace

hipError_t push_rows_launch(const double* v, double* prev_slot, double* next_slot, int64_t ny,
                            int64_t nx, int64_t ld, hipStream_t s) {
  if (!v || !prev_slot || !next_slot || ny < 4 || nx < 1 || nx > ld) return hipErrorInvalidValue;
  hipLaunchKernelGGL(push_rows_kernel, dim3(unsigned(halo_blocks(nx)), 4), dim3(kHaloBlock), 0, s,
                     v, prev_slot, next_slot, ny, nx, ld);
  return hipGetLastError();
}

bool peer_fuse_enabled() {
  const char* e = std::getenv("NKHIP_PEER_FUSE");
  return !(e && e[0] == '0');
}

bool slab_x_enabled(const nk_comm* c) {
  const char* e = std::getenv("NKHIP_SLAB_XK");
  if (!(e && (e[0] == '1' || e[0] == '2')) || !c || !peer_fuse_enabled()) return false;
  return e[0] == '1' || !c->group_shares_device();
}

int comm_peer_handle_bytes() { return int(sizeof(PeerBlob)); }

int comm_create_peer(nk_comm** out, int rank, int nranks, int64_t max_nx, void* handle_out) {
  if (!out || !handle_out || nranks < 1 || nranks > kMaxPeers || rank < 0 || rank >= nranks ||
      max_nx < 1)
    return NK_EINVAL;
  auto c = std::make_unique<PeerComm>();
  c->r = rank;
  c->p = nranks;
  c->max_nx = max_nx;
  c->bytes = buffer_bytes(nranks, max_nx);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return NK_EHIP;
  if (hipExtMallocWithFlags(reinterpret_cast<void**>(&c->local), size_t(c->bytes),
                            hipDeviceMallocFinegrained) != hipSuccess) {
    c->local = nullptr;
    (void)hipGetLastError();
    return NK_ENOMEM;
  }
  if (hipMemset(c->local, 0, size_t(c->bytes)) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&c->counter), sizeof(uint32_t)) != hipSuccess ||
      hipMemset(c->counter, 0, sizeof(uint32_t)) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&c->err), sizeof(int), hipHostMallocCoherent) !=
          hipSuccess ||
      hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess)
    return NK_EHIP;
  *c->err = 0;
  c->ticks = wait_ticks();
  PeerBlob& b = c->blob;
  std::memset(&b, 0, sizeof(b));
  if (hipIpcGetMemHandle(&b.ipc, c->local) != hipSuccess) {
    (void)hipGetLastError();  // single-process groups do not need it
    std::memset(&b.ipc, 0, sizeof(b.ipc));
  }
  b.ptr = reinterpret_cast<uint64_t>(c->local);
  b.nonce = process_nonce();
  b.pid = int32_t(getpid());
  (void)hipDeviceGetAttribute(&b.bus, hipDeviceAttributePciBusId, dev);
  (void)hipDeviceGetAttribute(&b.dev, hipDeviceAttributePciDeviceId, dev);
  (void)hipDeviceGetAttribute(&b.domain, hipDeviceAttributePciDomainID, dev);
  b.bytes = c->bytes;
  std::memcpy(handle_out, &b, sizeof(b));
  *out = c.release();
  return NK_OK;
}

int comm_peer_connect(nk_comm* comm, const void* handles) {
  auto* c = dynamic_cast<PeerComm*>(comm);
  if (!c || !handles || c->connected) return NK_EINVAL;
  const auto* blobs = static_cast<const PeerBlob*>(handles);
  if (std::memcmp(&blobs[c->r], &c->blob, sizeof(PeerBlob)) != 0) return NK_EINVAL;
  // One process per rank.  Ranks as threads of one process share its GPU_MAX_HW_QUEUES in-order
  // hardware queues, so a collective kernel waiting for a peer rank can sit in a queue ahead of
  // the very launch it waits for: such a group would time out, so it is refused here.
  auto same_process = [](const PeerBlob& x, const PeerBlob& y) {
    return x.pid == y.pid && x.nonce == y.nonce;
  };
  for (int q = 0; q < c->p; ++q)
    if (q != c->r && same_process(blobs[q], c->blob)) {
      std::fprintf(stderr, "nkhip: peer comm ranks %d and %d are one process (one process per "
                           "rank is required)\n", c->r, q);
      return NK_EINVAL;
    }
  c->base.assign(c->p, nullptr);
  c->opened.assign(c->p, false);
  for (int q1 = 0; q1 < c->p; ++q1)  // every rank sees every blob: the same answer everywhere
    for (int q2 = q1 + 1; q2 < c->p; ++q2)
      if (blobs[q1].bus == blobs[q2].bus && blobs[q1].dev == blobs[q2].dev &&
          blobs[q1].domain == blobs[q2].domain)
        c->any_shared = true;
  for (int q = 0; q < c->p; ++q) {
    const PeerBlob& b = blobs[q];
    if (b.bytes != c->bytes) return NK_EINVAL;  // every rank built for the same group shape
    if (q != c->r && b.bus == c->blob.bus && b.dev == c->blob.dev && b.domain == c->blob.domain)
      c->same_dev = true;
    if (q == c->r) {  // the rank itself: its own pointer (other ranks are other processes)
      c->base[q] = c->local;
      continue;
    }
    void* ptr = nullptr;
    if (hipIpcOpenMemHandle(&ptr, b.ipc, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
      std::fprintf(stderr, "nkhip: peer comm rank %d cannot map rank %d's buffer: %s\n", c->r, q,
                   hipGetErrorString(hipGetLastError()));
      return NK_ECOMM;
    }
    c->base[q] = static_cast<char*>(ptr);
    c->opened[q] = true;
  }
  c->connected = true;
  return NK_OK;
}

}  // namespace nk

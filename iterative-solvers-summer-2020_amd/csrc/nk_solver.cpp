// Host-side inexact Newton / LGMRES driver (see nk_solver.h).
//
// Algorithm follows SciPy 1.15.3 line by line where it is observable:
//   nonlin_solve ............ scipy/optimize/_nonlin.py:122-268
//   _nonlin_line_search ..... scipy/optimize/_nonlin.py:272-314
//   scalar_search_armijo .... scipy/optimize/_linesearch.py:684-739
//   TerminationCondition .... scipy/optimize/_nonlin.py:317-375
//   KrylovJacobian .......... scipy/optimize/_nonlin.py:1453-1540
//   lgmres (maxiter=1) ...... scipy/sparse/linalg/_isolve/lgmres.py:120-230
//   _fgmres ................. scipy/sparse/linalg/_isolve/_gcrotmk.py:14-180
// The C++ twin's solver (`nonlin_solve`, `KrylovJacobian`, `lgmres`, `scalar_search_armijo`,
// `maxnorm` from newton_krylov.obj) is the same algorithm.
#include "nk_solver.h"

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>

namespace nk {

namespace {
constexpr double kEps = DBL_EPSILON;
constexpr int kReduceSlots = Engine::kSlots;
}  // namespace

const char* kind_name(int kind) {
  static const char* names[K_NKINDS] = {"sh_fdjvp", "sh_ajvp", "sh_trial", "sh_bold",
                                         "krylov_mdot", "krylov_combo", "reduce_final", "copy",
                                         "halo", "user_F", "axpby", "arnoldi_fused",
                                         "arnoldi_edge", "edge_gather", "arnoldi_slab_edges",
                                         "arnoldi_ctl", "halo_push"};
  return (kind >= 0 && kind < K_NKINDS) ? names[kind] : "?";
}

void log_launch(int kind, double bytes) {
  static std::FILE* f = [] {
    const char* p = std::getenv("NKHIP_LAUNCH_LOG");
    return (p && *p) ? std::fopen(p, "w") : nullptr;
  }();
  if (!f) return;
  static std::mutex mu;
  std::lock_guard<std::mutex> lk(mu);
  std::fprintf(f, "%s %.0f\n", kind_name(kind), bytes);
  std::fflush(f);
}

nk_opts default_opts() {
  nk_opts o;
  o.f_tol = NAN;
  o.f_rtol = NAN;
  o.x_tol = NAN;
  o.x_rtol = NAN;
  o.rdiff = 0.0;
  o.maxiter = 0;
  o.inner_m = 30;
  o.outer_k = 10;
  o.line_search = 1;
  o.jvp_mode = NK_JVP_FD;
  o.verbose = 0;
  o.profile = 0;
  return o;
}

// ============================================================================================
// Engine
// ============================================================================================
Engine::Engine(int64_t n_, nk_comm* comm_, hipStream_t s_, bool profile_, int64_t min_partial)
    : n(n_), npad(pad(n_)), comm(comm_), s(s_), profile(profile_) {
  // partial-sum slots: the larger of the Krylov multi-dot and the problem's stencil reductions
  const int64_t kb = krylov_blocks(npad) + 1;
  // (at least 64 Ki slots: the fused Arnoldi kernel writes (2 nv + 3) values per wave)
  const int64_t cap = std::max<int64_t>(std::max<int64_t>((2 * kMaxVec + 1) * kb, min_partial), 1 << 16);
  if (hipMalloc(reinterpret_cast<void**>(&partial_), sizeof(double) * cap) != hipSuccess)
    partial_ = nullptr;
  else
    partial_cap_ = cap;
  if (hipMalloc(reinterpret_cast<void**>(&dres_), sizeof(double) * kReduceSlots) != hipSuccess)
    dres_ = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(&hres_), sizeof(double) * kReduceSlots, 0) !=
      hipSuccess)
    hres_ = nullptr;
  bytes_ = sizeof(double) * (cap + kReduceSlots);
}

Engine::~Engine() {
  if (s) hipStreamSynchronize(s);
  for (auto& p : pend_) {
    hipEventDestroy(p.a);
    hipEventDestroy(p.b);
  }
  for (auto e : free_ev_) hipEventDestroy(e);
  if (vmm_base_) {
    vmm_free();  // the pool and its edge arrays
  } else {
    if (own_pool_ && pool_) hipFree(pool_);
    if (epool_) hipFree(epool_);
  }
  if (partial_) hipFree(partial_);
  if (dres_) hipFree(dres_);
  if (hres_) hipHostFree(hres_);
}

// The pool as `chunk`-sized physical allocations mapped back to back into a chunk-aligned
// virtual range (hipMemCreate / hipMemMap): virtual and physical addresses then agree modulo the
// chunk, so the page tables may use fragments up to the chunk size.
int Engine::vmm_alloc(size_t bytes, size_t chunk) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return NK_EHIP;
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = dev;
  size_t gran = 0;
  if (hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended) !=
          hipSuccess || gran == 0)
    return NK_EHIP;
  chunk = (chunk + gran - 1) / gran * gran;
  const size_t total = (bytes + chunk - 1) / chunk * chunk;
  if (hipMemAddressReserve(&vmm_base_, total, chunk, nullptr, 0) != hipSuccess) {
    vmm_base_ = nullptr;
    return NK_ENOMEM;
  }
  vmm_size_ = total;
  vmm_chunk_ = chunk;
  for (size_t off = 0; off < total; off += chunk) {
    hipMemGenericAllocationHandle_t h;
    if (hipMemCreate(&h, chunk, &prop, 0) != hipSuccess) {
      vmm_free();
      return NK_ENOMEM;
    }
    vmm_h_.push_back(h);
    if (hipMemMap(static_cast<char*>(vmm_base_) + off, chunk, 0, h, 0) != hipSuccess) {
      vmm_free();
      return NK_EHIP;
    }
  }
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  if (hipMemSetAccess(vmm_base_, total, &acc, 1) != hipSuccess) {
    vmm_free();
    return NK_EHIP;
  }
  return NK_OK;
}

void Engine::vmm_free() {
  if (!vmm_base_) return;
  for (size_t i = 0; i < vmm_h_.size(); ++i) {
    hipMemUnmap(static_cast<char*>(vmm_base_) + i * vmm_chunk_, vmm_chunk_);
    hipMemRelease(vmm_h_[i]);
  }
  vmm_h_.clear();
  hipMemAddressFree(vmm_base_, vmm_size_);
  vmm_base_ = nullptr;
  (void)hipGetLastError();
}

int Engine::alloc(int count, std::vector<double*>* out, void* external, int64_t external_bytes) {
  if (!partial_ || !dres_ || !hres_) return NK_ENOMEM;
  const int64_t bytes = sizeof(double) * npad * int64_t(count);
  const bool edges = edge_ny_ > 0 && edge_nx_ > 0;
  edge_n_ = edges ? edge_elems(edge_ny_, edge_nx_) : 0;
  const int64_t eb = (sizeof(double) * edge_n_ * count + 255) / 256 * 256;
  if (external) {
    if (external_bytes < bytes || (reinterpret_cast<uintptr_t>(external) & 255u)) return NK_EINVAL;
    pool_ = static_cast<double*>(external);
    own_pool_ = false;
  } else {
    // Large pools are mapped through the virtual memory API in 1-GB (64-MB) chunks rather than
    // taken from hipMalloc: the streaming kernels ran up to 5 % apart on hipMalloc pools that
    // differed only in where they landed (one process, several steppers, each stable over
    // rounds: fused kernel 0.632-0.640 on three pools in four, 0.66-0.675 on the fourth), and
    // 0.667-0.683 on every chunk-mapped pool (scripts/dbg/pool_placement.py, profiles/
    // r03_pool_placement.md) -- consistent with page-table fragments limited by how the
    // hipMalloc range's virtual and physical alignments happen to match, which the chunk-aligned
    // mapping fixes.  The edge arrays share the mapping.  NKHIP_POOL_ALLOC=malloc: hipMalloc.
    const char* how = std::getenv("NKHIP_POOL_ALLOC");
    const bool vmm = !(how && std::strcmp(how, "malloc") == 0) && bytes + eb >= (int64_t(1) << 28);
    int rc = NK_ENOMEM;
    if (vmm) {
      const size_t chunk = size_t(1) << ((bytes + eb >= (int64_t(1) << 33)) ? 30 : 26);
      rc = vmm_alloc(size_t(bytes + eb), chunk);
      if (rc == NK_OK) {
        pool_ = static_cast<double*>(vmm_base_);
        if (edges) epool_ = pool_ + bytes / int64_t(sizeof(double));
      }
    }
    if (rc != NK_OK) {  // small pools, or the mapping failed: plain allocations
      (void)hipGetLastError();
      if (hipMalloc(reinterpret_cast<void**>(&pool_), bytes) != hipSuccess) {
        pool_ = nullptr;
        return NK_ENOMEM;
      }
      if (edges && hipMalloc(reinterpret_cast<void**>(&epool_), eb) != hipSuccess) {
        epool_ = nullptr;
        return NK_ENOMEM;
      }
    }
    own_pool_ = true;
    bytes_ += bytes + (edges ? eb : 0);
  }
  if (external && edges) {
    if (hipMalloc(reinterpret_cast<void**>(&epool_), eb) != hipSuccess) {
      epool_ = nullptr;
      return NK_ENOMEM;
    }
    bytes_ += eb;
  }
  if (hipMemsetAsync(pool_, 0, bytes, s) != hipSuccess) return NK_EHIP;
  if (epool_ && hipMemsetAsync(epool_, 0, eb, s) != hipSuccess) return NK_EHIP;
  if (std::getenv("NKHIP_DEBUG_POOL"))
    std::fprintf(stderr, "nkhip pool %p (%lld vectors of %lld B, %s)\n", static_cast<void*>(pool_),
                 static_cast<long long>(count), static_cast<long long>(sizeof(double) * npad),
                 vmm_base_ ? "chunk-mapped" : (external ? "external" : "hipMalloc"));
  out->resize(count);
  for (int i = 0; i < count; ++i) (*out)[i] = pool_ + npad * i;
  pool_count_ = count;
  return NK_OK;
}

int64_t Engine::pool_index(const double* v) const {
  if (!pool_ || !v || v < pool_) return -1;
  const int64_t off = v - pool_;
  if (off % npad != 0 || off / npad >= pool_count_) return -1;
  return off / npad;
}

void Engine::mark_edges(const double* v) {
  const int64_t q = pool_index(v);
  if (q < 0 || !epool_) return;
  if (ekept_.size() < size_t(pool_count_)) ekept_.assign(pool_count_, 0);
  ekept_[q] = 1;
}

bool Engine::edges_kept(const double* v) const {
  const int64_t q = pool_index(v);
  return q >= 0 && size_t(q) < ekept_.size() && ekept_[q] != 0;
}

double* Engine::edges(const double* v) const {
  if (!epool_ || !v || v < pool_) return nullptr;
  const int64_t off = v - pool_;
  if (off % npad != 0 || off / npad >= pool_count_) return nullptr;
  return epool_ + edge_n_ * (off / npad);
}

int Engine::gather_edges(const double* v) {
  double* e = edges(v);
  if (!e) return NK_OK;
  mark_edges(v);
  return launch(K_EDGE, 8.0 * edge_n_ * 2,
                [&] { return edge_gather_launch(v, e, edge_ny_, edge_nx_, s); });
}

EdgeOut Engine::edge_out(const double* v) {
  EdgeOut eo;
  eo.E = edges(v);
  if (!eo.E) return eo;
  mark_edges(v);
  eo.nx = edge_nx_;
  eo.ny = edge_ny_;
  return eo;
}

hipEvent_t Engine::ev() {
  if (!free_ev_.empty()) {
    hipEvent_t e = free_ev_.back();
    free_ev_.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  hipEventCreate(&e);
  return e;
}

void Engine::harvest() {
  for (auto& p : pend_) {
    float ms = 0.f;
    hipEventElapsedTime(&ms, p.a, p.b);
    stats_[p.kind].timed += 1;
    stats_[p.kind].ms += ms;
    stats_[p.kind].tbytes += p.bytes;
    free_ev_.push_back(p.a);
    free_ev_.push_back(p.b);
  }
  pend_.clear();
}

void Engine::void_last(int kind, int count) {
  if (kind < 0 || kind >= K_NKINDS) return;
  for (int c = 0; c < count && c < kRecent && stats_[kind].launches > 0; ++c) {
    const int64_t idx = stats_[kind].launches - 1;
    stats_[kind].launches = idx;
    stats_[kind].bytes -= recent_bytes_[kind][idx % kRecent];
    for (size_t i = 0; i < pend_.size(); ++i) {
      if (pend_[i].kind == kind && pend_[i].idx == idx) {
        free_ev_.push_back(pend_[i].a);
        free_ev_.push_back(pend_[i].b);
        pend_.erase(pend_.begin() + i);
        break;
      }
    }
  }
}

void Engine::reset_stats() {
  for (auto& k : stats_) k = KStat{};
  for (auto& t : tick_) t = 0;
}

int Engine::sync() {
  if (hipStreamSynchronize(s) != hipSuccess) return NK_EHIP;
  harvest();
  // a collective the stream ran may have failed on the device (peer.hip: timeout / abort)
  return (comm && comm->failed()) ? NK_ECOMM : NK_OK;
}

int Engine::copy(double* dst, const double* src, int64_t cnt) {
  if (dst == src) return NK_OK;
  // large copies as a streaming kernel (out = 1.0 x, exact): the runtime's blit moves a 4096^2
  // field at ~0.9 TB/s, the element-wise kernel at HBM speed
  return launch(K_COPY, 16.0 * cnt, [&] {
    if (cnt >= (int64_t(1) << 16)) return axpby_launch(1.0, src, 0.0, nullptr, dst, cnt, s);
    return hipMemcpyAsync(dst, src, sizeof(double) * cnt, hipMemcpyDeviceToDevice, s);
  });
}

namespace {
// a signalling-NaN bit pattern no reduction of finite or NaN data writes (NaNs a reduction
// propagates are quiet): marks a pinned result slot as not yet written
constexpr uint64_t kUnset = 0x7FF0DEADBEEF0001ull;
bool poll_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("NKHIP_POLL");
    return !(e && e[0] == '0');
  }();
  return on;
}
}  // namespace

int Engine::wait_results(int slot, int nv) {
  // the slots are written by a kernel (one GPU: the reduction; peer-memory slabs: the all-reduce)
  // unless the communicator's result comes back by a runtime copy
  if ((comm && !comm->allreduce_writes_host()) || !poll_enabled()) return sync();
  volatile uint64_t* h = reinterpret_cast<volatile uint64_t*>(hres_ + slot);
  for (int k = 0; k < nv; ++k) {
    for (int64_t spins = 0; h[k] == kUnset; ++spins) {
      if (spins > (int64_t(1) << 26)) return sync();  // not arriving: take the slow path
      __builtin_ia32_pause();
    }
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  return NK_OK;
}

uint32_t Engine::wait_flag(const uint32_t* flag) {
  const volatile uint32_t* f = flag;
  for (int64_t spins = 0; *f == 0; ++spins) {
    if (spins > (int64_t(1) << 26)) {  // not arriving: drain the stream, then look once more
      if (sync() != NK_OK) return 0;
      break;
    }
    __builtin_ia32_pause();
  }
  const uint32_t v = *f;
  std::atomic_thread_fence(std::memory_order_acquire);
  return v;
}

int Engine::reduce_async(int64_t nblk, int nsum, int nv, int slot, bool host_copy) {
  if (slot < 0 || slot + nv > kReduceSlots) return NK_EINVAL;
  // any communicator (also a world of one) takes the all-reduce path
  const bool multi = comm != nullptr;
  // a kernel fills these pinned slots (the reduction on one GPU, the peer all-reduce on slabs);
  // wait_results() polls for them
  if (!multi || (host_copy && comm->allreduce_writes_host())) {
    uint64_t* h = reinterpret_cast<uint64_t*>(hres_ + slot);
    for (int k = 0; k < nv; ++k) h[k] = kUnset;
    std::atomic_thread_fence(std::memory_order_release);
  }
  int rc = launch(K_REDUCE, 8.0 * nblk * nv, [&] {
    return reduce_final_launch(partial_, nblk, nsum, nv, dres_ + slot,
                               multi ? nullptr : hres_ + slot, s);
  });
  if (rc || !multi) return rc;
  if (!host_copy) return comm->allreduce(dres_ + slot, nsum, nv, s);
  return comm->allreduce_host(dres_ + slot, hres_ + slot, nsum, nv, s);
}

int Engine::reduce(int64_t nblk, int nsum, int nv, double* out) {
  int rc = reduce_async(nblk, nsum, nv, kSlotSync);
  if (!rc) rc = sync();
  if (rc) return rc;
  std::memcpy(out, hres_ + kSlotSync, sizeof(double) * nv);
  return NK_OK;
}

// ============================================================================================
// Newton-Krylov core
// ============================================================================================
namespace detail {

void givens(double a, double b, double* c, double* s) {
  if (b == 0.0) {
    *c = 1.0;
    *s = 0.0;
    return;
  }
  const double r = std::hypot(a, b);
  *c = a / r;
  *s = b / r;
}

// Least-squares solve of the (n x n) upper-triangular R y = g (lstsq in _gcrotmk.py:177):
// back-substitution when R is well conditioned on its diagonal, otherwise a one-sided Jacobi
// SVD pseudo-inverse with gelsd's cut-off rcond = eps * n.
void lstsq_upper(const double (*R)[kMaxVec + 1], int n, const double* g, double* y) {
  double dmax = 0.0, dmin = INFINITY;
  for (int i = 0; i < n; ++i) {
    dmax = std::max(dmax, std::fabs(R[i][i]));
    dmin = std::min(dmin, std::fabs(R[i][i]));
  }
  if (n > 0 && dmin > kEps * n * dmax) {
    for (int i = n - 1; i >= 0; --i) {
      double acc = g[i];
      for (int k = i + 1; k < n; ++k) acc -= R[i][k] * y[k];
      y[i] = acc / R[i][i];
    }
    return;
  }
  // A = R (n x n), one-sided Jacobi: A V = U S
  std::vector<double> A(n * n), Vm(n * n, 0.0);
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < n; ++k) A[i * n + k] = (k >= i) ? R[i][k] : 0.0;
  for (int i = 0; i < n; ++i) Vm[i * n + i] = 1.0;
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0.0;
    for (int p = 0; p < n - 1; ++p)
      for (int q = p + 1; q < n; ++q) {
        double a = 0, b = 0, c = 0;
        for (int i = 0; i < n; ++i) {
          a += A[i * n + p] * A[i * n + p];
          b += A[i * n + q] * A[i * n + q];
          c += A[i * n + p] * A[i * n + q];
        }
        if (c == 0.0) continue;
        off = std::max(off, std::fabs(c) / std::sqrt(a * b + 1e-300));
        const double zeta = (b - a) / (2.0 * c);
        const double t = std::copysign(1.0, zeta) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
        const double cs = 1.0 / std::sqrt(1.0 + t * t), sn = cs * t;
        for (int i = 0; i < n; ++i) {
          const double ap = A[i * n + p], aq = A[i * n + q];
          A[i * n + p] = cs * ap - sn * aq;
          A[i * n + q] = sn * ap + cs * aq;
          const double vp = Vm[i * n + p], vq = Vm[i * n + q];
          Vm[i * n + p] = cs * vp - sn * vq;
          Vm[i * n + q] = sn * vp + cs * vq;
        }
      }
    if (off < 1e-15) break;
  }
  std::vector<double> sig(n);
  double smax = 0.0;
  for (int k = 0; k < n; ++k) {
    double acc = 0;
    for (int i = 0; i < n; ++i) acc += A[i * n + k] * A[i * n + k];
    sig[k] = std::sqrt(acc);
    smax = std::max(smax, sig[k]);
  }
  const double cut = kEps * n * smax;
  for (int i = 0; i < n; ++i) y[i] = 0.0;
  for (int k = 0; k < n; ++k) {
    if (!(sig[k] > cut)) continue;
    double ug = 0.0;  // u_k . g with u_k = A[:,k] / sig_k
    for (int i = 0; i < n; ++i) ug += A[i * n + k] * g[i];
    ug /= sig[k] * sig[k];
    for (int i = 0; i < n; ++i) y[i] += Vm[i * n + k] * ug;
  }
}

}  // namespace detail

NewtonKrylov::NewtonKrylov(Engine& E, Problem& P, const nk_opts& o, void* external,
                           int64_t external_bytes)
    : E_(E), P_(P), o_(o) {
  if (o.inner_m < 1 || o.outer_k < 0 || o.inner_m + o.outer_k + 1 > kMaxVec) {
    init_status_ = NK_EINVAL;
    return;
  }
  std::vector<double*> v;
  init_status_ = E_.alloc(vectors_needed(o), &v, external, external_bytes);
  if (init_status_) return;
  int q = 0;
  X_ = v[q++];
  Xt_ = v[q++];
  Fx_ = v[q++];
  Ft_ = v[q++];
  G0_ = v[q++];
  Gt_ = v[q++];
  Sv_ = v[q++];
  const int nv = o.inner_m + o.outer_k + 1;
  V_.assign(nv, nullptr);
  for (int i = 1; i < nv; ++i) V_[i] = v[q++];
  outer_.assign(std::max(o.outer_k, 1), nullptr);
  for (int i = 0; i < std::max(o.outer_k, 1); ++i) outer_[i] = v[q++];
  osig_.assign(outer_.size(), 0.0);
  orn_.assign(outer_.size(), 0.0);
  // the Arnoldi loop state (pinned: uploaded to / read back from dS_ by DMA) and the device side
  // of its control
  if (hipHostMalloc(reinterpret_cast<void**>(&hS_), sizeof(ArnCtlState), 0) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&status_), sizeof(uint32_t) * (kMaxVec + 2), 0) !=
          hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&dS_), sizeof(ArnCtlState)) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&prm_), sizeof(double) * kCtlPrm) != hipSuccess) {
    init_status_ = NK_ENOMEM;
    return;
  }
  std::memset(hS_, 0, sizeof(ArnCtlState));
}

NewtonKrylov::~NewtonKrylov() {
  if (E_.s) hipStreamSynchronize(E_.s);
  if (hS_) hipHostFree(hS_);
  if (status_) hipHostFree(status_);
  if (dS_) hipFree(dS_);
  if (prm_) hipFree(prm_);
}

// NewtonKrylov::lgmres lives in lgmres.cpp

int NewtonKrylov::line_search(double* s_out, double* fnorm_new, double* fmax, double* xmax) {
  // _nonlin_line_search(search_type='armijo', smin=1e-2) + scalar_search_armijo(c1=1e-4)
  double tmp_s = 0.0, tmp_phi = fx_norm_ * fx_norm_;
  double tmp_fmax = 0.0, tmp_xmax = 0.0, tmp_sum = tmp_phi;
  int rc = NK_OK;
  auto phi = [&](double s) -> double {
    if (s == tmp_s) return tmp_phi;
    double red[3];
    rc = P_.eval(X_, d_, -s, Xt_, Ft_, Gt_, red);
    st_->nfev += 1;
    const double p = std::isfinite(red[0]) ? red[0] : INFINITY;
    tmp_s = s;
    tmp_phi = p;
    tmp_sum = red[0];
    tmp_fmax = std::isfinite(red[0]) ? red[1] : NAN;
    tmp_xmax = red[2];
    return p;
  };
  double s = 1.0;
  bool found = true;
  if (o_.line_search) {
    const double phi0 = tmp_phi, derphi0 = -tmp_phi, c1 = 1e-4, amin = 1e-2;
    double alpha0 = 1.0;
    // The next LGMRES call's first JVP (J applied to its first augmentation vector at the trial
    // point, _gcrotmk.py:107-110 with prepend_outer_v) is queued behind this s = 1 trial, before
    // the host reads the trial's reduction: the pass runs on the device only if the full step
    // passes this Armijo test and the iteration goes on (the usual outcome), with the FD step
    // the host would compute from the same values (StencilArgs::spec).  The GPU then does not
    // idle through the host's round trip before that JVP.
    const double thr = phi0 + c1 * alpha0 * derphi0;
    const int K = int(outer_.size());
    spec_.valid = false;
    Problem::SpecJvp sp{};
    const bool arm = P_.can_spec_jvp() && ocount_ > 0 && K > 0 && V_.size() > 1;
    if (arm) {
      const int slot = ohead_ % K;
      sp = Problem::SpecJvp{outer_[slot], osig_[slot], osig_[slot] * orn_[slot], thr, f_tol_,
                            rdiff_, V_[1]};
      if (sp.zn != 0.0) P_.arm_spec(&sp);
    }
    double phi_a0 = phi(alpha0);
    P_.arm_spec(nullptr);
    if (rc) return rc;
    if (arm && sp.zn != 0.0) {  // what the pass decided, from the same values
      const bool ran = std::isfinite(tmp_sum) && tmp_sum <= thr && !(tmp_fmax <= f_tol_);
      if (ran) {
        spec_.valid = true;
        spec_.z = sp.z;
        spec_.zs = sp.zs;
        spec_.zn = sp.zn;
        spec_.w = sp.w;
        spec_.x = Xt_;  // the trial this eval wrote (phi(1.0): Xt_, Gt_)
        spec_.g = Gt_;
      } else {
        E_.void_last(K_FDJVP, 1);  // a launch that did nothing
      }
    }
    if (phi_a0 <= phi0 + c1 * alpha0 * derphi0) {
      s = alpha0;
    } else {
      double alpha1 = -(derphi0)*alpha0 * alpha0 / 2.0 / (phi_a0 - phi0 - derphi0 * alpha0);
      double phi_a1 = phi(alpha1);
      if (rc) return rc;
      if (phi_a1 <= phi0 + c1 * alpha1 * derphi0) {
        s = alpha1;
      } else {
        found = false;
        while (alpha1 > amin) {
          const double factor = alpha0 * alpha0 * alpha1 * alpha1 * (alpha1 - alpha0);
          double a = alpha0 * alpha0 * (phi_a1 - phi0 - derphi0 * alpha1) -
                     alpha1 * alpha1 * (phi_a0 - phi0 - derphi0 * alpha0);
          a = a / factor;
          double b = -alpha0 * alpha0 * alpha0 * (phi_a1 - phi0 - derphi0 * alpha1) +
                     alpha1 * alpha1 * alpha1 * (phi_a0 - phi0 - derphi0 * alpha0);
          b = b / factor;
          double alpha2 = (-b + std::sqrt(std::fabs(b * b - 3 * a * derphi0))) / (3.0 * a);
          const double phi_a2 = phi(alpha2);
          if (rc) return rc;
          if (phi_a2 <= phi0 + c1 * alpha2 * derphi0) {
            s = alpha2;
            found = true;
            break;
          }
          if ((alpha1 - alpha2) > alpha1 / 2.0 || (1 - alpha2 / alpha1) < 0.96) alpha2 = alpha1 / 2.0;
          alpha0 = alpha1;
          alpha1 = alpha2;
          phi_a0 = phi_a1;
          phi_a1 = phi_a2;
        }
        if (!found) s = 1.0;  // "take the full Newton step and hope for the best"
      }
    }
    if (s != tmp_s) phi(s);  // Fx = func(x) at the accepted step
    if (rc) return rc;
  } else {
    phi(1.0);
    if (rc) return rc;
  }
  *s_out = s;
  *fnorm_new = std::sqrt(tmp_sum);
  *fmax = tmp_fmax;
  *xmax = tmp_xmax;
  return NK_OK;
}

int NewtonKrylov::solve(const double* x_in, double* x_out, nk_stats* st) {
  if (init_status_) return init_status_;
  nk_stats dummy;
  st_ = st ? st : &dummy;
  std::memset(st_, 0, sizeof(nk_stats));
  st_->step_min = 1.0;
  steps_.clear();
  ocount_ = 0;
  ohead_ = 0;
  const int64_t n = E_.n;
  const double f_tol = std::isnan(o_.f_tol) ? std::pow(kEps, 1.0 / 3.0) : o_.f_tol;
  f_tol_ = f_tol;
  spec_.valid = false;
  const double f_rtol = std::isnan(o_.f_rtol) ? INFINITY : o_.f_rtol;
  const double x_tol = std::isnan(o_.x_tol) ? INFINITY : o_.x_tol;
  const double x_rtol = std::isnan(o_.x_rtol) ? INFINITY : o_.x_rtol;
  rdiff_ = (o_.rdiff > 0) ? o_.rdiff : std::pow(kEps, 0.5);
  const int64_t maxiter = (o_.maxiter > 0) ? o_.maxiter : 100 * (P_.n_global() + 1);
  const bool talk = o_.verbose && (!E_.comm || E_.comm->rank() == 0);

  // the initial evaluation reads x_in and writes the iterate's pool copy X_ = x_in + 0 x_in as
  // its trial output (no separate copy pass)
  int rc = P_.set_x0(x_in);
  double red[3];
  if (!rc) rc = P_.eval(x_in, x_in, 0.0, X_, Fx_, G0_, red);  // (Fx_ = V_0: edges written)
  if (rc) return rc;
  st_->nfev = 1;
  fx_norm_ = std::sqrt(red[0]);
  double fmax = std::isfinite(red[0]) ? red[1] : NAN;
  double xmax = red[2];
  // KrylovJacobian.setup / _update_diff_step
  omega_ = rdiff_ * std::max(1.0, xmax) / std::max(1.0, fmax);
  const double gamma = 0.9, eta_max = 0.9999, eta_treshold = 0.1;
  double eta = 1e-3;
  double dxmax = INFINITY;
  double f0_norm = NAN;
  bool converged = false;
  int64_t it = 0;
  for (it = 0; it < maxiter; ++it) {
    // TerminationCondition.check (max-norm)
    const double f_norm = fmax;
    if (std::isnan(f0_norm)) f0_norm = f_norm;
    if (f_norm == 0.0 || ((f_norm <= f_tol && f_norm / f_rtol <= f0_norm) &&
                          (dxmax <= x_tol && dxmax / x_rtol <= xmax))) {
      converged = true;
      break;
    }
    const double tol = std::min(eta, eta * fx_norm_);
    double dnorm = 0.0, dmx = 0.0;
    rc = lgmres(tol, &dnorm, &dmx, &d_);
    if (rc) break;
    if (!(dnorm != 0.0) || d_ == nullptr) {
      rc = NK_ZERO_STEP;
      break;
    }
    dxmax = dmx;
    rc = P_.set_dir(d_);
    if (rc) break;
    double s = 1.0, fnorm_new = 0.0;
    rc = line_search(&s, &fnorm_new, &fmax, &xmax);
    if (rc) break;
    if (s != 1.0) st_->n_backtrack += 1;
    st_->step_min = std::min(st_->step_min, s);
    steps_.push_back(s);
    std::swap(X_, Xt_);
    std::swap(Fx_, Ft_);
    std::swap(G0_, Gt_);
    rc = P_.set_x0(X_);  // (Fx_, the accepted trial's F, came with its edge array)
    if (rc) break;
    omega_ = rdiff_ * std::max(1.0, xmax) / std::max(1.0, fmax);  // jacobian.update
    const double eta_A = gamma * fnorm_new * fnorm_new / (fx_norm_ * fx_norm_);
    if (gamma * eta * eta < eta_treshold)
      eta = std::min(eta_max, eta_A);
    else
      eta = std::min(eta_max, std::max(eta_A, gamma * eta * eta));
    fx_norm_ = fnorm_new;
    if (talk) {
      std::printf("%lld:  |F(x)| = %g; step %g\n", static_cast<long long>(it), fmax, s);
      std::fflush(stdout);
    }
  }
  st_->nit = it;
  st_->fnorm_inf = fmax;
  st_->fnorm_2 = fx_norm_;
  if (rc) {
    st_->status = rc;
    return rc;
  }
  rc = E_.copy(x_out, X_, n);
  if (!rc) rc = E_.sync();
  if (rc) return rc;
  st_->status = converged ? NK_OK : NK_NO_CONVERGENCE;
  return st_->status;
}

}  // namespace nk

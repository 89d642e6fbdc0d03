// Host-side inexact Newton / LGMRES driver of libnkhip.
//
// A C++ restatement of SciPy 1.15.3's newton_krylov stack as the reference calls it
// (sh_scipy_nk.py:61 `newton_krylov(residual, Uo)`; the C++ twin's external `nonlin_solve`,
// main.cpp:104), re-designed for one GPU stream per rank:
//   * every N^2-sized vector lives in HBM; the host only holds scalars and the <= 64x64
//     Hessenberg factorisation;
//   * per Arnoldi step: one JVP kernel, one fused multi-dot (V^T w, new Gram row incl. the
//     previous vector's |v|^2, |w|^2), one update (w - V h) -- the MGS coefficients are recovered
//     from the Gram row (inverse compact-WY MGS), which equals scipy's MGS in exact arithmetic;
//     the norm of the new vector arrives with the next multi-dot (lgmres.cpp), so a step costs
//     one reduction and one host synchronisation;
//   * basis vectors are kept un-normalised with a host-side scale (no scal pass).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/nkhip.h"
#include "comm.h"
#include "nk_kernels.h"

namespace nk {

enum Kind : int {
  K_FDJVP = 0,
  K_AJVP,
  K_TRIAL,
  K_BOLD,
  K_MDOT,
  K_COMBO,
  K_REDUCE,
  K_COPY,
  K_HALO,
  K_USERF,
  K_AXPBY,
  K_ARNOLDI,
  K_ARN_EDGE,
  K_EDGE,
  K_ARN_SLAB,
  K_CTL,
  K_PUSH,  // pushed halo rows of a producer (peer-memory slabs)
  K_NKINDS
};

// Short class name of a launch kind (the names nk_sh_kernel_profile reports).
const char* kind_name(int kind);
// NKHIP_LAUNCH_LOG=<path>: every Engine launch appends "<class> <algorithmic bytes>" to <path>,
// in launch order, so a profiler's per-dispatch counters can be matched to the solver's
// algorithmic bytes one dispatch at a time (scripts/traffic_match.py).
void log_launch(int kind, double bytes);

struct KStat {
  int64_t launches = 0;  // all launches of the class
  double bytes = 0.0;    // algorithmic bytes of all launches
  int64_t timed = 0;     // launches timed with HIP events (every `sample`-th one)
  double ms = 0.0;       // their summed duration
  double tbytes = 0.0;   // their algorithmic bytes
};

// Device workspace, reductions and per-kernel profiling for one rank's solver.
class Engine {
 public:
  // min_partial: partial-sum slots any kernel of the problem needs beyond the Krylov ones.
  Engine(int64_t n, nk_comm* comm, hipStream_t s, bool profile, int64_t min_partial = 0);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  // Allocate `count` zeroed vectors of npad doubles from one pool (or carve from `external`).
  // With enable_edges() called first, every pool vector also gets an edge array (edges()).
  // Pools of >= 256 MB are mapped in chunks through the virtual memory API (vmm_alloc).
  int alloc(int count, std::vector<double*>* out, void* external = nullptr,
            int64_t external_bytes = 0);
  bool pool_chunk_mapped() const { return vmm_base_ != nullptr; }
  // Edge arrays (nk_kernels.h, kEdgeW) of an ny x nx grid for the pool vectors.
  void enable_edges(int64_t ny, int64_t nx) {
    edge_ny_ = ny;
    edge_nx_ = nx;
  }
  // The edge array of pool vector v (nullptr when v is not a pool vector or edges are off).
  double* edges(const double* v) const;
  // index of pool vector v in the workspace pool (-1: not a pool vector); vectors in the pool
  int64_t pool_index(const double* v) const;
  int pool_count() const { return pool_count_; }
  // v's edge array is maintained: every kernel that writes v also writes its edge array (the
  // stencil passes' outputs, the fused kernel's, vectors refreshed by gather_edges); only those
  // may be read in place of a stencil field's side columns.  (The LGMRES augmentation vectors
  // are written by combinations only and are never marked.)
  void mark_edges(const double* v);
  bool edges_kept(const double* v) const;
  // Refresh the edge array of pool vector v from v (no-op without one).
  int gather_edges(const double* v);
  // The edge array a combination writing pool vector v fills in place of gather_edges (marked
  // kept; E == nullptr when v has none).
  EdgeOut edge_out(const double* v);
  // Vector stride in the pool.  Large vectors get an odd multiple of 128 KiB: consecutive basis
  // vectors read at the same offset then spread over the HBM channels instead of landing on the
  // same ones (scripts/micro/march_bench.hip, 24 vectors of 4096^2 streamed row by row: pool
  // stride 2^27 B 5.2-5.6 TB/s, 2^27 + 2^17 B 6.4-6.5 TB/s; contiguous chunks 6.0 -> 6.6 TB/s).
  static int64_t pad(int64_t n) {
    const int64_t p = (n + 255) / 256 * 256;
    if (p < (int64_t(1) << 16)) return p;
    return (p + 32767) / 32768 * 32768 + 16384;
  }

  template <class L>
  int launch(int kind, double bytes, L&& fn) {
    return launch_on(kind, bytes, s, static_cast<L&&>(fn));
  }
  // The same for a launch on another stream `st` (timed with events on st).
  template <class L>
  int launch_on(int kind, double bytes, hipStream_t st, L&& fn);
  // Finish a reduction whose per-block partials are in partial(): values [0,nsum) summed,
  // [nsum,nv) max-reduced, across blocks and ranks; result in out[0,nv).  Synchronises.
  int reduce(int64_t nblk, int nsum, int nv, double* out);
  // The same without synchronising: the result lands in device slot dres(slot) (ordered on the
  // stream, all-reduced across ranks) and, after the next sync(), in host slot hres(slot).
  // host_copy = false: with a communicator, leave out the D2H copy of the all-reduced result
  // (a device-side consumer copies what the host needs itself).
  int reduce_async(int64_t nblk, int nsum, int nv, int slot, bool host_copy = true);
  const double* dres(int slot) const { return dres_ + slot; }
  const double* hres(int slot) const { return hres_ + slot; }
  double* dres_mut(int slot) const { return dres_ + slot; }  // for a kernel that writes a slot
  double* hres_mut(int slot) const { return hres_ + slot; }
  static constexpr int kSlots = 1024;
  // multi-dot results of Arnoldi step j (<= 2*kMaxVec+1 values): a ring of four, so the results
  // of a step stay readable while the device-side control queues the next two
  static int slot_mdot(int j) { return (j & 3) * 136; }
  static constexpr int kSlotCombo = 560;  // 2 values
  static constexpr int kSlotSync = 600;   // reduce()
  int sync();
  // Wait for the nv results a reduce_async(.., slot) writes to the pinned host slots, by polling
  // them (the reduction kernel stores every value straight into pinned memory, the slots were
  // marked beforehand); no stream synchronisation.  Falls back to sync() with a communicator
  // (results come through a D2H copy), after ~1 s, or with NKHIP_POLL=0.
  int wait_results(int slot, int nv);
  // Wait until a kernel sets the pinned word *flag (non-zero); returns its value, or 0 after a
  // stream synchronisation found it still unset (the writer did not run).
  uint32_t wait_flag(const uint32_t* flag);
  int copy(double* dst, const double* src, int64_t n);
  // The last `count` launches of `kind` did nothing (device-controlled steps queued past a step
  // the control handed back, nk_kernels.h arn_halted): take them out of the launch counts, the
  // algorithmic bytes and, where they were timed, the timed sample -- a no-op timed with a fused
  // step's bytes would inflate the roofline figure.
  void void_last(int kind, int count);

  double* partial() const { return partial_; }
  int64_t partial_cap() const { return partial_cap_; }
  const KStat& stat(int k) const { return stats_[k]; }
  void reset_stats();
  int64_t bytes_allocated() const { return bytes_; }

  int64_t n;
  int64_t npad;
  nk_comm* comm;
  hipStream_t s;
  bool profile;
  int sample = 1;  // with profile: time every sample-th launch of each class (events cost ~5 us)

 private:
  void harvest();
  hipEvent_t ev();
  double* pool_ = nullptr;
  bool own_pool_ = false;
  int pool_count_ = 0;
  std::vector<uint8_t> ekept_;  // per pool vector: mark_edges
  double* epool_ = nullptr;
  int64_t edge_ny_ = 0, edge_nx_ = 0, edge_n_ = 0;
  double* partial_ = nullptr;
  int64_t partial_cap_ = 0;
  double* dres_ = nullptr;
  double* hres_ = nullptr;
  int64_t bytes_ = 0;
  // a pool mapped through the virtual memory API (vmm_alloc): reserved range and its handles
  void* vmm_base_ = nullptr;
  size_t vmm_size_ = 0, vmm_chunk_ = 0;
  std::vector<hipMemGenericAllocationHandle_t> vmm_h_;
  int vmm_alloc(size_t bytes, size_t chunk);
  void vmm_free();
  struct Pending {
    int kind;
    hipEvent_t a, b;
    double bytes;
    int64_t idx;  // the launch's index in its class
  };
  static constexpr int kRecent = 8;
  double recent_bytes_[K_NKINDS][kRecent] = {};  // bytes of the latest launches per class
  std::vector<Pending> pend_;
  std::vector<hipEvent_t> free_ev_;
  KStat stats_[K_NKINDS];
  int64_t tick_[K_NKINDS] = {};
};

template <class L>
int Engine::launch_on(int kind, double bytes, hipStream_t st, L&& fn) {
  hipEvent_t a = nullptr, b = nullptr;
  const bool timed = profile && (tick_[kind]++ % sample == 0);
  if (timed) {
    a = ev();
    hipEventRecord(a, st);
  }
  const hipError_t e = fn();
  if (timed) {
    b = ev();
    hipEventRecord(b, st);
    pend_.push_back(Pending{kind, a, b, bytes, stats_[kind].launches});
  }
  recent_bytes_[kind][stats_[kind].launches % kRecent] = bytes;
  stats_[kind].launches += 1;
  stats_[kind].bytes += bytes;
  log_launch(kind, bytes);
  return e == hipSuccess ? NK_OK : NK_EHIP;
}

// The nonlinear problem seen by the Newton-Krylov core.
struct Problem {
  virtual ~Problem() = default;
  virtual int64_t n_global() const = 0;
  // F(x + alpha p) -> F; G = the x-dependent part that the FD JVP differences (F = G + const);
  // xt = x + alpha p if non-null.  red = {sum F^2, max|F|, max|x + alpha p|} over all ranks.
  virtual int eval(const double* x, const double* p, double alpha, double* xt, double* F,
                   double* G, double red[3]) = 0;
  // w = J z.  FD: w = (G(x0 + sc*zs*z) - G0)/sc (KrylovJacobian.matvec); analytic: zs*J(x0) z.
  virtual int jvp(const double* x0, const double* G0, const double* z, double zs, double sc,
                  double* w) = 0;
  // As jvp() for z = raw basis vector whose |z|^2 sits in device memory (znorm2): the scale is
  // computed in-kernel, so no host round trip is needed before the JVP.
  virtual bool has_dev_scale() const { return false; }
  virtual int jvp_dev(const double* /*x0*/, const double* /*G0*/, const double* /*z*/,
                      const double* /*znorm2*/, double /*omega*/, double* /*w*/) {
    return NK_EINVAL;
  }
  // May the solver evaluate a JVP it later discards (the step after the last Arnoldi step)?  A
  // user callback must see exactly scipy's F calls, so the generic problem says no.
  virtual bool may_speculate() const { return true; }
  // Device-side Arnoldi control without a fused kernel (lgmres.cpp device_steps): w = J z with
  // the JVP's scale and FD step from the control's parameter block prm (nk_kernels.h kCtlPrm);
  // nothing when the step was handed back.  Problems whose Arnoldi steps are latency-bound
  // launches (the moving-mesh residuals) prefer the device control even on one GPU.
  virtual bool has_jvp_prm() const { return false; }
  virtual int jvp_prm(const double* /*x0*/, const double* /*G0*/, const double* /*z*/,
                      const double* /*prm*/, double* /*w*/) {
    return NK_EINVAL;
  }
  virtual bool prefers_devctl() const { return false; }
  // Fused Arnoldi step (arnoldi.hip): v = tau w + sum c_i V_i -> out_v, w' = J z -> out_w with
  // z = v (z == nullptr) or z = the given vector (scale zs, norm-free step sc), and the multi-dot
  // partials of w' and v against V_0..V_{nv-1}, v; *nwaves = partial columns.
  virtual bool has_fused(int /*nv*/) const { return false; }
  virtual int fused_step(const double* const* /*V*/, const double* /*c*/, int /*nv*/,
                         const double* /*w*/, double /*tau*/, const double* /*x0*/,
                         const double* /*G0*/, const double* /*z*/, double /*zs*/, double /*sc*/,
                         double* /*out_v*/, double* /*out_w*/, int64_t* /*nwaves*/,
                         const double* /*ctl*/, const ArnTail* /*tail*/ = nullptr,
                         bool* /*tail_used*/ = nullptr) {
    return NK_EINVAL;
  }
  // ctl of fused_step (device-side Arnoldi control, nk_kernels.h ArnoldiArgs): c, tau, zs and sc
  // come from the device parameter block ctl, and the step does nothing when its halt entry is set.
  // tail (optional): the step's reduction + control run in the launch's last blocks
  // (ArnoldiArgs::tail) where the step is one launch; *tail_used says whether it did.
  // v (a pool vector) may enter the update of a later fused step: refresh its edge array.
  // eval()'s F and jvp()'s w come with fresh edge arrays (written by the pass itself); the solver
  // calls this after the other producers of update entries (its in-place combinations).
  // written: the combination already wrote v's edge array (edge_out), only the rest is left.
  virtual int publish_edges(const double* /*v*/, bool /*written*/ = false) { return NK_OK; }
  // The edge array a combination that writes v should write itself (EdgeOut{}: none).
  virtual EdgeOut edge_out(const double* /*v*/) { return EdgeOut{}; }
  // The last `count` fused steps were no-ops (queued past a step the device control handed
  // back): take their launches out of the kernel profile (Engine::void_last).
  virtual void void_fused_steps(int /*count*/) {}
  virtual int set_x0(const double* /*x0*/) { return NK_OK; }   // new Newton iterate (halo)
  virtual int set_dir(const double* /*d*/) { return NK_OK; }   // new search direction (halo)
  // Speculative first JVP of the next LGMRES call (NewtonKrylov::line_search): w = J z at the
  // trial point x0 = xt, G0 = G of the NEXT eval(), issued by that eval right behind its
  // reduction and before it synchronises; the pass itself decides from the reduction whether it
  // runs (StencilArgs::spec) and computes the host's FD step.  arm_spec(nullptr) disarms.
  struct SpecJvp {
    const double* z;
    double zs, zn;           // z's scale and |zs z| (the host's input(0) of the next call)
    double thr, ftol, rdiff;  // Armijo threshold of s = 1, f_tol, rdiff
    double* w;               // the next call's V_[1]
  };
  virtual bool can_spec_jvp() const { return false; }
  virtual void arm_spec(const SpecJvp* /*sp*/) {}
};

// nonlin_solve + KrylovJacobian + lgmres(maxiter=1, outer_k, prepend_outer_v) on one Problem.
class NewtonKrylov {
 public:
  NewtonKrylov(Engine& E, Problem& P, const nk_opts& o, void* external = nullptr,
               int64_t external_bytes = 0);
  ~NewtonKrylov();
  NewtonKrylov(const NewtonKrylov&) = delete;
  NewtonKrylov& operator=(const NewtonKrylov&) = delete;
  int status() const { return init_status_; }
  void set_opts(const nk_opts& o) { o_ = o; }
  // x_out = root of F starting from x_in (device, length n; may alias).  Returns NK_* status.
  int solve(const double* x_in, double* x_out, nk_stats* st);
  static int vectors_needed(const nk_opts& o) { return o.inner_m + 2 * o.outer_k + 8; }
  // Accepted Armijo step s of every Newton iteration of the last solve (scipy's
  // scalar_search_armijo result, _nonlin.py:294-314; 1 where no line search ran).
  const std::vector<double>& step_log() const { return steps_; }

 private:
  int lgmres(double tol, double* dnorm, double* dmax, double** dvec);
  // Launch JVP_j (w = V[j+1] = J z_j) and the fused multi-dot of step j; no synchronisation.
  int issue_step(int j, const double* z, double zs, double znorm, bool dev_scale,
                 bool have_w = false);
  // Device-side Arnoldi control (arnctl.hip): from step S.j (whose fused launch and reduction
  // are queued), queue fused step + reduction + control per step, one step ahead of the
  // control's status words, until the control hands a step back; then restore the host's view
  // of the vectors at that step (the control mirrors the state into hS_ itself).
  int device_steps();
  const double* zp_[kMaxVec + 1];
  ArnCtlState* hS_ = nullptr;   // the loop state (pinned; zs_ of the final combination inside)
  ArnCtlState* dS_ = nullptr;   // its device copy
  double* prm_ = nullptr;       // parameter block of the next fused step (device)
  uint32_t* status_ = nullptr;  // per-step status words the control kernel writes (pinned)
  int line_search(double* s_out, double* fnorm_new, double* fmax, double* xmax);

  Engine& E_;
  Problem& P_;
  nk_opts o_;
  int init_status_ = NK_OK;
  // vectors
  double *X_ = nullptr, *Xt_ = nullptr, *Fx_ = nullptr, *Ft_ = nullptr, *G0_ = nullptr,
         *Gt_ = nullptr;
  double* Sv_ = nullptr;  // spare vector: target of the fused update (swapped into V_)
  std::vector<double*> V_;      // V_[0] aliases Fx_ during a solve
  std::vector<double*> outer_;  // LGMRES augmentation ring
  std::vector<double> osig_, orn_;
  int ocount_ = 0, ohead_ = 0;
  double omega_ = 0.0;
  double* d_ = nullptr;  // current search direction (an outer slot)
  nk_stats* st_ = nullptr;
  std::vector<double> steps_;  // step_log()
  double fx_norm_ = 0.0;
  double rdiff_ = 0.0;
  double f_tol_ = 0.0;
  // the speculative first JVP of the next LGMRES call (line_search): ran on the device at the
  // trial point x with G(x) = g (the pool vectors an accepted s = 1 swaps into X_ / G0_)
  struct {
    bool valid = false;
    const double* z = nullptr;
    double zs = 0.0, zn = 0.0;
    double* w = nullptr;
    const double* x = nullptr;
    const double* g = nullptr;
  } spec_;
};

// Default options (SciPy newton_krylov defaults).
nk_opts default_opts();

namespace detail {
void givens(double a, double b, double* c, double* s);
void lstsq_upper(const double (*R)[kMaxVec + 1], int n, const double* g, double* y);
}  // namespace detail

}  // namespace nk

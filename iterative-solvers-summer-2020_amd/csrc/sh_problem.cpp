// Swift-Hohenberg stepper problem and generic callback problem (see sh_problem.h).
#include "sh_problem.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "peer_dev.h"

namespace nk {

// ============================================================================================
// SHProblem
// ============================================================================================
SHProblem::SHProblem(Engine& E, int64_t ny, int64_t nx, int64_t ny_global, SHCoef c, int jvp_mode)
    : E_(E), ny_(ny), nx_(nx), ny_g_(ny_global), c_(c), jvp_mode_(jvp_mode) {
  // edge arrays for the fused Arnoldi kernel's block halos (1/64 of each pool vector)
  if (arnoldi_supported(1, ny, nx)) E_.enable_edges(ny, nx);
  // the fused kernel's mailbox, unless the slabs of several ranks share this device (their
  // launches run concurrently, so a band's blocks need not be resident together)
  if (arnoldi_supported(1, ny, nx) && !(E_.comm && E_.comm->shares_device())) {
    const int64_t n = arnoldi_mbox_elems(ny, nx);
    if (hipMalloc(reinterpret_cast<void**>(&mb_), sizeof(double) * n) == hipSuccess &&
        hipMemset(mb_, 0, sizeof(double) * n) == hipSuccess) {
      mb_cap_ = n;
    } else {
      if (mb_) hipFree(mb_);
      mb_ = nullptr;  // optional: the packed halo loads
      (void)hipGetLastError();
    }
  }
  if (hipMalloc(reinterpret_cast<void**>(&B_), sizeof(double) * Engine::pad(ny * nx)) !=
      hipSuccess) {
    B_ = nullptr;
    status_ = NK_ENOMEM;
    return;
  }
  if (dist()) {
    if (ny < 2) {
      status_ = NK_EINVAL;  // a 2-row halo must come from one neighbour
      return;
    }
    double* h = nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&h), sizeof(double) * 24 * nx) != hipSuccess) {
      status_ = NK_ENOMEM;
      return;
    }
    hx_ = h;
    hz_ = h + 4 * nx;
    hd_ = h + 8 * nx;
    hu_ = h + 12 * nx;
    y4_ = h + 16 * nx;
    yh_ = h + 20 * nx;
    // the halo slots of the pushed-halo-rows path (peer-memory communicator, one stepper)
    if (!E_.comm->claim_slots(this, &slots_) || slots_.ld < nx) {
      if (slots_.mine) E_.comm->release_slots(this);
      slots_ = nk_halo_slots{};
    }
    // every rank must take the fused Arnoldi path or none, and the pushed halo rows or none:
    // decide on the smallest and the largest slab and on whether any rank went without its
    // slots (one all-reduce; every rank constructs its problem).  A rank whose slots another
    // stepper still holds would otherwise read slots its neighbours never push, or wait in halo
    // exchanges they never join.
    double mm[3] = {-double(ny), double(ny), slots_.mine ? 0.0 : 1.0};
    if (hipMemcpyAsync(y4_, mm, sizeof(mm), hipMemcpyHostToDevice, E_.s) != hipSuccess ||
        E_.comm->allreduce(y4_, 0, 3, E_.s) != NK_OK ||
        hipMemcpyAsync(mm, y4_, sizeof(mm), hipMemcpyDeviceToHost, E_.s) != hipSuccess ||
        hipStreamSynchronize(E_.s) != hipSuccess) {
      status_ = NK_ECOMM;
      return;
    }
    ny_min_ = int64_t(-mm[0]);
    ny_max_ = int64_t(mm[1]);
    if (mm[2] > 0.0 && slots_.mine) {  // some rank has none: no rank pushes
      E_.comm->release_slots(this);
      slots_ = nk_halo_slots{};
    }
    if (hipStreamCreateWithFlags(&side_, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&ev_in_, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ev_out_, hipEventDisableTiming) != hipSuccess) {
      status_ = NK_EHIP;
      return;
    }
  }
}

SHProblem::~SHProblem() {
  if (slots_.mine) E_.comm->release_slots(this);
  if (side_) hipStreamSynchronize(side_);
  if (B_) hipFree(B_);
  if (hx_) hipFree(hx_);
  if (mb_) hipFree(mb_);
  if (ev_in_) hipEventDestroy(ev_in_);
  if (ev_out_) hipEventDestroy(ev_out_);
  if (side_) hipStreamDestroy(side_);
}

namespace {
// Rows [r0, r1) of a slab field as a field of its own: the two rows above / below come from the
// slab itself, or from the slab's halo at its top / bottom edge.
Field sub_field(const Field& f, int64_t r0, int64_t r1, int64_t ny, int64_t nx) {
  if (!f.base) return f;
  Field s;
  s.base = f.base + r0 * nx;
  s.lo = (r0 >= 2) ? f.base + (r0 - 2) * nx : f.lo;
  s.hi = (r1 + 2 <= ny) ? f.base + r1 * nx : f.hi;
  return s;
}

StencilArgs sub_args(const StencilArgs& A, int64_t r0, int64_t r1) {
  StencilArgs B = A;
  B.ny = r1 - r0;
  B.a = sub_field(A.a, r0, r1, A.ny, A.nx);
  B.b = sub_field(A.b, r0, r1, A.ny, A.nx);
  const int64_t off = r0 * A.nx;
  B.e_row0 = A.e_row0 + r0;
  if (A.p0) B.p0 = A.p0 + off;
  if (A.out0) B.out0 = A.out0 + off;
  if (A.out1) B.out1 = A.out1 + off;
  if (A.out2) B.out2 = A.out2 + off;
  return B;
}
}  // namespace

int SHProblem::halo_stencil(int kind, SMode m, const StencilArgs& A, const double* z, double* zh) {
  const double bytes = stencil_bytes_per_point(m, false);
  if (!z)  // the halo rows are already in place (pushed slots): just the pass
    return E_.launch(kind, bytes * ny_ * nx_, [&] { return stencil_launch(m, A, E_.s, nullptr); });
  if (!dist() || ny_ < 8 || !side_) {
    int rc = halo(z, zh);
    if (rc) return rc;
    return E_.launch(kind, bytes * ny_ * nx_,
                     [&] { return stencil_launch(m, A, E_.s, nullptr); });
  }
  // interior rows [2, ny-2) need no halo: run them on the side stream during the exchange
  if (hipEventRecord(ev_in_, E_.s) != hipSuccess ||
      hipStreamWaitEvent(side_, ev_in_, 0) != hipSuccess)
    return NK_EHIP;
  const StencilArgs I = sub_args(A, 2, ny_ - 2);
  if (stencil_launch(m, I, side_, nullptr) != hipSuccess) return NK_EHIP;
  if (hipEventRecord(ev_out_, side_) != hipSuccess) return NK_EHIP;
  int rc = halo(z, zh);
  if (rc) return rc;
  const StencilArgs T = sub_args(A, 0, 2), Bm = sub_args(A, ny_ - 2, ny_);
  // the profile books the whole pass under `kind` (edges timed on the main stream, the interior
  // overlapping the exchange)
  rc = E_.launch(kind, bytes * ny_ * nx_, [&] {
    hipError_t e = stencil_launch(m, T, E_.s, nullptr);
    if (e == hipSuccess) e = stencil_launch(m, Bm, E_.s, nullptr);
    if (e == hipSuccess) e = hipStreamWaitEvent(E_.s, ev_out_, 0);
    return e;
  });
  return rc;
}

Field SHProblem::field(const double* p, const double* halo) const {
  if (!dist()) return periodic(p);
  return Field{p, halo, halo + 2 * nx_};
}

int SHProblem::halo(const double* v, double* h) {
  if (!dist()) return NK_OK;
  return E_.launch(K_HALO, 2.0 * 4 * 8 * nx_,
                   [&] {
                     return E_.comm->halo(v, h, h + 2 * nx_, ny_, nx_, E_.s) == NK_OK
                                ? hipSuccess
                                : hipErrorUnknown;
                   }) == NK_OK
             ? NK_OK
             : NK_ECOMM;
}

int SHProblem::prepare(const double* u_prev) {
  int rc = halo(u_prev, hu_);
  if (rc) return rc;
  StencilArgs A;
  A.ny = ny_;
  A.nx = nx_;
  A.a = field(u_prev, hu_);
  A.c = c_;
  A.out0 = B_;
  return E_.launch(K_BOLD, stencil_bytes_per_point(SMode::BOLD, false) * ny_ * nx_,
                   [&] { return stencil_launch(SMode::BOLD, A, E_.s, nullptr); });
}

// The halo of the Newton iterate / the search direction: from the pushed slots when the producer
// pushed them before an all-reduce issued since (the TRIAL pass pushes x + alpha p, the final
// combination pushes d), else exchanged
int SHProblem::set_x0(const double* x0) {
  hxp_ = slot_halo(x0);
  if (hxp_) return NK_OK;
  hxp_ = hx_;
  return halo(x0, hx_);
}
int SHProblem::set_dir(const double* d) {
  hdp_ = slot_halo(d);
  if (hdp_) return NK_OK;
  hdp_ = hd_;
  return halo(d, hd_);
}

// A stencil pass's outputs pushed in-kernel (pushed halo rows): out0 (and out2) into the
// neighbours' slots, with the pass (march path: A->E0 set, so e_ny / e_row0 are)
void SHProblem::set_push(StencilArgs* A, const double* out0, const double* out2) {
  if (!push_mode() || !A->E0) return;
  double* p0 = slot(slots_.prev, out0);
  double* n0 = slot(slots_.next, out0);
  if (!p0 || !n0) return;
  A->PS0[0] = p0;
  A->PS0[1] = n0;
  A->ps_ld = slots_.ld;
  pushed(out0);
  if (out2) {
    double* p2 = slot(slots_.prev, out2);
    double* n2 = slot(slots_.next, out2);
    if (p2 && n2) {
      A->PS2[0] = p2;
      A->PS2[1] = n2;
      pushed(out2);
    }
  }
}

void SHProblem::pushed(const double* v) {
  const int64_t q = E_.pool_index(v);
  if (q < 0) return;
  if (push_ep_.size() < size_t(E_.pool_count())) push_ep_.assign(E_.pool_count(), ~uint64_t(0));
  push_ep_[q] = E_.comm->epoch();
}

const double* SHProblem::slot_halo(const double* v) const {
  if (!push_mode() || slots_.ld != nx_ || !has_fused(1)) return nullptr;
  const int64_t q = E_.pool_index(v);
  if (q < 0 || size_t(q) >= push_ep_.size() || push_ep_[q] == ~uint64_t(0) ||
      !(E_.comm->epoch() > push_ep_[q]))
    return nullptr;
  return slots_.mine + q * 4 * slots_.ld;
}

bool SHProblem::push_mode() const {
  if (!slots_.mine || E_.pool_count() > slots_.count || slab_x_enabled(E_.comm)) return false;
  const char* e = std::getenv("NKHIP_SLAB_PUSH");
  return !(e && e[0] == '0');
}

double* SHProblem::slot(double* base, const double* v) const {
  const int64_t q = E_.pool_index(v);
  return q < 0 ? nullptr : base + q * 4 * slots_.ld;
}

int SHProblem::push(const double* v) {
  if (!push_mode() || !has_fused(1)) return NK_OK;
  double* pp = slot(slots_.prev, v);
  double* pn = slot(slots_.next, v);
  if (!pp || !pn) return NK_OK;  // not a pool vector: never an entry of a fused step
  const int rc = E_.launch(K_PUSH, 2.0 * 4 * 8 * nx_, [&] {
    return push_rows_launch(v, pp, pn, ny_, nx_, slots_.ld, E_.s);
  });
  if (!rc) pushed(v);
  return rc;
}

int SHProblem::eval(const double* x, const double* p, double alpha, double* xt, double* F,
                    double* G, double red[3]) {
  StencilArgs A;
  A.ny = ny_;
  A.nx = nx_;
  A.a = field(x, hxp_ ? hxp_ : hx_);
  A.b = (p == x) ? A.a : field(p, hdp_ ? hdp_ : hd_);
  A.alpha = alpha;
  A.p0 = B_;
  A.out0 = F;
  A.out1 = G;
  A.out2 = xt;
  A.c = c_;
  A.partial = E_.partial();
  set_edges(&A, F);
  if (A.E0 && xt && (A.E2 = E_.edges(xt)) != nullptr) E_.mark_edges(xt);  // the next x0
  set_push(&A, F, xt);
  int64_t nblk = 0;
  int rc = E_.launch(K_TRIAL, stencil_bytes_per_point(SMode::TRIAL, xt != nullptr) * ny_ * nx_,
                     [&] { return stencil_launch(SMode::TRIAL, A, E_.s, &nblk); });
  // (F may become V_0 and xt the next iterate x0: their edge rows went into the neighbours'
  // slots in the pass, before the all-reduce of the reduction below)
  if (rc) return rc;
  const SpecJvp sp = spec_;
  spec_ = SpecJvp{};
  if (!sp.z || !xt || dist()) return E_.reduce(nblk, 1, 3, red);
  // the next LGMRES call's first JVP at x0 = xt, right behind the reduction it depends on (the
  // pass decides from it whether it runs): the GPU goes on while the host reads the result
  rc = E_.reduce_async(nblk, 1, 3, Engine::kSlotSync);
  if (!rc) {
    StencilArgs J;
    J.ny = ny_;
    J.nx = nx_;
    J.c = c_;
    J.out0 = sp.w;
    set_edges(&J, sp.w);
    J.a = field(xt, hx_);
    J.b = field(sp.z, hz_);
    J.p0 = G;
    J.spec = E_.dres(Engine::kSlotSync);
    J.spec_thr = sp.thr;
    J.spec_ftol = sp.ftol;
    J.spec_rdiff = sp.rdiff;
    J.spec_zn = sp.zn;
    J.spec_zs = sp.zs;
    side_edges(&J, xt, sp.z);
    rc = halo_stencil(K_FDJVP, SMode::FDJVP, J, nullptr, hz_);
  }
  // the reduction writes its pinned host slot itself: read it there without draining the
  // stream, so the JVP keeps the GPU busy while the host decides and queues the next launches
  if (!rc) rc = E_.wait_results(Engine::kSlotSync, 3);
  if (rc) return rc;
  std::memcpy(red, E_.hres(Engine::kSlotSync), sizeof(double) * 3);
  return NK_OK;
}

// one slab, FD JVP, and not switched off (NKHIP_SPEC_JVP=0, read per call)
bool SHProblem::can_spec_jvp() const {
  const char* e = std::getenv("NKHIP_SPEC_JVP");
  return !dist() && jvp_mode_ == NK_JVP_FD && !(e && e[0] == '0');
}

int SHProblem::jvp(const double* x0, const double* G0, const double* z, double zs, double sc,
                   double* w) {
  StencilArgs A;
  A.ny = ny_;
  A.nx = nx_;
  A.c = c_;
  A.out0 = w;
  set_edges(&A, w);
  set_push(&A, w, nullptr);
  const double* zsh = slot_halo(z);  // z's halo rows already here (pushed): no exchange
  if (jvp_mode_ == NK_JVP_ANALYTIC) {
    A.a = field(z, zsh ? zsh : hz_);
    A.alpha = zs;
    A.p0 = x0;
    const int rc = halo_stencil(K_AJVP, SMode::AJVP, A, zsh ? nullptr : z, hz_);
    return rc;
  }
  A.a = field(x0, hxp_ ? hxp_ : hx_);
  A.b = field(z, zsh ? zsh : hz_);
  A.alpha = sc * zs;
  A.p0 = G0;
  A.sc = sc;
  side_edges(&A, x0, z);
  const int rc = halo_stencil(K_FDJVP, SMode::FDJVP, A, zsh ? nullptr : z, hz_);
  return rc;
}

int SHProblem::jvp_dev(const double* x0, const double* G0, const double* z, const double* znorm2,
                       double omega, double* w) {
  StencilArgs A;
  A.ny = ny_;
  A.nx = nx_;
  A.c = c_;
  A.out0 = w;
  set_edges(&A, w);
  set_push(&A, w, nullptr);
  A.znorm2 = znorm2;
  A.omega = omega;
  const double* zsh = slot_halo(z);
  if (jvp_mode_ == NK_JVP_ANALYTIC) {
    A.a = field(z, zsh ? zsh : hz_);
    A.p0 = x0;
    const int rc = halo_stencil(K_AJVP, SMode::AJVP, A, zsh ? nullptr : z, hz_);
    return rc;
  }
  A.a = field(x0, hxp_ ? hxp_ : hx_);
  A.b = field(z, zsh ? zsh : hz_);
  A.p0 = G0;
  side_edges(&A, x0, z);
  const int rc = halo_stencil(K_FDJVP, SMode::FDJVP, A, zsh ? nullptr : z, hz_);
  return rc;
}

// One launch per Arnoldi step with the FD JVP (arnoldi.hip).  On a row slab the kernel needs u
// on the neighbours' two edge rows: every rank first evaluates u on its own edge rows (a 4-row
// launch), exchanges them, then runs the fused pass with those rows as its halo.
// NKHIP_FUSED=0 disables it (read per call, so a test can compare both paths in one process).
bool SHProblem::has_fused(int nv) const {
  const char* e = std::getenv("NKHIP_FUSED");
  if (e && e[0] == '0') return false;
  if (jvp_mode_ != NK_JVP_FD) return false;
  if (!dist()) return arnoldi_supported(nv, ny_, nx_);
  return arnoldi_supported(nv, ny_min_, nx_) && arnoldi_supported(nv, ny_max_, nx_);
}

int SHProblem::fused_step(const double* const* V, const double* c, int nv, const double* w,
                          double tau, const double* x0, const double* G0, const double* z,
                          double zs, double sc, double* out_v, double* out_w, int64_t* nwaves,
                          const double* ctl, const ArnTail* tail, bool* tail_used) {
  ArnoldiArgs A;
  A.ctl = ctl;
  if (tail_used) *tail_used = false;
  // the step's reduction + control in the fused launch's last blocks (single-launch paths only)
  auto with_tail = [&] {
    if (!tail) return;
    A.tail = *tail;
    if (tail_used) *tail_used = true;
  };
  A.ny = ny_;
  A.nx = nx_;
  A.nv = nv;
  for (int i = 0; i < nv; ++i) {
    A.V[i] = V[i];
    A.c[i] = c[i];
  }
  A.w = w;
  A.tau = tau;
  A.x0 = x0;
  A.g0 = G0;
  A.z = z;
  A.alpha = sc * zs;  // y = x0 + sc*zs*z (KrylovJacobian.matvec, _nonlin.py:1505-1509)
  A.sc = sc;
  A.k = c_;
  A.out_v = out_v;
  A.out_w = out_w;
  A.partial = E_.partial();
  A.partial_cap = E_.partial_cap();
  // block halos from the entries' edge arrays when every entry has one (else from the vectors)
  bool all = true;
  for (int i = 0; i < nv; ++i) all = all && (A.E[i] = E_.edges(V[i])) != nullptr;
  all = all && (A.E[nv] = E_.edges(w)) != nullptr;
  const char* eoff = std::getenv("NKHIP_EDGES");
  if (!all || (eoff && eoff[0] == '0'))
    for (int i = 0; i <= nv; ++i) A.E[i] = nullptr;
  A.Eout_v = E_.edges(out_v);
  A.Eout_w = E_.edges(out_w);
  if (A.Eout_v) E_.mark_edges(out_v);
  if (A.Eout_w) E_.mark_edges(out_w);
  if (mb_) {
    const int mode = arnoldi_mbox_mode();
    if (mode != 0) {
      A.mb = mb_;
      A.mb_cap = mb_cap_;
      A.mb_tag = ++mb_tag_;
      A.mb_recompute = mode == 2;
    }
  }
  // algorithmic bytes per row: read V (nv), w, x0 (, z); write v, w'
  const double rowb = 8.0 * double(nx_) * (nv + 4 + (z ? 1 : 0));
  if (!dist()) {
    with_tail();
    return E_.launch(K_ARNOLDI, rowb * ny_, [&] { return arnoldi_launch(A, E_.s, nwaves); });
  }

  // Row slab: the stencil of rows 0, 1, ny-2, ny-1 needs u on the neighbours' edge rows, which
  // this step computes.  Every rank evaluates u on its own edge rows (a 4-row launch) and
  // exchanges them with its ring neighbours; meanwhile the interior rows [2, ny-2), whose
  // stencil reads only this slab's rows, run on the side stream.  The two 2-row edge bands follow
  // the exchange.  All three launches write disjoint columns of one partial buffer, so the
  // multi-dot stays one reduction (one all-reduce).  Opt-in (NKHIP_SLAB_OVERLAP=1): measured at
  // world size 1 over RCCL (4096 rows, scripts/slab_ab.sh, profiles/r02_slab_overlap.md) the
  // interior pass loses more to the CUs it leaves for the exchange kernels, plus the two
  // latency-bound 2-row launches after it, than the exchange costs in series (0.678 vs 0.658 ms
  // per Arnoldi step); the default is one launch after the exchange.
  // Pushed halo rows: every entry's halo rows already sit in this rank's slots (arnoldi.hip):
  // one launch, no exchange before it; its outputs' edge rows go into the neighbours' slots
  if (push_mode()) {
    bool ok = true;
    for (int i = 0; i < nv; ++i) ok = ok && (A.HS[i] = slot(slots_.mine, V[i])) != nullptr;
    ok = ok && (A.HS[nv] = slot(slots_.mine, w)) != nullptr;
    if (z) ok = ok && (A.HS[nv + 1] = slot(slots_.mine, z)) != nullptr;
    ok = ok && (A.PS[0] = slot(slots_.prev, out_v)) != nullptr &&
         (A.PS[1] = slot(slots_.next, out_v)) != nullptr &&
         (A.PS[2] = slot(slots_.prev, out_w)) != nullptr &&
         (A.PS[3] = slot(slots_.next, out_w)) != nullptr;
    if (ok) {
      A.hs_ld = slots_.ld;
      pushed(out_v);
      pushed(out_w);
      A.yh = y4_;  // u on the halo rows, filled by the edge bands (4 rows of nx)
      A.yh_ld = nx_;
      last_split_ = false;
      edge_launched_ = false;
      with_tail();
      return E_.launch(K_ARNOLDI, rowb * ny_, [&] { return arnoldi_launch(A, E_.s, nwaves); });
    }
    for (int i = 0; i <= nv + 1; ++i) A.HS[i] = nullptr;
    for (auto& p : A.PS) p = nullptr;
  }
  const char* ov = std::getenv("NKHIP_SLAB_OVERLAP");
  const bool split = ny_ >= 12 && side_ && (ov && ov[0] == '1');
  last_split_ = split;
  ArnoldiArgs I = A, T = A, Bm = A;
  int64_t nwI = 0, nwT = 0, nwB = 0;
  if (split) {
    I.r_begin = 2;
    I.r_end = ny_ - 2;
    // leave CUs for the edge kernel and the RCCL send/recv kernels that run beside it (a
    // resident round of fused blocks holds every CU until it ends)
    static const int reserve = [] {
      const char* e = std::getenv("NKHIP_SLAB_RESERVE_CUS");
      return (e && *e) ? std::atoi(e) : 8;
    }();
    I.reserve_cus = reserve;
    T.r_begin = 0;
    T.r_end = 2;
    Bm.r_begin = ny_ - 2;
    Bm.r_end = ny_;
    I.plan_only = T.plan_only = Bm.plan_only = true;
    if (arnoldi_launch(I, E_.s, &nwI) != hipSuccess || arnoldi_launch(T, E_.s, &nwT) != hipSuccess ||
        arnoldi_launch(Bm, E_.s, &nwB) != hipSuccess)
      return NK_EHIP;
    I.plan_only = T.plan_only = Bm.plan_only = false;
    I.pstride = T.pstride = Bm.pstride = nwI + nwT + nwB;
    I.pcol0 = 0;
    T.pcol0 = nwI;
    Bm.pcol0 = nwI + nwT;
    if (hipEventRecord(ev_in_, E_.s) != hipSuccess || hipStreamWaitEvent(side_, ev_in_, 0) != hipSuccess)
      return NK_EHIP;
    int64_t nw = 0;
    int rc = E_.launch_on(K_ARNOLDI, rowb * (ny_ - 4), side_,
                          [&] { return arnoldi_launch(I, side_, &nw); });
    if (rc) return rc;
    if (hipEventRecord(ev_out_, side_) != hipSuccess) return NK_EHIP;
  }
  // edge rows of u -> the ring neighbours (y4_ holds rows 0, 1, ny-2, ny-1 as a 4-row slab)
  const double eb = 8.0 * 4 * nx_ * (z ? 2 : nv + 2);
  int rc = NK_OK;
  PeerArgs pa;
  edge_launched_ = true;
  if (!split && slab_x_enabled(E_.comm) && E_.comm->take_halo(&pa, nx_)) {
    // peer-memory communicator: the fused kernel's edge bands exchange the edge rows themselves
    // (arnoldi.hip "Slab exchange"); the halo rows are read from this rank's staging rows
    const int par = int(pa.tag & 1);
    A.x.me = pa.base[pa.rank];
    A.x.prev = pa.base[(pa.rank - 1 + pa.P) % pa.P];
    A.x.next = pa.base[(pa.rank + 1) % pa.P];
    A.x.P = pa.P;
    A.x.max_nx = pa.max_nx;
    A.x.tag = pa.tag;
    A.x.err = pa.err;
    A.x.wait_ticks = pa.wait_ticks;
    A.yh = stage(A.x.me, pa.P, pa.max_nx, par, 0, 0);
    A.yh_ld = pa.max_nx;
    edge_launched_ = false;
    with_tail();
    return E_.launch(K_ARNOLDI, rowb * ny_, [&] { return arnoldi_launch(A, E_.s, nwaves); });
  }
  if (!split && peer_fuse_enabled() && E_.comm->take_halo(&pa, nx_)) {
    // peer-memory communicator: the edge rows go straight into the neighbours' staging rows
    // and come back into yh_ in the same launch (no y4_ round trip, no separate halo kernel)
    rc = E_.launch(K_ARN_EDGE, eb + 2.0 * 4 * 8 * nx_,
                   [&] { return arnoldi_edge_halo_launch(A, pa, yh_, E_.s); });
    if (rc) return rc;
  } else {
    rc = E_.launch(K_ARN_EDGE, eb, [&] { return arnoldi_edge_launch(A, y4_, E_.s); });
    if (rc) return rc;
    rc = E_.launch(K_HALO, 2.0 * 4 * 8 * nx_, [&] {
      return E_.comm->halo(y4_, yh_, yh_ + 2 * nx_, 4, nx_, E_.s) == NK_OK ? hipSuccess
                                                                         : hipErrorUnknown;
    });
    if (rc) return NK_ECOMM;
  }
  if (!split) {
    A.yh = yh_;
    with_tail();
    return E_.launch(K_ARNOLDI, rowb * ny_, [&] { return arnoldi_launch(A, E_.s, nwaves); });
  }
  T.yh = Bm.yh = yh_;
  int64_t nw = 0;
  rc = E_.launch(K_ARN_SLAB, rowb * 4, [&] {
    hipError_t e = arnoldi_launch(T, E_.s, &nw);
    if (e == hipSuccess) e = arnoldi_launch(Bm, E_.s, &nw);
    if (e == hipSuccess) e = hipStreamWaitEvent(E_.s, ev_out_, 0);
    return e;
  });
  *nwaves = nwI + nwT + nwB;
  return rc;
}

void SHProblem::void_fused_steps(int count) {
  E_.void_last(K_ARNOLDI, count);
  if (dist() && edge_launched_) E_.void_last(K_ARN_EDGE, count);
  if (last_split_) E_.void_last(K_ARN_SLAB, count);
}

// The edge array of a stencil pass's output, written by the pass itself (when the fused kernel
// will read block halos from it): TRIAL's F becomes V_0, the JVP's w the next update entry.
void SHProblem::set_edges(StencilArgs* A, const double* out) {
  if (!has_fused(1)) return;
  A->E0 = E_.edges(out);
  A->e_ny = ny_;
  A->e_row0 = 0;
  if (A->E0) E_.mark_edges(out);
}

// The stencil fields' side columns from their edge arrays, where every writer of the field keeps
// them (NKHIP_EDGES=0, read per call, reads the neighbouring blocks' lines instead)
void SHProblem::side_edges(StencilArgs* A, const double* a, const double* b) const {
  const char* e = std::getenv("NKHIP_EDGES");
  if (!has_fused(1) || (e && e[0] == '0')) return;
  A->e_ny = ny_;
  A->e_row0 = 0;
  if (a && E_.edges_kept(a)) A->Ea = E_.edges(a);
  if (b && E_.edges_kept(b)) A->Eb = E_.edges(b);
}

int SHProblem::publish_edges(const double* v, bool written) {
  if (!has_fused(1)) return NK_OK;
  const int rc = written ? NK_OK : E_.gather_edges(v);
  return rc ? rc : push(v);
}

EdgeOut SHProblem::edge_out(const double* v) {
  const char* e = std::getenv("NKHIP_COMBO_EDGES");  // 0: an edge_gather pass after each
  if (!has_fused(1) || (e && e[0] == '0')) return EdgeOut{};
  return E_.edge_out(v);
}

// ============================================================================================
// CallbackProblem
// ============================================================================================
CallbackProblem::CallbackProblem(Engine& E, nk_residual_fn F, void* ctx, double* tmp, double* tmp2)
    : E_(E), F_(F), ctx_(ctx), tmp_(tmp), tmp2_(tmp2) {}

int CallbackProblem::norms(double* v, double* sum2, double* vmax) {
  VecList none;
  int64_t nblk = 0;
  int rc = E_.launch(K_COMBO, 16.0 * E_.n, [&] {
    return combo_launch(tmp2_, v, 1.0, none, 0, E_.n, E_.partial(), E_.s, &nblk);
  });
  if (rc) return rc;
  double red[2];
  rc = E_.reduce(nblk, 1, 2, red);
  *sum2 = red[0];
  *vmax = red[1];
  return rc;
}

int CallbackProblem::eval(const double* x, const double* p, double alpha, double* xt, double* F,
                          double* G, double red[3]) {
  const int64_t n = E_.n;
  const double* xe = x;
  if (xt || alpha != 0.0) {
    double* dst = xt ? xt : tmp_;
    int rc = E_.launch(K_AXPBY, 24.0 * n,
                       [&] { return axpby_launch(1.0, x, alpha, p, dst, n, E_.s); });
    if (rc) return rc;
    xe = dst;
  }
  int rc = E_.launch(K_USERF, 0.0, [&] {
    return F_(ctx_, xe, F, n) == 0 ? hipSuccess : hipErrorUnknown;
  });
  if (rc) return rc;
  double s2 = 0, fm = 0, xs = 0, xm = 0;
  rc = norms(F, &s2, &fm);
  if (!rc) rc = norms(const_cast<double*>(xe), &xs, &xm);
  if (rc) return rc;
  red[0] = s2;
  red[1] = fm;
  red[2] = xm;
  if (G != F) rc = E_.copy(G, F, n);
  return rc;
}

int CallbackProblem::jvp(const double* x0, const double* G0, const double* z, double zs, double sc,
                         double* w) {
  const int64_t n = E_.n;
  int rc = E_.launch(K_AXPBY, 24.0 * n,
                     [&] { return axpby_launch(1.0, x0, sc * zs, z, tmp_, n, E_.s); });
  if (rc) return rc;
  rc = E_.launch(K_USERF, 0.0, [&] {
    return F_(ctx_, tmp_, w, n) == 0 ? hipSuccess : hipErrorUnknown;
  });
  if (rc) return rc;
  return E_.launch(K_AXPBY, 24.0 * n, [&] { return fddiff_launch(w, G0, sc, n, E_.s); });
}

}  // namespace nk

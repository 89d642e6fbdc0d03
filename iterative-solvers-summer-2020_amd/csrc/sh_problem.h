// Problems handed to the Newton-Krylov core: the fused Swift-Hohenberg stepper (north-star path)
// and a generic device residual supplied through a C callback (the newton_krylov drop-in).
#pragma once

#include "nk_solver.h"

namespace nk {

// Crank-Nicolson Swift-Hohenberg residual on one row slab (sh_scipy_nk.py:47-49 / main.cpp:19-32),
// F(u) = G(u) + B with G(u) = u/k - (L u + g u^2 - u^3)/2 and B = -Uo/k - (L Uo + g Uo^2 - Uo^3)/2
// hoisted once per time step (the reference recomputes L@Uo on every call).
class SHProblem final : public Problem {
 public:
  SHProblem(Engine& E, int64_t ny, int64_t nx, int64_t ny_global, SHCoef c, int jvp_mode);
  ~SHProblem() override;
  int status() const { return status_; }
  void set_jvp_mode(int m) { jvp_mode_ = m; }
  int64_t n_global() const override { return ny_g_ * nx_; }
  int prepare(const double* u_prev);  // B <- B(u_prev)
  int eval(const double* x, const double* p, double alpha, double* xt, double* F, double* G,
           double red[3]) override;
  int jvp(const double* x0, const double* G0, const double* z, double zs, double sc,
          double* w) override;
  bool has_dev_scale() const override { return true; }
  bool can_spec_jvp() const override;
  void arm_spec(const SpecJvp* sp) override { spec_ = sp ? *sp : SpecJvp{}; }
  int jvp_dev(const double* x0, const double* G0, const double* z, const double* znorm2,
              double omega, double* w) override;
  bool has_fused(int nv) const override;
  int fused_step(const double* const* V, const double* c, int nv, const double* w, double tau,
                 const double* x0, const double* G0, const double* z, double zs, double sc,
                 double* out_v, double* out_w, int64_t* nwaves, const double* ctl,
                 const ArnTail* tail = nullptr, bool* tail_used = nullptr) override;
  int set_x0(const double* x0) override;
  int set_dir(const double* d) override;
  int publish_edges(const double* v, bool written = false) override;
  EdgeOut edge_out(const double* v) override;
  void set_edges(StencilArgs* A, const double* out);
  void side_edges(StencilArgs* A, const double* a, const double* b) const;
  void void_fused_steps(int count) override;

 private:
  // any communicator (also a world of one: its halo is the periodic wrap through RCCL)
  bool dist() const { return E_.comm != nullptr; }
  Field field(const double* p, const double* halo) const;
  int halo(const double* v, double* h);
  // the JVP pass on a slab: halo of z + stencil; interior rows overlap the exchange
  int halo_stencil(int kind, SMode m, const StencilArgs& A, const double* z, double* zh);
  // pushed halo rows (arnoldi.hip): on when the communicator lent this stepper its halo slots
  // (NKHIP_SLAB_PUSH=0, read per call, turns it off)
  bool push_mode() const;
  double* slot(double* base, const double* v) const;  // v's halo slot in a slot region
  int push(const double* v);  // v's edge rows into the neighbours' slots (push_rows_launch)
  void pushed(const double* v);  // v's rows went out now (records the all-reduce epoch)
  void set_push(StencilArgs* A, const double* out0, const double* out2);
  // v's halo rows as a stencil field's halo (4 rows: lo, hi) straight from this rank's slot, when
  // the rows were pushed before an all-reduce already issued; nullptr: exchange them
  const double* slot_halo(const double* v) const;
  Engine& E_;
  int64_t ny_, nx_, ny_g_;
  SHCoef c_;
  int jvp_mode_;
  int status_ = NK_OK;
  double* B_ = nullptr;
  SpecJvp spec_{};        // armed speculative JVP (z == nullptr: none), issued by the next eval
  double* hx_ = nullptr;  // halos (4 rows each: lo = rows -2,-1 ; hi = rows ny, ny+1)
  double* hz_ = nullptr;
  double* hd_ = nullptr;
  double* hu_ = nullptr;
  double* y4_ = nullptr;  // fused Arnoldi step: u on this slab's edge rows 0, 1, ny-2, ny-1
  double* yh_ = nullptr;  // ... and on the halo rows -2, -1, ny, ny+1 from the neighbours
  int64_t ny_min_ = 0, ny_max_ = 0;  // smallest / largest slab over the ranks
  hipStream_t side_ = nullptr;       // interior rows of the JVP while the halo is in flight
  hipEvent_t ev_in_ = nullptr, ev_out_ = nullptr;
  double* mb_ = nullptr;  // the fused kernel's block-halo mailbox (arnoldi.hip)
  int64_t mb_cap_ = 0;
  uint64_t mb_tag_ = 0;   // one tag per fused launch
  bool last_split_ = false;  // the last fused step ran as interior + edge-band launches
  bool edge_launched_ = false;  // the last fused step launched the slab edge kernel
  nk_halo_slots slots_{};       // claimed from the communicator (mine == nullptr: none)
  std::vector<uint64_t> push_ep_;  // per pool vector: comm epoch of its last push (~0: none)
  const double* hxp_ = nullptr;  // the halo of the current x0 / direction (hx_ / hd_ or a slot)
  const double* hdp_ = nullptr;
};

// newton_krylov(F, xin) for an arbitrary device residual (droplet.py:383, PMA2_nk.py:100, ...):
// the FD Jacobian of KrylovJacobian.matvec built from F evaluations.
class CallbackProblem final : public Problem {
 public:
  CallbackProblem(Engine& E, nk_residual_fn F, void* ctx, double* tmp, double* tmp2);
  int64_t n_global() const override { return E_.n; }
  int eval(const double* x, const double* p, double alpha, double* xt, double* F, double* G,
           double red[3]) override;
  int jvp(const double* x0, const double* G0, const double* z, double zs, double sc,
          double* w) override;
  bool may_speculate() const override { return false; }  // scipy calls F exactly nfev + njvp times

 private:
  int norms(double* v, double* sum2, double* vmax);
  Engine& E_;
  nk_residual_fn F_;
  void* ctx_;
  double* tmp_;
  double* tmp2_;
};

}  // namespace nk

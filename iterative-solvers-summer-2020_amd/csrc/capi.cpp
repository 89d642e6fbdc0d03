// extern "C" boundary of libnkhip (declared in include/nkhip.h).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <memory>
#include <new>
#include <vector>

#include "../../include/nkhip.h"
#include "comm.h"
#include "nk_kernels.h"
#include "nk_solver.h"
#include "droplet_problem.h"
#include "mems_problem.h"
#include "sh_problem.h"
#include "shlin.h"

using namespace nk;

namespace {

hipStream_t S(void* s) { return static_cast<hipStream_t>(s); }

int hip_rc(hipError_t e) {
  if (e == hipSuccess) return NK_OK;
  std::fprintf(stderr, "nkhip: HIP error %d (%s)\n", int(e), hipGetErrorString(e));
  return NK_EHIP;
}

// Runs a kernel that leaves per-block partials, then reduces them into host `out`.
template <class L>
int reduce_call(int64_t n, int nslots, int nsum, int nv, double* out, hipStream_t s, L&& fn) {
  const int64_t kb = krylov_blocks(n) + 1;
  double* buf = nullptr;
  const size_t bytes = sizeof(double) * (size_t(kb) * nslots + nv);
  hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&buf), bytes, s);
  if (e != hipSuccess) return hip_rc(e);
  int64_t nblk = 0;
  e = fn(buf, &nblk);
  double* res = buf + size_t(kb) * nslots;
  if (e == hipSuccess) e = reduce_final_launch(buf, nblk, nsum, nv, res, nullptr, s);
  if (e == hipSuccess) e = hipMemcpyAsync(out, res, sizeof(double) * nv, hipMemcpyDeviceToHost, s);
  hipFreeAsync(buf, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  return hip_rc(e);
}

}  // namespace

struct nk_sh {
  std::unique_ptr<Engine> E;
  std::unique_ptr<SHProblem> P;
  std::unique_ptr<NewtonKrylov> NK;
  nk_opts opts;
  int64_t ny, nx;
};

extern "C" {

const char* nk_version(void) { return "nkhip 0.3.0 (gfx950)"; }
int nk_abi_version(void) { return NKHIP_ABI_VERSION; }

int nk_opts_default(nk_opts* o) {
  if (!o) return NK_EINVAL;
  *o = default_opts();
  return NK_OK;
}

const char* nk_status_string(int code) {
  switch (code) {
    case NK_OK: return "ok";
    case NK_NO_CONVERGENCE: return "no convergence (maxiter reached)";
    case NK_NONFINITE: return "Function returned non-finite results";
    case NK_ZERO_STEP:
      return "Jacobian inversion yielded zero vector. This indicates a bug in the Jacobian "
             "approximation.";
    case NK_BAD_RHS: return "RHS must contain only finite numbers";
    case NK_EINVAL: return "invalid argument";
    case NK_EHIP: return "HIP runtime error";
    case NK_ECOMM: return "RCCL error";
    case NK_ENOMEM: return "out of device memory";
  }
  return "unknown status";
}

// ------------------------------------------------------------------------------ operators
int nk_lap5_apply(const double* v, double* y, int64_t ny, int64_t nx, double e, void* stream) {
  if (!v || !y || ny <= 0 || nx <= 0) return NK_EINVAL;
  StencilArgs A;
  A.ny = ny;
  A.nx = nx;
  A.a = periodic(v);
  A.out0 = y;
  A.e = e;
  return hip_rc(stencil_launch(SMode::LAP5, A, S(stream), nullptr));
}

int nk_sh13_apply(const double* v, double* y, int64_t ny, int64_t nx, double h, double r,
                  void* stream) {
  if (!v || !y || ny <= 0 || nx <= 0) return NK_EINVAL;
  StencilArgs A;
  A.ny = ny;
  A.nx = nx;
  A.a = periodic(v);
  A.out0 = y;
  A.c = sh_coef(h, r, 1.0, 0.0);
  return hip_rc(stencil_launch(SMode::SH13, A, S(stream), nullptr));
}

int nk_sh_residual(const double* u, const double* uo, double* F, int64_t ny, int64_t nx, double h,
                   double r, double k, double g, void* stream) {
  if (!u || !uo || !F || ny <= 0 || nx <= 0) return NK_EINVAL;
  StencilArgs A;
  A.ny = ny;
  A.nx = nx;
  A.a = periodic(u);
  A.b = periodic(uo);
  A.out0 = F;
  A.c = sh_coef(h, r, k, g);
  return hip_rc(stencil_launch(SMode::RESID, A, S(stream), nullptr));
}

int nk_sh_jvp(const double* u, const double* v, double* y, int64_t ny, int64_t nx, double h,
              double r, double k, double g, void* stream) {
  if (!u || !v || !y || ny <= 0 || nx <= 0) return NK_EINVAL;
  StencilArgs A;
  A.ny = ny;
  A.nx = nx;
  A.a = periodic(v);
  A.p0 = u;
  A.alpha = 1.0;
  A.out0 = y;
  A.c = sh_coef(h, r, k, g);
  return hip_rc(stencil_launch(SMode::AJVP, A, S(stream), nullptr));
}

int nk_sh_fdjvp(const double* x0, const double* G0, const double* z, double* y, int64_t ny,
                int64_t nx, double h, double r, double k, double g, double zs, double sc,
                void* stream) {
  if (!x0 || !G0 || !z || !y || ny <= 0 || nx <= 0 || !(sc != 0.0)) return NK_EINVAL;
  StencilArgs A;
  A.ny = ny;
  A.nx = nx;
  A.a = periodic(x0);
  A.b = periodic(z);
  A.alpha = sc * zs;
  A.sc = sc;
  A.p0 = G0;
  A.out0 = y;
  A.c = sh_coef(h, r, k, g);
  return hip_rc(stencil_launch(SMode::FDJVP, A, S(stream), nullptr));
}

namespace {
// the mailbox of the kernel-level entry points (one buffer for every caller; a launch on another
// stream that overwrites records only sends consumers to their recompute path)
int attach_mbox(ArnoldiArgs& A) {
  const int mode = arnoldi_mbox_mode();
  if (mode == 0) return NK_OK;
  static std::mutex mu;
  static double* buf = nullptr;
  static int64_t cap = 0;
  static uint64_t tag = 0;
  // grow-only: a buffer once handed out is never freed (another thread may be about to launch
  // with it after this lock is released); the outgrown ones are kept until process exit
  static std::vector<double*> retired;
  std::lock_guard<std::mutex> lk(mu);
  const int64_t need = arnoldi_mbox_elems(A.ny, A.nx);
  if (cap < need) {
    if (buf) retired.push_back(buf);
    buf = nullptr;
    cap = 0;
    if (hipMalloc(reinterpret_cast<void**>(&buf), sizeof(double) * need) != hipSuccess)
      return NK_ENOMEM;
    if (hipMemset(buf, 0, sizeof(double) * need) != hipSuccess) return NK_EHIP;
    cap = need;
  }
  A.mb = buf;
  A.mb_cap = cap;
  A.mb_tag = ++tag;
  A.mb_recompute = mode == 2;
  return NK_OK;
}

int arnoldi_fused_call(const double* const* V, const double* const* E, const double* coef,
                       int32_t nv, const double* w, double tau, const double* x0, const double* G0,
                       const double* z, int64_t ny, int64_t nx, double h, double r, double k,
                       double g, double zs, double sc, double* v_out, double* w_out,
                       double* Ev_out, double* Ew_out, double* dots, void* stream) {
  // G0 is not read (closed-form difference quotient) and may be NULL
  if (!V || !coef || !w || !x0 || !v_out || !w_out || !(sc != 0.0)) return NK_EINVAL;
  if (!arnoldi_supported(nv, ny, nx)) return NK_EINVAL;
  ArnoldiArgs A;
  if (E) {
    for (int i = 0; i <= nv; ++i) {
      if (!E[i]) return NK_EINVAL;
      A.E[i] = E[i];
    }
  }
  A.Eout_v = Ev_out;
  A.Eout_w = Ew_out;
  A.ny = ny;
  A.nx = nx;
  A.nv = nv;
  for (int i = 0; i < nv; ++i) {
    if (!V[i]) return NK_EINVAL;
    A.V[i] = V[i];
    A.c[i] = coef[i];
  }
  A.w = w;
  A.tau = tau;
  A.x0 = x0;
  A.g0 = G0;
  A.z = z;
  A.alpha = sc * zs;
  A.sc = sc;
  A.k = sh_coef(h, r, k, g);
  A.out_v = v_out;
  A.out_w = w_out;
  if (int rc = attach_mbox(A)) return rc;
  const int nval = 2 * nv + 3;
  if (!dots) {  // no reduction wanted (timing): a persistent partial buffer, no synchronisation
    static std::mutex mu;  // the buffer is shared by every caller thread
    std::lock_guard<std::mutex> lk(mu);
    static double* buf = nullptr;
    static int64_t cap = 0;
    const int64_t need = int64_t(nval) * 65536;
    if (cap < need) {
      if (buf) hipFree(buf);
      buf = nullptr;
      cap = 0;
      if (hipMalloc(reinterpret_cast<void**>(&buf), sizeof(double) * need) != hipSuccess)
        return NK_ENOMEM;
      cap = need;
    }
    A.partial = buf;
    A.partial_cap = cap;
    int64_t nw = 0;
    return hip_rc(arnoldi_launch(A, S(stream), &nw));
  }
  return reduce_call(int64_t(65536) * 2048, nval, nval, nval, dots, S(stream),
                     [&](double* part, int64_t* nb) {
                       A.partial = part;
                       A.partial_cap = int64_t(nval) * (65536 + 1);
                       return arnoldi_launch(A, S(stream), nb);
                     });
}
}  // namespace

int64_t nk_arnoldi_mbox_launches(void) { return arnoldi_mbox_launches(); }

int nk_sh_arnoldi_fused(const double* const* V, const double* coef, int32_t nv, const double* w,
                        double tau, const double* x0, const double* G0, const double* z,
                        int64_t ny, int64_t nx, double h, double r, double k, double g, double zs,
                        double sc, double* v_out, double* w_out, double* dots, void* stream) {
  return arnoldi_fused_call(V, nullptr, coef, nv, w, tau, x0, G0, z, ny, nx, h, r, k, g, zs, sc,
                            v_out, w_out, nullptr, nullptr, dots, stream);
}

int nk_sh_arnoldi_fused_edges(const double* const* V, const double* const* E, const double* coef,
                              int32_t nv, const double* w, double tau, const double* x0,
                              const double* G0, const double* z, int64_t ny, int64_t nx, double h,
                              double r, double k, double g, double zs, double sc, double* v_out,
                              double* w_out, double* Ev_out, double* Ew_out, double* dots,
                              void* stream) {
  if (!E) return NK_EINVAL;
  return arnoldi_fused_call(V, E, coef, nv, w, tau, x0, G0, z, ny, nx, h, r, k, g, zs, sc, v_out,
                            w_out, Ev_out, Ew_out, dots, stream);
}

int64_t nk_edge_elems(int64_t ny, int64_t nx) {
  return (ny > 0 && nx > 0) ? edge_elems(ny, nx) : NK_EINVAL;
}

int nk_edge_gather(const double* v, double* E, int64_t ny, int64_t nx, void* stream) {
  if (!v || !E || ny < 1 || nx < 4 || nx % 2) return NK_EINVAL;
  return hip_rc(edge_gather_launch(v, E, ny, nx, S(stream)));
}

// ------------------------------------------------------------------------------ BLAS-1
int nk_dot(const double* x, const double* y, int64_t n, double* out, void* stream) {
  if (!x || !y || !out || n < 0) return NK_EINVAL;
  VecList P;
  P.p[0] = y;
  return reduce_call(n, 3, 3, 1, out, S(stream), [&](double* part, int64_t* nb) {
    return mdot_launch(x, nullptr, P, 1, n, part, S(stream), nb);
  });
}

int nk_nrm2(const double* x, int64_t n, double* out, void* stream) {
  if (!x || !out || n < 0) return NK_EINVAL;
  double s2 = 0.0;
  VecList P;
  P.p[0] = x;
  const int rc = reduce_call(n, 3, 3, 1, &s2, S(stream), [&](double* part, int64_t* nb) {
    return mdot_launch(x, nullptr, P, 1, n, part, S(stream), nb);
  });
  *out = std::sqrt(s2);
  return rc;
}

int nk_maxnorm(const double* x, int64_t n, double* out, void* stream) {
  if (!x || !out || n <= 0) return NK_EINVAL;
  // combo with no vectors: out = 1*x (written to scratch), partial [sum x^2, max|x|]
  double* tmp = nullptr;
  hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&tmp), sizeof(double) * n, S(stream));
  if (e != hipSuccess) return hip_rc(e);
  VecList none;
  double r2[2];
  const int rc = reduce_call(n, 2, 1, 2, r2, S(stream), [&](double* part, int64_t* nb) {
    return combo_launch(tmp, x, 1.0, none, 0, n, part, S(stream), nb);
  });
  hipFreeAsync(tmp, S(stream));
  hipStreamSynchronize(S(stream));
  *out = r2[1];
  return rc;
}

int nk_axpy(double a, const double* x, double* y, int64_t n, void* stream) {
  if (!x || !y || n < 0) return NK_EINVAL;
  return hip_rc(axpby_launch(a, x, 1.0, y, y, n, S(stream)));
}

int nk_scal(double a, double* x, int64_t n, void* stream) {
  if (!x || n < 0) return NK_EINVAL;
  return hip_rc(axpby_launch(a, x, 0.0, nullptr, x, n, S(stream)));
}

int nk_mdot(const double* const* V, int32_t m, const double* w, int64_t n, double* out,
            void* stream) {
  if (!V || !w || !out || m < 0 || m > kMaxVec || n < 0) return NK_EINVAL;
  if (m == 0) return NK_OK;
  VecList P;
  for (int i = 0; i < m; ++i) P.p[i] = V[i];
  const int nv = 2 * m + 1;
  double res[2 * kMaxVec + 1];
  const int rc = reduce_call(n, nv, nv, nv, res, S(stream), [&](double* part, int64_t* nb) {
    return mdot_launch(w, nullptr, P, m, n, part, S(stream), nb);
  });
  for (int i = 0; i < m; ++i) out[i] = res[i];
  return rc;
}

int nk_maxpy(const double* const* V, const double* coef, int32_t m, double* y, int64_t n,
             void* stream) {
  if (!V || !coef || !y || m < 0 || m > kMaxVec || n < 0) return NK_EINVAL;
  VecList P;
  for (int i = 0; i < m; ++i) {
    P.p[i] = V[i];
    P.c[i] = coef[i];
  }
  int64_t nb = 0;
  return hip_rc(combo_launch(y, y, 1.0, P, m, n, nullptr, S(stream), &nb));
}

int nk_stream_copy(const double* src, double* dst, int64_t n, void* stream) {
  if (!src || !dst || n < 0) return NK_EINVAL;
  return hip_rc(stream_copy_launch(src, dst, n, S(stream)));
}

int nk_debug_bounds(int64_t* violations, int32_t* first_line, int32_t reset) {
  const int rc = arnoldi_check_counters(violations, first_line, reset != 0);
  return rc == 0 ? NK_OK : (rc == -1 ? NK_EINVAL : NK_EHIP);
}

int nk_debug_mailbox(int64_t* counts, int32_t reset) {
  if (!counts) return NK_EINVAL;
  const int rc = arnoldi_mailbox_counters(counts, reset != 0);
  return rc == 0 ? NK_OK : (rc == -1 ? NK_EINVAL : NK_EHIP);
}

// ------------------------------------------------------------------------------ comms
int nk_comm_unique_id_bytes(void) { return comm_unique_id_bytes(); }
int nk_comm_get_unique_id(void* out) { return out ? comm_get_unique_id(out) : NK_EINVAL; }
int nk_comm_create_rccl(nk_comm** out, const void* uid, int32_t rank, int32_t nranks) {
  return comm_create_rccl(out, uid, rank, nranks);
}
int nk_comm_create_loopback(nk_comm** out, int32_t nranks) {
  return comm_create_loopback(out, nranks);
}
int nk_comm_peer_handle_bytes(void) { return comm_peer_handle_bytes(); }
int nk_comm_create_peer(nk_comm** out, int32_t rank, int32_t nranks, int64_t max_nx,
                        void* handle_out) {
  return comm_create_peer(out, rank, nranks, max_nx, handle_out);
}
int nk_comm_peer_connect(nk_comm* c, const void* handles) { return comm_peer_connect(c, handles); }
int nk_comm_destroy(nk_comm* c) {
  delete c;
  return NK_OK;
}
int nk_comm_abort(nk_comm* c) {
  if (!c) return NK_EINVAL;
  c->abort();
  return NK_OK;
}

// One all-reduce and one halo exchange of known values through the communicator, checked on the
// host: every rank contributes (rank + 1 + i) to the sums and (rank + i) to the maxima, and a
// 4-row slab whose entries encode (rank, row, column).
int nk_comm_selftest(nk_comm* c, int64_t nx, void* stream) {
  if (!c || nx < 1) return NK_EINVAL;
  const hipStream_t s = S(stream);
  const int P = c->size(), r = c->rank();
  constexpr int kV = 8, kSum = 5;
  const int64_t nslab = 4 * nx, nhalo = 4 * nx;
  std::vector<double> h(kV + nslab + nhalo);
  for (int i = 0; i < kV; ++i) h[i] = (i < kSum) ? r + 1.0 + i : r + double(i);
  auto code = [&](int q, int64_t row, int64_t j) { return 1e6 * q + double(row * nx + j); };
  for (int64_t row = 0; row < 4; ++row)
    for (int64_t j = 0; j < nx; ++j) h[kV + row * nx + j] = code(r, row, j);
  double* d = nullptr;
  if (hipMalloc(reinterpret_cast<void**>(&d), h.size() * sizeof(double)) != hipSuccess)
    return NK_EHIP;
  int rc = hipMemcpyAsync(d, h.data(), (kV + nslab) * sizeof(double), hipMemcpyHostToDevice, s) ==
                   hipSuccess
               ? NK_OK
               : NK_EHIP;
  if (!rc) rc = c->allreduce(d, kSum, kV, s);
  if (!rc) rc = c->halo(d + kV, d + kV + nslab, d + kV + nslab + 2 * nx, 4, nx, s);
  if (!rc && (hipMemcpyAsync(h.data(), d, h.size() * sizeof(double), hipMemcpyDeviceToHost, s) !=
                  hipSuccess ||
              hipStreamSynchronize(s) != hipSuccess))
    rc = NK_EHIP;
  (void)hipFree(d);
  if (rc) return rc;
  if (c->failed()) return NK_ECOMM;
  for (int i = 0; i < kV; ++i) {
    const double want = (i < kSum) ? P * (P + 1) / 2.0 + double(P) * i : (P - 1.0) + i;
    if (h[i] != want) return NK_ECOMM;
  }
  const int prev = (r - 1 + P) % P, next = (r + 1) % P;
  const double* lo = h.data() + kV + nslab;
  const double* hi = lo + 2 * nx;
  for (int64_t row = 0; row < 2; ++row)
    for (int64_t j = 0; j < nx; ++j)
      if (lo[row * nx + j] != code(prev, 2 + row, j) || hi[row * nx + j] != code(next, row, j))
        return NK_ECOMM;
  return NK_OK;
}

namespace {
// plain global loads, as the fused kernel's edge bands read the halo slots (slab_push_prologue)
__global__ void slot_read_kernel(const double* src, double* dst, int64_t n) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}
}  // namespace

// The pushed-halo-rows protocol exactly as the solver runs it (arnoldi.hip "Pushed halo rows"):
// every rank clears its own slots, passes an all-reduce, pushes a 4-row slab of known codes into
// its ring neighbours' slots with push_rows_launch (system-scope fence, no flag), passes ONE
// all-reduce, then reads its own slots back with plain loads in a kernel and checks them on the
// host -- rows 0, 1 the previous rank's rows ny-2, ny-1, rows 2, 3 the next rank's rows 0, 1.
// Slots 0 and count-1 are checked.  NKHIP_PEER_SELFTEST_BREAK_PUSH=<rank>: that rank pushes
// wrong codes (fault injection for the fallback path).
int nk_comm_selftest_push(nk_comm* c, int64_t nx, void* stream) {
  if (!c || nx < 1) return NK_EINVAL;
  const hipStream_t s = S(stream);
  nk_halo_slots sl;
  static const char owner = 0;  // a claim of its own: refused while a stepper holds the slots
  const bool claimed = c->claim_slots(&owner, &sl);
  struct Release {
    nk_comm* c;
    bool on;
    ~Release() {
      if (on) c->release_slots(&owner);
    }
  } rel{c, claimed};
  const bool have = claimed && sl.ld >= nx && sl.count >= 1;
  const int P = c->size(), r = c->rank();
  const int64_t ny = 4;
  const int64_t slots[2] = {0, sl.count - 1};
  const char* be = std::getenv("NKHIP_PEER_SELFTEST_BREAK_PUSH");
  const bool broken = be && *be && std::atoi(be) == r;
  auto code = [&](int q, int64_t slot, int64_t row, int64_t j) {
    return 1e9 * (q + 1) + 1e6 * slot + double(row * nx + j);
  };
  const int64_t nslot = have ? 4 * sl.ld : 0;
  std::vector<double> h(2 * ny * nx + 2 * nslot + 2);
  h[2 * ny * nx + 2 * nslot] = have ? 0.0 : 1.0;  // max over ranks: some rank has no slots
  double* d = nullptr;
  if (hipMalloc(reinterpret_cast<void**>(&d), h.size() * sizeof(double)) != hipSuccess)
    return NK_EHIP;
  double* vsrc = d;                  // [2][ny][nx] the pushed slabs
  double* rd = d + 2 * ny * nx;      // [2][4][ld] the slots read back
  double* ar = rd + 2 * nslot;       // 2 values for the all-reduces
  for (int k = 0; k < 2; ++k)
    for (int64_t row = 0; row < ny; ++row)
      for (int64_t j = 0; j < nx; ++j)
        h[(k * ny + row) * nx + j] = code(r, slots[k], row, j) + (broken ? 0.5 : 0.0);
  int rc = NK_OK;
  auto ok = [&](hipError_t e) {
    if (!rc && e != hipSuccess) rc = NK_EHIP;
  };
  for (int k = 0; k < 2 && have; ++k)
    ok(hipMemsetAsync(sl.mine + slots[k] * 4 * sl.ld, 0xff, sizeof(double) * nslot, s));  // NaN
  ok(hipMemcpyAsync(d, h.data(), sizeof(double) * (2 * ny * nx + 2 * nslot + 2),
                    hipMemcpyHostToDevice, s));
  // every rank cleared its slots before any pushes, and every rank has slots
  if (!rc) rc = c->allreduce(ar, 0, 2, s);
  double any_without = 1.0;
  if (!rc && (hipMemcpyAsync(&any_without, ar, sizeof(double), hipMemcpyDeviceToHost, s) !=
                  hipSuccess ||
              hipStreamSynchronize(s) != hipSuccess))
    rc = NK_EHIP;
  if (!rc && any_without != 0.0) rc = NK_EINVAL;  // on every rank alike: nothing to check
  for (int k = 0; k < 2 && !rc; ++k)
    ok(push_rows_launch(vsrc + k * ny * nx, sl.prev + slots[k] * 4 * sl.ld,
                        sl.next + slots[k] * 4 * sl.ld, ny, nx, sl.ld, s));
  if (!rc) rc = c->allreduce(ar, 1, 2, s);  // the one all-reduce that orders the pushes
  for (int k = 0; k < 2 && !rc; ++k) {
    hipLaunchKernelGGL(slot_read_kernel, dim3(unsigned((nslot + 255) / 256)), dim3(256), 0, s,
                       sl.mine + slots[k] * 4 * sl.ld, rd + k * nslot, nslot);
    ok(hipGetLastError());
  }
  if (!rc && (hipMemcpyAsync(h.data(), rd, sizeof(double) * 2 * nslot, hipMemcpyDeviceToHost, s) !=
                  hipSuccess ||
              hipStreamSynchronize(s) != hipSuccess))
    rc = NK_EHIP;
  (void)hipFree(d);
  if (rc) return rc;
  if (c->failed()) return NK_ECOMM;
  const int prev = (r - 1 + P) % P, next = (r + 1) % P;
  for (int k = 0; k < 2; ++k) {
    const double* m = h.data() + k * nslot;
    for (int64_t row = 0; row < 4; ++row)
      for (int64_t j = 0; j < nx; ++j) {
        const double want = row < 2 ? code(prev, slots[k], ny - 2 + row, j)
                                    : code(next, slots[k], row - 2, j);
        if (m[row * sl.ld + j] != want) return NK_ECOMM;
      }
  }
  return NK_OK;
}

// ------------------------------------------------------------------------------ SH stepper
int nk_sh_create(nk_sh** out, int64_t ny_local, int64_t nx, int64_t ny_global, double h, double r,
                 double k, double g, const nk_opts* opts, nk_comm* comm, void* stream) {
  if (!out || ny_local <= 0 || nx <= 0 || ny_global < ny_local || !(h > 0) || !(k != 0))
    return NK_EINVAL;
  if (comm && comm->size() > 1 && ny_local < 2) return NK_EINVAL;
  if ((!comm || comm->size() == 1) && ny_global != ny_local) return NK_EINVAL;
  std::unique_ptr<nk_sh> sh(new (std::nothrow) nk_sh());
  if (!sh) return NK_ENOMEM;
  sh->opts = opts ? *opts : default_opts();
  sh->ny = ny_local;
  sh->nx = nx;
  sh->E = std::make_unique<Engine>(ny_local * nx, comm, S(stream), sh->opts.profile > 0,
                                   stencil_partial_slots(ny_local, nx));
  sh->E->sample = sh->opts.profile > 1 ? sh->opts.profile : 1;
  sh->P = std::make_unique<SHProblem>(*sh->E, ny_local, nx, ny_global, sh_coef(h, r, k, g),
                                      sh->opts.jvp_mode);
  if (sh->P->status()) return sh->P->status();
  sh->NK = std::make_unique<NewtonKrylov>(*sh->E, *sh->P, sh->opts);
  if (sh->NK->status()) return sh->NK->status();
  const int rc = sh->E->sync();
  if (rc) return rc;
  *out = sh.release();
  return NK_OK;
}

int nk_sh_destroy(nk_sh* s) {
  delete s;
  return NK_OK;
}

int nk_sh_set_opts(nk_sh* s, const nk_opts* opts) {
  if (!s || !opts) return NK_EINVAL;
  if (opts->inner_m != s->opts.inner_m || opts->outer_k != s->opts.outer_k) return NK_EINVAL;
  s->opts = *opts;
  s->E->profile = opts->profile > 0;
  s->E->sample = opts->profile > 1 ? opts->profile : 1;
  s->P->set_jvp_mode(opts->jvp_mode);
  s->NK->set_opts(*opts);
  return NK_OK;
}

int nk_sh_step(nk_sh* s, const double* u_prev, double* u_next, nk_stats* stats) {
  if (!s || !u_prev || !u_next) return NK_EINVAL;
  int rc = s->P->prepare(u_prev);
  if (!rc) rc = s->NK->solve(u_prev, u_next, stats);
  // a failed rank must not leave its peers waiting in the next collective
  if (rc < 0 && s->E->comm) s->E->comm->abort();
  return rc;
}

int nk_sh_kernel_profile(nk_sh* s, nk_kprof* out, int32_t max) {
  if (!s) return NK_EINVAL;
  for (int k = 0; k < K_NKINDS && k < max; ++k) {
    std::memset(out[k].name, 0, sizeof(out[k].name));
    std::strncpy(out[k].name, kind_name(k), sizeof(out[k].name) - 1);
    out[k].launches = s->E->stat(k).launches;
    out[k].total_ms = s->E->stat(k).ms;
    out[k].alg_bytes = s->E->stat(k).bytes;
    out[k].timed = s->E->stat(k).timed;
    out[k].timed_bytes = s->E->stat(k).tbytes;
  }
  return K_NKINDS;
}

int nk_sh_reset_profile(nk_sh* s) {
  if (!s) return NK_EINVAL;
  s->E->reset_stats();
  return NK_OK;
}

int nk_sh_step_log(nk_sh* s, double* steps, int32_t max) {
  if (!s || max < 0 || (max > 0 && !steps)) return NK_EINVAL;
  const std::vector<double>& log = s->NK->step_log();
  for (int32_t i = 0; i < max && size_t(i) < log.size(); ++i) steps[i] = log[i];
  return int(log.size());
}

int64_t nk_sh_workspace_bytes(nk_sh* s) { return s ? s->E->bytes_allocated() : -1; }

// ------------------------------------------------------------------------------ generic
int64_t nk_solve_workspace_bytes(int64_t n, const nk_opts* opts) {
  if (n <= 0) return NK_EINVAL;
  const nk_opts o = opts ? *opts : default_opts();
  return int64_t(sizeof(double)) * Engine::pad(n) * (NewtonKrylov::vectors_needed(o) + 2);
}

int nk_solve(nk_residual_fn F, void* ctx, const double* x0, double* x, int64_t n,
             const nk_opts* opts, nk_stats* stats, void* stream, void* workspace,
             int64_t workspace_bytes) {
  if (!F || !x0 || !x || n <= 0) return NK_EINVAL;
  const nk_opts o = opts ? *opts : default_opts();
  if (o.jvp_mode != NK_JVP_FD) return NK_EINVAL;  // a user residual has no analytic Jacobian
  Engine E(n, nullptr, S(stream), o.profile != 0);
  const int nvec = NewtonKrylov::vectors_needed(o);
  const int64_t npad = Engine::pad(n);
  const int64_t need = nk_solve_workspace_bytes(n, &o);
  double* ws = static_cast<double*>(workspace);
  const bool own = (ws == nullptr);
  if (!own && (workspace_bytes < need || (reinterpret_cast<uintptr_t>(ws) & 255u)))
    return NK_EINVAL;
  if (own && hipMalloc(reinterpret_cast<void**>(&ws), need) != hipSuccess) return NK_ENOMEM;
  CallbackProblem P(E, F, ctx, ws + npad * nvec, ws + npad * (nvec + 1));
  int rc;
  {
    NewtonKrylov NK(E, P, o, ws, int64_t(sizeof(double)) * npad * nvec);
    rc = NK.status();
    if (!rc) rc = NK.solve(x0, x, stats);
  }
  hipStreamSynchronize(S(stream));
  if (own) hipFree(ws);
  return rc;
}

// ------------------------------------------------------------------------------ droplet
int nk_drop_params_default(nk_drop_params* p) {
  if (!p) return NK_EINVAL;
  *p = nk_drop_params{};
  p->nx = 91;
  p->ny = 61;
  p->endl = -3;
  p->endr = 6;
  p->endb = -3;
  p->endt = 3;
  p->epsilon = 1e-2;
  p->n_exp = 6;
  p->m_exp = 3;
  p->Bo = 0.01;
  p->alpha2 = 0.0;
  p->alpha = 0.01;
  p->gamma = 0.1;
  p->C = 0.15;
  p->smoothing_iters = 4;
  p->a = 100.0;
  return NK_OK;
}

int nk_drop_create(nk_drop** out, const nk_drop_params* p, const nk_opts* opts, void* stream) {
  if (!out || !p || p->nx < 7 || p->ny < 7) return NK_EINVAL;
  if (p->n_exp < 0 || p->m_exp < 0) return NK_EINVAL;  // (integer powers by multiplication)
  DropParams P{};
  P.nx = p->nx;
  P.ny = p->ny;
  P.endl = p->endl;
  P.endr = p->endr;
  P.endb = p->endb;
  P.endt = p->endt;
  P.dksi = (p->endr - p->endl) / (p->nx - 1);  // droplet.py:36
  P.deta = (p->endt - p->endb) / (p->ny - 1);  // :37
  P.epsilon = p->epsilon;
  P.n_exp = p->n_exp;
  P.m_exp = p->m_exp;
  P.Bo = p->Bo;
  P.alpha2 = p->alpha2;
  P.epsilon2 = 1.0 / (p->endt - p->endb);  // :51
  P.alpha = p->alpha;
  P.gamma = p->gamma;
  P.C = p->C;
  P.smoothing_iters = p->smoothing_iters;
  P.a = p->a;
  const nk_opts o = opts ? *opts : default_opts();
  std::unique_ptr<DropletStepper> d(new (std::nothrow) DropletStepper(P, o, S(stream)));
  if (!d) return NK_ENOMEM;
  if (d->status()) return d->status();
  *out = reinterpret_cast<nk_drop*>(d.release());
  return NK_OK;
}

static DropletStepper* DS(nk_drop* d) { return reinterpret_cast<DropletStepper*>(d); }

int nk_drop_destroy(nk_drop* d) {
  delete DS(d);
  return NK_OK;
}
int nk_drop_set_state(nk_drop* d, const double* U, const double* Q) {
  return (d && U && Q) ? DS(d)->set_state(U, Q) : NK_EINVAL;
}
int nk_drop_get_state(nk_drop* d, double* U, double* Q) {
  return d ? DS(d)->get_state(U, Q) : NK_EINVAL;
}
int nk_drop_step(nk_drop* d, double dt, double dtmesh, int32_t pmaloops, nk_stats* stats,
                 double* dt_used, double* scale) {
  if (!d || pmaloops < 0) return NK_EINVAL;
  const int rc = DS(d)->step(dt, dtmesh, pmaloops, stats, dt_used);
  if (scale) *scale = DS(d)->scale;
  return rc;
}
int nk_drop_set_scale(nk_drop* d, double scale) {
  if (!d) return NK_EINVAL;
  DS(d)->scale = scale;
  return NK_OK;
}
int nk_drop_prepare(nk_drop* d) {
  if (!d) return NK_EINVAL;
  int rc = DS(d)->E.copy(DS(d)->P.uval, DS(d)->P.unew, DS(d)->E.n);
  if (!rc) rc = DS(d)->prepare();
  return rc ? rc : DS(d)->E.sync();
}
int nk_drop_field(nk_drop* d, int32_t which, double* out) {
  return (d && out) ? DS(d)->field(which, out) : NK_EINVAL;
}
int nk_drop_residual(nk_drop* d, const double* u, double dt, double* R) {
  return (d && u && R) ? DS(d)->residual(u, dt, R) : NK_EINVAL;
}
int nk_drop_solve(nk_drop* d, double dt, double* U, nk_stats* stats) {
  return (d && U) ? DS(d)->solve(dt, U, stats) : NK_EINVAL;
}
int nk_drop_pma(nk_drop* d, double dtmesh, int32_t loops) {
  if (!d || loops < 1) return NK_EINVAL;
  const int rc = DS(d)->pma(dtmesh, loops);
  return rc ? rc : DS(d)->E.sync();
}

int nk_drop_init_coalescing(nk_drop* d, int32_t vsteps, const double* info, int32_t ndrops,
                            double dtmesh, int32_t loops) {
  if (!d || vsteps < 1 || loops < 0 || ndrops < 0 || ndrops > kMaxDrops || (ndrops && !info))
    return NK_EINVAL;
  DropSet D{};
  D.n = ndrops;
  for (int k = 0; k < ndrops; ++k)
    for (int c = 0; c < 4; ++c) D.v[k][c] = info[4 * k + c];
  return DS(d)->init_coalescing(vsteps, D, dtmesh, loops);
}

// ------------------------------------------------------------------------------ sh_linearised
int nk_shlin_create(nk_shlin** out, int64_t ny, int64_t nx, double h, double r, double g, double k,
                    double rtol, int64_t maxiter, void* stream) {
  if (!out || ny < 5 || nx < 5 || !(h > 0) || !(k > 0) || !(rtol > 0) || maxiter < 1)
    return NK_EINVAL;
  std::unique_ptr<ShLinStepper> p(
      new (std::nothrow) ShLinStepper(ny, nx, h, r, g, k, rtol, maxiter, S(stream), false));
  if (!p) return NK_ENOMEM;
  if (p->status()) return p->status();
  *out = reinterpret_cast<nk_shlin*>(p.release());
  return NK_OK;
}
int nk_shlin_destroy(nk_shlin* s) {
  delete reinterpret_cast<ShLinStepper*>(s);
  return NK_OK;
}
int nk_shlin_step(nk_shlin* s, const double* U, const double* Uo, double* Unew, int64_t* iters,
                  double* relres) {
  if (!s || !U || !Uo || !Unew) return NK_EINVAL;
  ShLinStats st;
  const int rc = reinterpret_cast<ShLinStepper*>(s)->step(U, Uo, Unew, &st);
  if (iters) *iters = st.iters;
  if (relres) *relres = st.relres;
  return rc;
}

// ------------------------------------------------------------------------------ PMA2 (MEMS)
int nk_mems_params_default(nk_mems_params* p) {
  if (!p) return NK_EINVAL;
  *p = nk_mems_params{};
  p->n = 51;
  p->m = 3;
  p->smoothing_iters = 4;
  p->p = 2;
  p->alpha = 0.1;
  p->gamma = 0.1;
  p->epsilon = 0.0;
  p->beta = 0.15;
  p->lambd = 1.0;
  p->endl = -1.0;
  p->endr = 1.0;
  p->k = 1e-4;
  return NK_OK;
}

int nk_mems_create(nk_mems** out, const nk_mems_params* p, const nk_opts* opts, void* stream) {
  if (!out || !p || p->n < 7 || p->p != 2 || p->m < 0 || !(p->endr > p->endl)) return NK_EINVAL;
  DropParams P{};
  P.nx = P.ny = p->n;
  P.endl = P.endb = p->endl;
  P.endr = P.endt = p->endr;
  P.dksi = P.deta = (p->endr - p->endl) / (p->n - 1);  // PMA2_nk.py:33-34
  P.alpha = p->alpha;
  P.gamma = p->gamma;
  P.C = 1.0;  // mon += integral (:384)
  P.smoothing_iters = p->smoothing_iters;
  MemsParams Mp{};
  Mp.lambd = p->lambd;
  Mp.lam_eps = p->lambd * std::pow(p->epsilon, double(p->m - 2));  // lambd_*(epsilon_**(m_-2))
  Mp.beta2 = p->beta * p->beta;
  Mp.k = p->k;
  Mp.m = p->m;
  const nk_opts o = opts ? *opts : default_opts();
  std::unique_ptr<MemsStepper> m(new (std::nothrow) MemsStepper(P, Mp, p->epsilon, o, S(stream)));
  if (!m) return NK_ENOMEM;
  if (m->status()) return m->status();
  *out = reinterpret_cast<nk_mems*>(m.release());
  return NK_OK;
}

static MemsStepper* MS(nk_mems* m) { return reinterpret_cast<MemsStepper*>(m); }

int nk_mems_destroy(nk_mems* m) {
  delete MS(m);
  return NK_OK;
}
int nk_mems_set_state(nk_mems* m, const double* U, const double* Q) {
  if (!m || !U || !Q) return NK_EINVAL;
  MS(m)->time = 0.0;
  return MS(m)->set_state(U, Q);
}
int nk_mems_get_state(nk_mems* m, double* U, double* Q) {
  return m ? MS(m)->get_state(U, Q) : NK_EINVAL;
}
int nk_mems_step(nk_mems* m, nk_stats* stats, double* dt_used, double* time) {
  if (!m) return NK_EINVAL;
  const int rc = MS(m)->step(stats, dt_used);
  if (time) *time = MS(m)->time;
  return rc;
}
int nk_mems_prepare(nk_mems* m, double* dt) {
  if (!m) return NK_EINVAL;
  int rc = MS(m)->E.copy(MS(m)->P.uval, MS(m)->P.unew, MS(m)->E.n);
  if (!rc) rc = MS(m)->prepare(dt);
  return rc ? rc : MS(m)->E.sync();
}
int nk_mems_field(nk_mems* m, int32_t which, double* out) {
  return (m && out) ? MS(m)->field(which, out) : NK_EINVAL;
}
int nk_mems_residual(nk_mems* m, const double* u, double* R) {
  return (m && u && R) ? MS(m)->residual(u, R) : NK_EINVAL;
}

}  // extern "C"

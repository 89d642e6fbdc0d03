// Internal kernel interface of libnkhip (not part of the C-ABI).
//
// Layout in HBM: every grid vector is one row-major fp64 array u[i*nx + j] over the rank's row
// slab (i = y, j = x; sh_scipy_nk.py:34-35 fixes the flattening).  Stencil inputs carry two halo
// rows on each side: `lo` = global rows row0-2, row0-1 and `hi` = rows row0+ny, row0+ny+1, each a
// contiguous 2*nx block.  A single slab (one GPU) wraps periodically instead (lo == nullptr).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "peer_dev.h"  // PeerArgs: the peer-memory communicator's device-side arguments

struct nk_comm;  // comm.h

namespace nk {

// Row slabs over the peer-memory communicator run their collectives inside the kernels around
// them (arnoldi_edge_halo_launch, arn_reduce_allreduce_ctl_launch); NKHIP_PEER_FUSE=0 (read per
// call) keeps the separate communicator launches.
bool peer_fuse_enabled();
// The fused kernel runs the slab exchange itself (arnoldi.hip "Slab exchange"), with the peer
// communicator (and NKHIP_PEER_FUSE on): NKHIP_SLAB_XK=2 when no two ranks share a GPU, 1
// always (tests: several processes on one GPU); unset / 0: off (read per call).
bool slab_x_enabled(const nk_comm* c);
// wall_clock64() ticks of one bounded device-side wait: NKHIP_PEER_TIMEOUT_S seconds (default
// 20) at the device's wall-clock rate (hipDeviceAttributeWallClockRate)
uint64_t device_wait_ticks();
double device_wait_seconds();  // the seconds device_wait_ticks() stands for

// ---------------------------------------------------------------------------------------------
struct Field {
  const double* base;  // rows [0, ny)
  const double* lo;    // rows -2, -1   (nullptr: periodic wrap on base)
  const double* hi;    // rows ny, ny+1
};

inline Field periodic(const double* p) { return Field{p, nullptr, nullptr}; }

// 13-point coefficients of L = -Lap^2 - 2 Lap + (r-1) I with e = 1/h^2 (sh_scipy_nk.py:32,38-39).
struct SHCoef {
  double c0, c1, c2, c3;  // centre, axial +-1, diagonal, axial +-2
  double k, g;            // time step, quadratic coefficient (sh_scipy_nk.py:18,29)
  double ik;              // 1/k
};
SHCoef sh_coef(double h, double r, double k, double g);

enum class SMode : int {
  LAP5 = 0,   // out0 = Lap a                                     (sh_scipy_nk.py:32-35)
  SH13 = 1,   // out0 = L a                                       (sh_scipy_nk.py:38-39)
  RESID = 2,  // out0 = F(a; uo = b), the reference residual       (sh_scipy_nk.py:47-49)
  BOLD = 3,   // out0 = B(uo = a) = -uo/k - (L uo + g uo^2 - uo^3)/2, so F(u) = G(u) + B
  TRIAL = 4,  // w = a + alpha b: out2 = w, out1 = G(w), out0 = G(w) + p0; sums |F|^2, max|F|, max|w|
  FDJVP = 5,  // w = a + alpha b: out0 = (G(w) - p0) / sc          (_nonlin.py:1505-1513)
  AJVP = 6,   // out0 = alpha*(a/k - (L a + (2 g u - 3 u^2) a)/2) with u = p0 (analytic J v)
  LINOP = 7,  // w = a + alpha b: out2 = w, out0 = (1 + p0) w - theta L w; sums w . out0
              // (the semi-implicit operator I + D - L k/2 of sh_linearised.py:56, as CG's A p)
};

struct StencilArgs {
  int64_t ny = 0, nx = 0;
  Field a{}, b{};
  double alpha = 0.0;
  const double* p0 = nullptr;
  double* out0 = nullptr;
  double* out1 = nullptr;
  double* out2 = nullptr;
  double e = 0.0;   // LAP5
  SHCoef c{};
  double sc = 1.0;  // FDJVP step
  double* partial = nullptr;  // TRIAL: [3][nblk]
  // FDJVP/AJVP: if set, the step / scale come from the device value |z_raw|^2 (see jvp_scale)
  const double* znorm2 = nullptr;
  double omega = 0.0;
  // FDJVP, speculative (NewtonKrylov::line_search): the first JVP of the NEXT LGMRES call, issued
  // behind the s = 1 trial before the host has its reduction spec[0..2] = (sum F^2, max|F|,
  // max|x|).  The pass runs only if that trial passes the Armijo test (sum F^2 <= spec_thr) and
  // the iteration goes on (max|F| > spec_ftol); its step is the host's: omega = spec_rdiff
  // max(1, max|x|) / max(1, max|F|), sc = omega / spec_zn, alpha = sc spec_zs.
  const double* spec = nullptr;
  double spec_thr = 0.0, spec_ftol = 0.0, spec_rdiff = 0.0, spec_zn = 1.0, spec_zs = 1.0;
  double theta = 0.0;  // LINOP
  // edge array of out0 (nk::edge_elems layout, below): written in-kernel for the pool vectors the
  // fused Arnoldi kernel reads block halos from (TRIAL's F, the JVP's w), so no edge_gather pass
  // follows them; rows e_row0.. of an e_ny-row field (a row-range launch of a slab)
  double* E0 = nullptr;
  double* E2 = nullptr;  // ... of out2 (TRIAL's x + alpha p: the next Newton iterate)
  // edge arrays of the stencil fields a and b (same geometry): the block's side columns of an
  // own row come from them (four rows per line) instead of the neighbouring blocks' lines
  const double* Ea = nullptr;
  const double* Eb = nullptr;
  int64_t e_ny = 0, e_row0 = 0;
  // pushed halo rows (peer-memory slabs, arnoldi.hip): out0's / out2's rows 0, 1 and e_ny-2,
  // e_ny-1 also go into the previous / next rank's halo slot ([0] / [1], row stride ps_ld),
  // written through and drained (peer_dev.h store_sys16) -- what push_rows_launch would do after
  // the pass
  double* PS0[2] = {};
  double* PS2[2] = {};
  int64_t ps_ld = 0;
  bool rev = false;    // set by stencil_launch (traversal_reverse)
  bool nt_p0 = false;  // set by stencil_launch: non-temporal loads of the point-wise input
};

// MALL-friendly ping-pong: successive streaming kernels launched from one host thread alternate
// their traversal direction, so each starts on the address range its predecessor touched last
// (up to 256 MB of which may still sit in the memory-side Infinity Cache).  Flips on every call;
// NKHIP_PINGPONG=0 keeps every kernel forward.
bool traversal_reverse();

// Launches one stencil pass.  *nblk receives the number of partial-sum slots written (TRIAL).
hipError_t stencil_launch(SMode m, const StencilArgs& a, hipStream_t s, int64_t* nblk);
// Upper bound of the partial-sum slots one stencil pass with reductions (TRIAL) writes.
int64_t stencil_partial_slots(int64_t ny, int64_t nx);
// Algorithmic HBM bytes per grid point of one pass (for roofline accounting).
double stencil_bytes_per_point(SMode m, bool has_xt);

// ---------------------------------------------------------------------------------------------
constexpr int kMaxVec = 64;
struct VecList {
  const double* p[kMaxVec];
  double c[kMaxVec];
};

constexpr int kKrylovBlock = 256;
constexpr int kKrylovPerThread = 8;
constexpr int64_t kKrylovChunk = int64_t(kKrylovBlock) * kKrylovPerThread;

inline int64_t krylov_blocks(int64_t n) { return (n + kKrylovChunk - 1) / kKrylovChunk; }
// Grid of the Krylov kernels: returns the block count, *cpb = 2048-element chunks per block.
int64_t krylov_grid(int64_t n, int* cpb, int64_t target_blocks);

// partial[(i)*nblk + b]: a.p_i for i < np, g.p_i at np+i (g may be null -> zeros), a.a at 2np.
hipError_t mdot_launch(const double* a, const double* g, const VecList& P, int np, int64_t n,
                       double* partial, hipStream_t s, int64_t* nblk);
// out's edge array (the fused kernel's block halos, kEdgeW below), written by the pass that
// writes out: E (edge_elems(ny, nx) values), out's row length nx (even) and row count ny.
struct EdgeOut {
  double* E = nullptr;
  int64_t nx = 0, ny = 0;
};
// out = cin*in + sum_i c_i p_i (in may be null); partial: [0] sum out^2, [1] max|out|.
// out may alias `in` or any p_i (element-wise, each element read and written by one thread).
// eo.E: also write out's edge array (n == eo.nx eo.ny < 2^31), so no edge_gather pass follows.
hipError_t combo_launch(double* out, const double* in, double cin, const VecList& P, int np,
                        int64_t n, double* partial, hipStream_t s, int64_t* nblk,
                        const EdgeOut& eo = EdgeOut{});
// The same under device-side Arnoldi control: out = prm[kArnMaxNV] in + sum_i prm[i] p_i (the
// coefficients the control kernel wrote); nothing when the step was handed back (prm halt entry).
hipError_t combo_prm_launch(double* out, const double* in, const double* prm, const VecList& P,
                            int np, int64_t n, hipStream_t s);
// result[k] = sum_b partial[k*nblk + b] for k < nsum, NaN-propagating max for nsum <= k < nv.
// result_host (optional): pinned host memory the kernel also writes (zero-copy readback).
hipError_t reduce_final_launch(const double* partial, int64_t nblk, int nsum, int nv,
                               double* result, double* result_host, hipStream_t s);
// out = a*x + b*y (y may be null; out may alias x or y).  Element-wise helper of the generic
// residual path (nk_solve) and of nk_axpy / nk_scal.
// w = (w - f0) / sc, the finite difference of KrylovJacobian.matvec (_nonlin.py:1509).
hipError_t fddiff_launch(double* w, const double* f0, double sc, int64_t n, hipStream_t s);
// CG (sh_linearised): x += alpha p; r -= alpha q; partial[0..*nblk) = per-block sums of r'^2
// (*nblk <= 1024).
hipError_t cg_update_launch(double* x, double* r, const double* p, const double* q, double alpha,
                            int64_t n, double* partial, hipStream_t s, int64_t* nblk);
// d = (5U - Uo)^2 k/16 - g k U (sh_linearised.py:50)
hipError_t shlin_diag_launch(const double* U, const double* Uo, double k, double g, double* d,
                             int64_t n, hipStream_t s);
// dst = src, streamed in 16-KB chunks per block (the bench's per-box bandwidth probe); n even,
// 16-B aligned
hipError_t stream_copy_launch(const double* src, double* dst, int64_t n, hipStream_t s);
hipError_t axpby_launch(double a, const double* x, double b, const double* y, double* out,
                        int64_t n, hipStream_t s);

// ---------------------------------------------------------------------------------------------
// Fused Arnoldi step (arnoldi.hip): update v = tau*w + sum c_i V_i, FD JVP w' of z = v (or of an
// external z), and the multi-dot of w' and v against V and v, in one launch (periodic grid only).
constexpr int kArnMaxNV = 35;
// Edge arrays: the fused kernel's blocks own kEdgeW-column groups and read the two columns
// either side of each group of every update entry (its block halo).  Read straight from the
// vectors those are two extra lines per entry and row that the NEIGHBOUR block streams (a
// non-temporal load away from L2): ~9 % of the launch (profiles/r02_arnoldi_ab.md).  An edge
// array holds, per group boundary b (column B = kEdgeW b) and row q, the four values
// v[q][B-2], v[q][B-1], v[q][B], v[q][B+1] (columns mod nx): E[(b ny + q) 4 + 0..3], so four
// consecutive rows share a line.  The fused kernel, the stencil passes and the combinations
// (EdgeOut) write the edge arrays of their outputs; other producers run edge_gather_launch.
constexpr int kEdgeW = 256;
__host__ __device__ inline int64_t edge_groups(int64_t nx) { return (nx + kEdgeW - 1) / kEdgeW; }
__host__ __device__ inline int64_t edge_elems(int64_t ny, int64_t nx) { return edge_groups(nx) * ny * 4; }
hipError_t edge_gather_launch(const double* v, double* E, int64_t ny, int64_t nx, hipStream_t s);
// In-kernel slab exchange over the peer-memory communicator (arnoldi.hip "Slab exchange"): the
// fused kernel's edge bands publish u on the slab's edge rows straight into the neighbours'
// staging rows and wait for theirs; me == nullptr: off.
struct SlabX {
  char* me = nullptr;  // this rank's peer buffer, and the ring neighbours' (peer_dev.h layout)
  char* prev = nullptr;
  char* next = nullptr;
  int P = 0;
  int64_t max_nx = 0;
  uint64_t tag = 0;
  int* err = nullptr;  // pinned host error word of the communicator
  uint64_t wait_ticks = 0;  // bound of one wait (PeerArgs::wait_ticks)
};
struct ArnCtlState;
// Tail of a fused launch under device-side Arnoldi control (arnoldi.hip "Tail"): the launch's
// last blocks reduce its partials into `result` (and `result_host`), all-reduce them over the
// peer-memory communicator on a row slab (peer), and the very last block runs the control of
// step t on them -- the reduction + control launch that would otherwise follow, without its
// kernel boundary.  S == nullptr: none.  S->arrive / S->done count the blocks (reset by the last).
struct ArnTail {
  ArnCtlState* S = nullptr;
  ArnCtlState* H = nullptr;
  double* result = nullptr;       // nval values (the multi-dot slot of step t)
  double* result_host = nullptr;  // pinned copy (optional)
  double* prm = nullptr;          // the parameter block the control writes (the next launch's ctl)
  uint32_t* status = nullptr;
  int t = 0;
  int nval = 0;                   // 2 nv + 3
  bool peer = false;
  uint64_t wait_ticks = 0;        // bound of the reducers' wait (device_wait_ticks)
  PeerArgs pa{};
};
struct ArnoldiArgs {
  int64_t ny = 0, nx = 0;
  int nv = 0;                      // basis vectors V_0..V_{nv-1}
  int strips = 0, nbands = 0, RY = 0;  // set by arnoldi_launch
  const double* V[kArnMaxNV] = {};
  double c[kArnMaxNV] = {};        // zero beyond nv
  const double* w = nullptr;       // previous JVP output
  double tau = 1.0;
  const double* x0 = nullptr;      // Newton iterate
  const double* g0 = nullptr;      // G(x0): not read (the JVP is evaluated in closed form)
  const double* z = nullptr;       // JVP input if not the new v (LGMRES augmentation vector)
  double alpha = 0.0;              // w' = (G(x0 + alpha u) - G(x0))/sc with u = v or z
  double sc = 1.0;
  SHCoef k{};
  double* out_v = nullptr;         // must not alias w or any V_i
  double* out_w = nullptr;
  // edge arrays of V_0..V_{nv-1} (E[i]) and w (E[nv]); E[0] == nullptr: block halos read from
  // the vectors themselves
  const double* E[kArnMaxNV + 1] = {};
  double* Eout_v = nullptr;        // edge arrays of out_v / out_w, written when non-null
  double* Eout_w = nullptr;
  // row slab (one of several): u on the halo rows -2, -1, ny, ny+1 (4 rows of nx, filled by
  // arnoldi_edge_launch on every rank + the halo exchange); nullptr = single periodic slab
  const double* yh = nullptr;
  int64_t yh_ld = 0;               // row stride of yh (0: nx)
  SlabX x{};                       // in-kernel slab exchange (yh = this rank's staging rows)
  // Pushed halo rows (row slabs over the peer-memory communicator, hs_ld > 0; arnoldi.hip
  // "Pushed halo rows"): every producer of an update entry wrote that vector's edge rows into its
  // ring neighbours' halo slots (kHaloRows rows of hs_ld per pool vector: rows 0, 1 = the previous
  // rank's last two rows, 2, 3 = the next rank's first two), before an all-reduce this launch
  // follows; the edge bands compute u on the halo rows from the slots into yh (rows of nx)
  // themselves, so no exchange runs between the control and this launch.
  const double* HS[kArnMaxNV + 2] = {};  // this rank's slots of V_0..V_{nv-1}, w, (z)
  int64_t hs_ld = 0;
  // this launch's outputs into the neighbours' slots: [0] the previous rank's slot of out_v (its
  // rows 2, 3 <- my rows 0, 1), [1] the next rank's slot of out_v (its rows 0, 1 <- my rows
  // ny-2, ny-1), [2], [3] the same for out_w
  double* PS[4] = {};
  double* partial = nullptr;       // [(2 nv + 3)][pstride], this launch's columns from pcol0
  int64_t partial_cap = 0;         // doubles available at partial
  // rows [r_begin, r_end) of the slab are computed (r_end < 0: ny); rows outside are read only
  // (a band's two halo rows on either side).  Several launches over disjoint row ranges may share
  // one partial buffer: pstride = the total columns (0: this launch's own), pcol0 = its first.
  int64_t r_begin = 0, r_end = -1;
  int64_t pstride = 0, pcol0 = 0;
  bool plan_only = false;          // set *nwaves only, launch nothing
  int reserve_cus = 0;             // size the grid to leave this many CUs free (a concurrent
                                   // halo exchange needs CUs for its kernels)
  // device-side Arnoldi control (arn_ctl_launch): c, tau, alpha, sc come from the parameter block
  // ctl[kCtlPrm] the control kernel wrote instead of the fields above, and the launch does
  // nothing when its halt entry is set (the control handed the loop back to the host)
  const double* ctl = nullptr;
  // block-halo mailbox (plain launches over whole periodic rows only; see arnoldi.hip "Mailbox"):
  // the blocks of a band publish u on their two edge column pairs per row, tagged with mb_tag
  // (unique per launch), and read their neighbours' instead of recomputing the halo from every
  // update entry.  mb == nullptr, or a grid it does not fit: the packed halo loads.
  double* mb = nullptr;
  int64_t mb_cap = 0;  // doubles at mb
  uint64_t mb_tag = 0;
  bool mb_recompute = false;  // test switch: every halo pair takes the mailbox's recompute path
  // alternating march (arnoldi.hip "March direction"): the ALT instantiations, whose even bands
  // march up their rows and load their prologue temporally, so the rows two adjacent bands both
  // read are read at the same time and the second read hits the XCD's L2.  Set by arnoldi_launch
  // (-1: for bands of at most 32 rows; NKHIP_ARN_ALT=1 / 0 forces it on / off).
  int alt = -1;
  ArnTail tail{};             // reduction + control in the launch's last blocks (S: on)
};
// doubles of mailbox a grid of ny rows and nx columns may need (any layout, any band count)
inline int64_t arnoldi_mbox_elems(int64_t ny, int64_t nx) {
  return (2 * ny + 64) * (nx / 128 + 2) * 8;
}
// NKHIP_ARN_MBOX (read per call): 0 = packed halo loads, 1 = mailbox (default), 2 = mailbox with
// every halo pair recomputed by its consumer (the path a missing neighbour takes; tests)
int arnoldi_mbox_mode();
int64_t arnoldi_mbox_launches();  // fused launches that ran with the mailbox (process-wide)
bool arnoldi_supported(int nv, int64_t ny, int64_t nx);
// basis length nv runs the wide layout (128-column waves, 512-column blocks; NKHIP_ARN_WIDE=0: off)
bool arnoldi_wide(int nv);
// *nwaves = partial columns written: [w'.V_i (nv)] [w'.v] [v.V_i (nv)] [v.v] [w'.w']
hipError_t arnoldi_launch(const ArnoldiArgs& A, hipStream_t s, int64_t* nwaves);
// u = v (or z) on the slab's edge rows 0, 1, ny-2, ny-1 into y4 (4 rows of nx),
// with the fused kernel's summation order: what the neighbours need as their halo rows
hipError_t arnoldi_edge_launch(const ArnoldiArgs& A, double* y4, hipStream_t s);
// Bounds-checked build only (`make check`, -DNKHIP_ARN_CHECK): indices of the fused / edge kernels
// that fell outside their arrays since the last reset, and the smallest arnoldi.hip source line
// among them.  0 = ok, -1 = not the checked build, -2 = HIP error.
// The same for row slabs over the peer-memory communicator (pa = nk_comm::take_halo), with the
// halo exchange in the same launch: yh (4 rows of nx) receives the neighbours' rows -- lo = the
// previous rank's rows ny-2, ny-1, hi = the next rank's rows 0, 1 -- the fused pass's halo rows.
hipError_t arnoldi_edge_halo_launch(const ArnoldiArgs& A, const PeerArgs& pa, double* yh,
                                    hipStream_t s);
int arnoldi_check_counters(int64_t* violations, int32_t* first_line, bool reset);
// the mailbox statistics build (NKHIP_ARN_MBSTAT): halo pairs needed, not there at the first look,
// extra polls, recomputed; -1 in other builds
int arnoldi_mailbox_counters(int64_t out[4], bool reset);
// Pushed halo rows (peer.hip): v's rows 0, 1 -> rows 2, 3 of prev_slot and rows ny-2, ny-1 ->
// rows 0, 1 of next_slot (the ring neighbours' halo slots of v's pool vector, row stride ld,
// peer memory), written through and drained (no fence); nothing waits (the next all-reduce
// orders it).
hipError_t push_rows_launch(const double* v, double* prev_slot, double* next_slot, int64_t ny,
                            int64_t nx, int64_t ld, hipStream_t s);

// ---------------------------------------------------------------------------------------------
// Device-side Arnoldi control (arnctl.hip, lgmres.cpp).  The loop state of one LGMRES call: the
// host loop works on it in pinned memory, and hands it to the device (one copy) for runs of
// fused steps whose control -- Givens update of the previous Hessenberg column, residual test,
// Gram row, MGS coefficients, the lagged norm of the next vector -- a one-wave kernel computes
// between the fused launches, so no host round trip separates two Arnoldi steps.  Whatever the
// kernel does not handle (the stop, a cancelling norm estimate, a non-finite |w|) it hands back:
// it leaves the state as it was before that step and sets `halt`.
struct ArnCtlState {
  int32_t j;           // the step whose multi-dot results are consumed next
  int32_t hn_pending;  // step j - 1 still waits for |v_j| (the Gram diagonal of those results)
  int32_t m;           // steps of this call (inner_m + augmentation vectors)
  int32_t nv_max;      // the device issues fused steps up to this basis length
  int32_t halt;        // 0: the device continues; else 1 + the step it handed back
  int32_t steps;       // steps the device completed
  uint32_t arrive;     // blocks of the running reduction that finished (arn_reduce_ctl_launch,
                       // a fused launch's tail)
  uint32_t done;       // a fused launch's tail: reducer blocks that finished
  double ptol, omega, lag_ratio2, pad2_;
  double sig[kMaxVec + 2];      // scale of basis vector i (kept raw: v_i = sig_i V_i)
  double rn[kMaxVec + 2];       // |V_i| raw
  double sig_est[kMaxVec + 2];  // the lagged scale JVP_i saw (0: exact)
  double wnorm[kMaxVec + 2];    // |w_i|
  double zs[kMaxVec + 2];       // scale of the JVP input z_i (the final combination)
  double cs[kMaxVec + 1], sn[kMaxVec + 1];  // Givens rotations of the Hessenberg QR
  double gv[kMaxVec + 2];       // rotated right-hand side (residual estimate gv[j+1])
  double h[kMaxVec + 2];        // MGS coefficients of the latest step
  double R[kMaxVec + 1][kMaxVec + 1];
  double gram[kMaxVec + 1][kMaxVec + 1];  // sig_i sig_k (V_i . V_k), k < i
};
// parameter block of one fused step the control kernel writes: c[0..kArnMaxNV), tau, alpha, sc,
// halt (non-zero: the step was handed back, the queued launches do nothing)
constexpr int kCtlPrm = kArnMaxNV + 4;
// Control of step t (== S->j): consumes the all-reduced multi-dot results `red` of step t and,
// if the device continues, writes the parameters of the fused step with nv = t + 1 to prm and
// advances S.  Every committed value is also written to H, the host's pinned copy of the state,
// so the host needs no read-back when the device hands a step back.  status[t] (pinned host
// memory) <- 1 (continued) or 2 (handed back) after those writes.  Nothing runs once S->halt is
// set.
// red_host (optional, pinned): the kernel also copies `red` there (the host reads it when the
// step is handed back; saves the all-reduce path its D2H copy per step).
// upload_rows >= 0: the launch first copies H's fields before R and its Gram rows
// 0 .. upload_rows-1 into S itself (the entry of a run of device steps; no runtime copy).
hipError_t arn_ctl_launch(ArnCtlState* S, ArnCtlState* H, const double* red, double* red_host,
                          double* prm, uint32_t* status, int t, hipStream_t s,
                          int upload_rows = -1);
// The same preceded by the reduction of the fused step's partials (one GPU: no all-reduce in
// between) in one launch: result[k] = sum_b partial[k nblk + b] for k < nval (and result_host,
// pinned), then the last block to finish runs the control of step t on result.
hipError_t arn_reduce_ctl_launch(const double* partial, int64_t nblk, int nval, double* result,
                                 double* result_host, ArnCtlState* S, ArnCtlState* H, double* prm,
                                 uint32_t* status, int t, hipStream_t s);
// The same for row slabs over the peer-memory communicator (pa = nk_comm::take_allreduce): the
// reduction, the all-reduce of the nval sums and the control in one launch; result_host (pinned)
// receives the all-reduced values (the host reads them when the step is handed back).
hipError_t arn_reduce_allreduce_ctl_launch(const double* partial, int64_t nblk, int nval,
                                           double* result, double* result_host, const PeerArgs& pa,
                                           ArnCtlState* S, ArnCtlState* H, double* prm,
                                           uint32_t* status, int t, hipStream_t s);

}  // namespace nk

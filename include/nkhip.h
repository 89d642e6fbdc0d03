/*
 * nkhip.h -- C-ABI of the MI355X-native Newton-Krylov Swift-Hohenberg time-stepper.
 *
 * Every pointer argument named *_dev is a device (HBM) pointer to fp64 data; the caller owns
 * all buffers.  `stream` is a hipStream_t passed as void* (NULL = the null stream).  No torch
 * or Eigen types cross this boundary.  Grids are row-major, u[i*nx + j], i = y (row), j = x.
 *
 * Each entry point names the reference interface it replaces (file:line into the reference
 * Shiakaron/Iterative-solvers-summer-2020, or into the third-party SciPy 1.15.3 it calls,
 * prefixed scipy/).  The C++ twin's solver library is not vendored; its API was recovered from
 * the symbols of cpp_work/NewtonKrylov_Implementation/Project1/Debug/newton_krylov.obj
 *  and is cited as "NewtonKrylov lib".
 *
 * Return codes: NK_OK = 0; NK_NO_CONVERGENCE = 1 (scipy NoConvergence, _nonlin.py:247-249);
 * NK_NONFINITE = 2 (ValueError 'Function returned non-finite results', _nonlin.py:1511-1512);
 * NK_ZERO_STEP = 3 (ValueError 'Jacobian inversion yielded zero vector', _nonlin.py:213-216);
 * < 0: argument (NK_EINVAL), HIP (NK_EHIP) or RCCL (NK_ECOMM) failure.
 */
#ifndef NKHIP_H
#define NKHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NK_OK 0
#define NK_NO_CONVERGENCE 1
#define NK_NONFINITE 2
#define NK_ZERO_STEP 3
#define NK_BAD_RHS 4 /* lgmres ValueError 'RHS must contain only finite numbers' (lgmres.py:125) */
#define NK_EINVAL (-1)
#define NK_EHIP (-2)
#define NK_ECOMM (-3)
#define NK_ENOMEM (-4)

/* Layout version of the structs and signatures below.  nk_stats is written whole by the library
 * (sizeof(nk_stats) bytes): a caller built against another version must not pass its own
 * struct.  3: nk_stats gained n_backtrack, step_min, n_device_steps (round 2); nk_sh_step_log. */
#define NKHIP_ABI_VERSION 3

#define NK_JVP_FD 0       /* KrylovJacobian.matvec finite difference (scipy-faithful) */
#define NK_JVP_ANALYTIC 1 /* exact J v = v/k - (L v + (2 g u - 3 u^2) v)/2 */

/* Options of newton_krylov (scipy/optimize/_nonlin.py:1553-1603, nonlin_solve :122-268).
 * NaN tolerances select the SciPy defaults: f_tol = eps^(1/3), the others +inf. */
typedef struct nk_opts {
  double f_tol, f_rtol, x_tol, x_rtol;
  double rdiff;        /* <= 0: sqrt(eps) (_nonlin.py:1538-1539) */
  int64_t maxiter;     /* <= 0: 100*(n+1) (_nonlin.py:188) */
  int32_t inner_m;     /* lgmres inner_m, default 30 (lgmres.py:15) */
  int32_t outer_k;     /* default 10 (_nonlin.py:1453) */
  int32_t line_search; /* 1 = 'armijo' (default), 0 = None */
  int32_t jvp_mode;    /* NK_JVP_FD (default) or NK_JVP_ANALYTIC */
  int32_t verbose;     /* print "%d:  |F(x)| = %g; step %g" per Newton iteration */
  int32_t profile;     /* 0: off; k >= 1: time every k-th launch of each kernel class with HIP
                          events (see nk_sh_kernel_profile; each event pair costs ~5 us) */
} nk_opts;

typedef struct nk_stats {
  int64_t nit;         /* Newton iterations */
  int64_t nfev;        /* residual evaluations (initial + line search) */
  int64_t njvp;        /* Jacobian-vector products (one per Arnoldi step) */
  int64_t n_arnoldi;   /* Arnoldi steps (== njvp) */
  double fnorm_inf;    /* max|F(x)| at exit */
  double fnorm_2;      /* ||F(x)||_2 at exit */
  int32_t status;
  int32_t pad_;
  int64_t n_backtrack; /* Newton iterations whose Armijo step s was < 1 (scalar_search_armijo,
                          scipy/optimize/_linesearch.py:684-739) */
  double step_min;     /* smallest accepted line-search step (1 when none backtracked) */
  int64_t n_device_steps; /* Arnoldi steps whose control ran on the device (arnctl.hip) */
} nk_stats;

/* Per-kernel-class timings recorded with HIP events on the solver's stream. */
typedef struct nk_kprof {
  char name[32];
  int64_t launches;    /* all launches */
  double total_ms;     /* summed duration of the timed launches */
  double alg_bytes;    /* algorithmic HBM bytes summed over all launches */
  int64_t timed;       /* launches timed (every opts.profile-th) */
  double timed_bytes;  /* algorithmic HBM bytes of the timed launches */
} nk_kprof;

typedef struct nk_comm nk_comm;
typedef struct nk_sh nk_sh;

const char* nk_version(void);
/* NKHIP_ABI_VERSION of the library: a binding checks it against the header it was built from. */
int nk_abi_version(void);
int nk_opts_default(nk_opts* o);
const char* nk_status_string(int code);

/* ---------------- discrete operators (sh_scipy_nk.py:31-49; main.cpp:19-81) ---------------- */

/* y = Lap v, periodic 5-point Laplacian, e = 1/h^2.  Replaces the CSR SpMV `Lap @ v`
 * (sh_scipy_nk.py:32-35; Eigen SpMV over main.cpp:38-71). */
int nk_lap5_apply(const double* v_dev, double* y_dev, int64_t ny, int64_t nx, double e, void* stream);

/* y = L v, L = -Lap*Lap - 2*Lap + (r-1)*I as a 13-point periodic stencil.  Replaces `L @ u`
 * (sh_scipy_nk.py:38-39,49; main.cpp:23-24,78-81). */
int nk_sh13_apply(const double* v_dev, double* y_dev, int64_t ny, int64_t nx, double h, double r,
                  void* stream);

/* F = (u-uo)/k - (L u + g u^2 - u^3 + L uo + g uo^2 - uo^3)/2, the reference residual
 * (sh_scipy_nk.py:47-49; main.cpp:19-32), evaluated in one fused pass. */
int nk_sh_residual(const double* u_dev, const double* uo_dev, double* F_dev, int64_t ny, int64_t nx,
                   double h, double r, double k, double g, void* stream);

/* y = J(u) v = v/k - (L v + (2 g u - 3 u^2) v)/2 (analytic Jacobian of the residual above). */
int nk_sh_jvp(const double* u_dev, const double* v_dev, double* y_dev, int64_t ny, int64_t nx,
              double h, double r, double k, double g, void* stream);

/* y = (G(x0 + sc*zs*z) - G0) / sc, the finite-difference matvec of KrylovJacobian
 * (scipy/optimize/_nonlin.py:1500-1513) with the solver's split F(u) = G(u) + B(uo):
 * G(w) = w/k - (L w + g w^2 - w^3)/2 and G0 = G(x0) (pass y = F(x0+..) - F(x0) over sc when G0 is
 * F(x0) - B).  One fused pass reading x0, z, G0: the kernel inside every Arnoldi step. */
int nk_sh_fdjvp(const double* x0_dev, const double* G0_dev, const double* z_dev, double* y_dev,
                int64_t ny, int64_t nx, double h, double r, double k, double g, double zs,
                double sc, void* stream);

/* One fused Arnoldi step of the solver (the loop body of scipy's _fgmres between two matvecs,
 * scipy/sparse/linalg/_isolve/_gcrotmk.py:104-143, plus the next KrylovJacobian.matvec,
 * scipy/optimize/_nonlin.py:1500-1513), in one pass over the basis:
 *   v = tau*w + sum_i coef[i]*V[i]                 -> v_out
 *   w' = (G(x0 + sc*zs*z) - G(x0))/sc,  z = v if z_dev == NULL   -> w_out
 *   dots[0..2nv+2] = [w'.V_i (nv)] [w'.v] [v.V_i (nv)] [v.v] [w'.w']  (host; NULL: no reduction,
 *   no synchronisation).  nv <= 35, ny >= 8, nx >= 4 even, 16-B aligned vectors, periodic grid;
 *   v_out must not alias w or V[i].  The difference quotient is evaluated in closed form (G is a
 *   cubic plus the linear 13-point stencil), equal to the two-evaluation quotient in exact
 *   arithmetic but free of its cancellation, so G0_dev is not read (kept for the interface). */
int nk_sh_arnoldi_fused(const double* const* V_dev, const double* coef, int32_t nv,
                        const double* w_dev, double tau, const double* x0_dev, const double* G0_dev,
                        const double* z_dev, int64_t ny, int64_t nx, double h, double r, double k,
                        double g, double zs, double sc, double* v_out_dev, double* w_out_dev,
                        double* dots, void* stream);

/* Edge arrays (the fused step's block halos, 1/64 of a grid vector): for every column group
 * boundary B = 256 b and row q, E[(b*ny + q)*4 + 0..3] = v[q][B-2], v[q][B-1], v[q][B], v[q][B+1]
 * (columns mod nx); nk_edge_elems() doubles, nx even. */
int64_t nk_edge_elems(int64_t ny, int64_t nx);
int nk_edge_gather(const double* v_dev, double* E_dev, int64_t ny, int64_t nx, void* stream);
/* nk_sh_arnoldi_fused with the block halos read from the entries' edge arrays E_dev[0..nv]
 * (those of V[0..nv-1], then of w) instead of from the vectors (same values, identical results),
 * and the edge arrays of v_out / w_out written (Ev_out / Ew_out, each may be NULL). */
int nk_sh_arnoldi_fused_edges(const double* const* V_dev, const double* const* E_dev,
                              const double* coef, int32_t nv, const double* w_dev, double tau,
                              const double* x0_dev, const double* G0_dev, const double* z_dev,
                              int64_t ny, int64_t nx, double h, double r, double k, double g,
                              double zs, double sc, double* v_out_dev, double* w_out_dev,
                              double* Ev_out_dev, double* Ew_out_dev, double* dots, void* stream);
/* Block-halo mailbox of the fused step (no reference counterpart: a property of this kernel's
 * grid).  The blocks of a band publish u on their edge columns and read their neighbours' instead
 * of recomputing the halo from every update entry; NKHIP_ARN_MBOX=0 turns it off, =2 makes every
 * consumer recompute (the path a missing neighbour takes).  Counts the fused launches, process-
 * wide, that ran with it (nx a multiple of the kernel's block width, >= 2 blocks per band). */
int64_t nk_arnoldi_mbox_launches(void);

/* ---------------- BLAS-1 (scipy get_blas_funcs dot/nrm2/axpy/scal in _gcrotmk.py:104-126) ------ */
/* Scalar results are written to host memory; the call synchronises `stream`. */
int nk_dot(const double* x_dev, const double* y_dev, int64_t n, double* out, void* stream);
int nk_nrm2(const double* x_dev, int64_t n, double* out, void* stream);
int nk_maxnorm(const double* x_dev, int64_t n, double* out, void* stream); /* _nonlin.py:36-37 */
int nk_axpy(double a, const double* x_dev, double* y_dev, int64_t n, void* stream);
int nk_scal(double a, double* x_dev, int64_t n, void* stream);
/* out[i] = V[i] . w for i < m, in one pass over w (V: host array of m device pointers). */
int nk_mdot(const double* const* V_dev, int32_t m, const double* w_dev, int64_t n, double* out,
            void* stream);
/* y += sum_i coef[i] * V[i] in one pass (coef: host array). */
int nk_maxpy(const double* const* V_dev, const double* coef, int32_t m, double* y_dev, int64_t n,
             void* stream);

/* dst = src (n doubles, n even, 16-B aligned), streamed in 16-KB chunks per block with
 * non-temporal loads and stores.  No reference counterpart: the bench's probe of the box's
 * achievable HBM streaming rate (roofline.peak_measured), the ~6.3 TB/s of a float4 copy. */
int nk_stream_copy(const double* src_dev, double* dst_dev, int64_t n, void* stream);

/* Debugging aid, bounds-checked build only (`make -C iterative-solvers-summer-2020_amd check` ->
 * nkhip/libnkhip_check.so): every index the fused Arnoldi / slab-edge kernels compute is checked
 * against its array; an out-of-range index is counted (and replaced by 0, so nothing faults).
 * *violations = the count since the last reset, *first_line = the smallest arnoldi.hip source
 * line among them (0: none); reset != 0 clears the counters.  Synchronises the device.
 * NK_EINVAL from the product library (no checks compiled in). */
int nk_debug_bounds(int64_t* violations, int32_t* first_line, int32_t reset);
/* The fused kernel's block-halo mailbox, counted by the statistics build
 * (`make mbstat`, nkhip/libnkhip_mbstat.so) since the last reset: counts[0] halo pairs the
 * consumer lanes needed, [1] records not there at the first look, [2] extra polls, [3] pairs
 * recomputed after kMBSpin polls.  NK_EINVAL from the other builds.  Diagnostic only: no
 * reference interface. */
int nk_debug_mailbox(int64_t* counts, int32_t reset);

/* ---------------- communicators (row-slab decomposition over RCCL / xGMI) ---------------- */
int nk_comm_unique_id_bytes(void);
int nk_comm_get_unique_id(void* out);
/* One process per GPU: RCCL communicator from a unique id shared by rank 0. */
int nk_comm_create_rccl(nk_comm** out, const void* unique_id, int32_t rank, int32_t nranks);
/* One process, `nranks` slabs driven by `nranks` host threads on one device (testing the slab
 * logic on a single GPU): fills out[0..nranks-1]. */
int nk_comm_create_loopback(nk_comm** out, int32_t nranks);
/* Peer-memory communicator (one process per GPU over xGMI, or several processes on one GPU):
 * the slab collectives are small kernels that write straight into the peers' exported buffers
 * and wait for tagged flags (csrc/peer.hip) instead of RCCL calls.  Two phases: create
 * (allocates this rank's buffer for slabs of up to max_nx columns and writes its handle blob,
 * nk_comm_peer_handle_bytes() bytes, to handle_out), exchange the blobs through any side
 * channel, then connect with all nranks blobs in rank order.  One PROCESS per rank: connect
 * returns NK_EINVAL when two ranks of a group of more than one are the same process (threads
 * of one process share its in-order hardware queues, so a collective waiting for a peer rank
 * could sit ahead of the launch it waits for). */
int nk_comm_peer_handle_bytes(void);
int nk_comm_create_peer(nk_comm** out, int32_t rank, int32_t nranks, int64_t max_nx,
                        void* handle_out);
int nk_comm_peer_connect(nk_comm* c, const void* handles);
int nk_comm_destroy(nk_comm* c);
/* Marks the group failed.  Loopback (one process): every rank blocked in, or later entering, a
 * collective of the group returns NK_ECOMM instead of waiting for the failed rank (the waiting
 * threads are woken).  Peer-memory communicator: the abort word is written into every rank's
 * buffer, so every rank's collective kernels stop waiting and its next synchronisation returns
 * NK_ECOMM (a wait also gives up by itself after NKHIP_PEER_TIMEOUT_S seconds of wall-clock
 * time, default 20).  RCCL (one process per GPU): this
 * rank's communicator is aborted at once (ncclCommAbort) and its later calls return NK_ECOMM;
 * peer processes are NOT notified -- a peer blocked in a collective with the failed rank is
 * released by the launcher's own failure handling (e.g. the torch.distributed watchdog).  A stepper calls it itself when one of its steps fails with a negative code; a host
 * thread that fails outside the library calls it before it exits. */
int nk_comm_abort(nk_comm* c);
/* One all-reduce (sums and maxima) and one halo exchange of known values through the group,
 * checked on the host; every rank calls it (a collective).  NK_OK, or NK_ECOMM when a value did
 * not arrive intact (bench.py falls back from the peer-memory communicator to RCCL on that). */
int nk_comm_selftest(nk_comm* c, int64_t nx, void* stream);
/* The pushed-halo-rows protocol the slab solver uses by default on the peer-memory
 * communicator, exactly as the solver runs it: every rank pushes 4 rows of
 * known codes into its ring neighbours' halo slots (push kernel, system-scope fence, no flag),
 * passes ONE all-reduce, then reads its own slots back in a kernel and checks them on the host;
 * every rank calls it (a collective).  NK_OK; NK_ECOMM when a row did not arrive intact (bench.py
 * then runs the edge + halo exchange path, NKHIP_SLAB_PUSH=0, on every rank); NK_EINVAL on every
 * rank when some rank's communicator has no halo slots (RCCL, loopback) or a stepper holds them.
 * Replaces no reference interface: the check before the multi-GPU path is trusted. */
int nk_comm_selftest_push(nk_comm* c, int64_t nx, void* stream);

/* ---------------- Swift-Hohenberg implicit time step (the north-star path) ---------------- */
/* A stepper for one row slab [row0, row0+ny_local) of an ny_global x nx periodic grid.
 * comm == NULL means a single slab (ny_local == ny_global).  Replaces the loop body
 * sh_scipy_nk.py:56-61 (`U = newton_krylov(residual, Uo)`) and main.cpp:97-104
 * (`U = nonlin_solve(residual, Uo, 6e-6, inf, inf, inf)`). */
int nk_sh_create(nk_sh** out, int64_t ny_local, int64_t nx, int64_t ny_global, double h, double r,
                 double k, double g, const nk_opts* opts, nk_comm* comm, void* stream);
int nk_sh_destroy(nk_sh* s);
/* u_next = the Crank-Nicolson step from u_prev (both local slabs, may alias). */
int nk_sh_step(nk_sh* s, const double* u_prev_dev, double* u_next_dev, nk_stats* stats);
int nk_sh_set_opts(nk_sh* s, const nk_opts* opts);
/* Copies up to `max` per-kernel-class records; returns the number of classes. */
int nk_sh_kernel_profile(nk_sh* s, nk_kprof* out, int32_t max);
int nk_sh_reset_profile(nk_sh* s);
/* The accepted line-search step s of every Newton iteration of the last nk_sh_step
 * (scalar_search_armijo's result inside _nonlin_line_search, scipy/optimize/_nonlin.py:294-314;
 * the `step %g` of the reference's verbose line, sh_scipy_nk.py:61): copies up to `max` of them
 * to `steps` (host) and returns how many there were. */
int nk_sh_step_log(nk_sh* s, double* steps, int32_t max);
int64_t nk_sh_workspace_bytes(nk_sh* s);

/* ---------------- generic drop-in: newton_krylov(F, xin) over a device residual ---------------- */
/* F(ctx, x_dev, f_dev, n) evaluates the residual on device buffers and returns 0 on success.
 * Replaces scipy.optimize.newton_krylov (scipy/optimize/_nonlin.py:1603) for any residual, e.g.
 * the droplet / PMA2 closures (droplet.py:383, PMA2_nk.py:100). */
/* `workspace` (device, 256-B aligned, nk_solve_workspace_bytes() long) may be NULL, in which case
 * the solver allocates it; every pointer handed to F points into the workspace or x0/x. */
typedef int (*nk_residual_fn)(void* ctx, const double* x_dev, double* f_dev, int64_t n);
int64_t nk_solve_workspace_bytes(int64_t n, const nk_opts* opts);
int nk_solve(nk_residual_fn F, void* ctx, const double* x0_dev, double* x_dev, int64_t n,
             const nk_opts* opts, nk_stats* stats, void* stream, void* workspace,
             int64_t workspace_bytes);

/* ---------------- thin-film droplet on a moving mesh (python_work/droplet.py, config 3) -------- */
/* Parameters = the module globals of droplet.py:22-53 (defaults from nk_drop_params_default). */
typedef struct nk_drop_params {
  int32_t nx, ny;                 /* 91, 61 (:29) */
  double endl, endr, endb, endt;  /* -3, 6, -3, 3 (:32-33) */
  double epsilon;                 /* precursor film 1e-2 (:24) */
  int32_t n_exp, m_exp;           /* 6, 3 (:48-49) */
  double Bo, alpha2;              /* 0.01, 0 (:47, :50) */
  double alpha, gamma, C;         /* PMA: 0.01, 0.1, 0.15 (:40-42) */
  int32_t smoothing_iters;        /* 4 (:31) */
  int32_t pad_;
  double a;                       /* droplet profile sharpness 100 (:24) */
} nk_drop_params;
typedef struct nk_drop nk_drop;

int nk_drop_params_default(nk_drop_params* p);
int nk_drop_create(nk_drop** out, const nk_drop_params* p, const nk_opts* opts, void* stream);
int nk_drop_destroy(nk_drop* d);
/* state: U.new (= U.val) and the mesh potential Q.val, device arrays of nx*ny */
int nk_drop_set_state(nk_drop* d, const double* U_dev, const double* Q_dev);
int nk_drop_get_state(nk_drop* d, double* U_dev, double* Q_dev);
/* one iteration of evolve_with_PDE (droplet.py:369-411): dt_n = dt*scale; U.val = U.new; the
 * mesh / old-time fields; U.new = newton_krylov(residual(u, F, dt_n), U.val) with the nk_opts
 * given at creation (the reference: maxiter=20, f_tol=1e-7, :383); loop_pma(dtmesh, pmaloops);
 * scale += exp(-10 |U.new - U.val|).  *dt_used = dt_n, *scale = the updated scale. */
int nk_drop_step(nk_drop* d, double dt, double dtmesh, int32_t pmaloops, nk_stats* stats,
                 double* dt_used, double* scale);
int nk_drop_set_scale(nk_drop* d, double scale);
/* pieces of the step (tests / tooling): */
int nk_drop_prepare(nk_drop* d);  /* droplet.py:371-381 for the current state (U.val = U.new) */
/* which: 0 d2ksi 1 d2eta 2 dksideta 3 J 4 A11 5 A22 6 A12 7 Q_dksi 8 Q_deta 9 F 10 U.xx 11 U.yy
 *        12 U.val 13 U.new 14 Q.val */
int nk_drop_field(nk_drop* d, int32_t which, double* out_dev);
int nk_drop_residual(nk_drop* d, const double* u_dev, double dt, double* R_dev); /* :435-450 */
int nk_drop_solve(nk_drop* d, double dt, double* U_dev, nk_stats* stats);         /* :383 */
int nk_drop_pma(nk_drop* d, double dtmesh, int32_t loops);                       /* :589-599 */
/* initialise_coalescing_droplets (droplet.py:132-189) from the current state (normally U = epsilon,
 * Q = (xi^2 + eta^2)/2, main() :103-106): `info` (host) holds ndrops <= 8 (x, y, R, V) rows; the
 * volumes grow linearly over vsteps steps, each followed by loop_pma(dtmesh, loops).  The
 * reference runs (1000, [[0,0,1,1],[3,0,1,1]], 5e-9, 20) and saves the result as
 * initdrop_coal_*.txt. */
int nk_drop_init_coalescing(nk_drop* d, int32_t vsteps, const double* info, int32_t ndrops,
                            double dtmesh, int32_t loops);

/* ---------------- semi-implicit SH step (python_work/sh_linearised.py) ----- */
/* U[s+1] = solve(I + D - L k/2, (I + L k/2) U[s]), D = diag((5U[s] - U[s-1])^2 k/16 - g k U[s])
 * (:48-56) on a periodic ny x nx grid of spacing h.  The reference factorises the sparse matrix
 * (scipy spsolve); here a matrix-free conjugate-gradient solve on the 13-point stencil (the
 * matrix is SPD whenever 1 + min D > k r/2, always for g = 0), warm-started from U[s], to
 * |b - A x| <= rtol |b|.  Returns NK_NO_CONVERGENCE after maxiter iterations and NK_NONFINITE
 * if p.Ap <= 0 (indefinite system) or the data are not finite. */
typedef struct nk_shlin nk_shlin;
int nk_shlin_create(nk_shlin** out, int64_t ny, int64_t nx, double h, double r, double g, double k,
                    double rtol, int64_t maxiter, void* stream);
int nk_shlin_destroy(nk_shlin* s);
int nk_shlin_step(nk_shlin* s, const double* U_dev, const double* Uo_dev, double* Unew_dev,
                  int64_t* iters, double* relres);

/* ---------------- MEMS on a moving mesh (python_work/PMA2_nk.py) ------------ */
/* u_t = -(-Lap)^2 u - lambda/(1+u)^2 + lambda eps^(m-2)/(1+u)^m on [endl, endr]^2 (N x N), one
 * PMA mesh step per time step.  Parameters = the module globals of PMA2_nk.py:22-37.  Only p = 2
 * exists: the reference's p = 1 branch of residual() raises (u.xx, :135). */
typedef struct nk_mems_params {
  int32_t n;                    /* 51 (:22) */
  int32_t m;                    /* 3 (:25) */
  int32_t smoothing_iters;      /* 4 (:30) */
  int32_t p;                    /* 2 (:24); anything else is NK_EINVAL */
  double alpha, gamma;          /* PMA: 0.1, 0.1 (:26-27) */
  double epsilon, beta, lambd;  /* 0, 0.15, 1 (:28-29, :31) */
  double endl, endr;            /* -1, 1 (:32) */
  double k;                     /* 1e-4 (:36): the dt residual() divides by (quirk, :51/:91) */
} nk_mems_params;
typedef struct nk_mems nk_mems;

int nk_mems_params_default(nk_mems_params* p);
int nk_mems_create(nk_mems** out, const nk_mems_params* p, const nk_opts* opts, void* stream);
int nk_mems_destroy(nk_mems* m);
/* state: U.new (= U.val) and Q.val, device arrays of n*n */
int nk_mems_set_state(nk_mems* m, const double* U_dev, const double* Q_dev);
int nk_mems_get_state(nk_mems* m, double* U_dev, double* Q_dev);
/* one pass of main()'s loop (PMA2_nk.py:77-103): U.val = U.new; mesh fields; dt = compute_g()*k;
 * solve_PMA; CN_term; U.new = newton_krylov(residual, U.val) with the nk_opts given at creation
 * (the reference: SciPy defaults, :97); Q.val += dt*Q.dt.  *dt_used = dt, *time = the clock. */
int nk_mems_step(nk_mems* m, nk_stats* stats, double* dt_used, double* time);
/* pieces (tests / tooling): prepare = :80-94 for the current state, *dt = compute_g()*k */
int nk_mems_prepare(nk_mems* m, double* dt);
/* which: as nk_drop_field, with 9 = CN_term */
int nk_mems_field(nk_mems* m, int32_t which, double* out_dev);
int nk_mems_residual(nk_mems* m, const double* u_dev, double* R_dev); /* :121-159 */

#ifdef __cplusplus
}
#endif
#endif /* NKHIP_H */

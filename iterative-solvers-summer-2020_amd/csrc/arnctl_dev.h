// Device-side Arnoldi control (arnctl.hip): the per-step host arithmetic of lgmres.cpp's fused
// path (scipy/sparse/linalg/_isolve/_gcrotmk.py:114-165 as restated there) as a device function
// run by one wave -- of the control kernels in arnctl.hip, or of the last block of a fused
// Arnoldi launch (arnoldi.hip "Tail").
//
// Lane i holds entry i of the step's vectors (j + 1 <= kArnMaxNV + 1 <= 64 entries).  The serial
// parts -- the Givens sweep over the previous Hessenberg column, the forward substitution of the
// inverse compact-WY MGS, |h|^2 -- run in the host loop's order (uniform loops over readlane'd
// values), so the device differs from the host only by fused multiply-adds.
#pragma once
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdint>

#include "nk_kernels.h"

namespace nk {

static_assert(kArnMaxNV + 1 <= 64, "one lane per basis entry");

__device__ __forceinline__ double ctl_bcast(double v, int l) {  // lane l's v, l wave-uniform
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_readlane(uint32_t(b), l);
  const uint32_t hi = __builtin_amdgcn_readlane(uint32_t(b >> 32), l);
  return __builtin_bit_cast(double, (uint64_t(hi) << 32) | lo);
}

// The control of step t, run by the first wave of a block (the other waves of the block must not
// take part).  S: device state, H: the host's pinned copy (committed values go to both).  G: LDS
// scratch of (kArnMaxNV + 1)^2 doubles (the Gram rows of the column sweep).
__device__ inline void ctl_body(ArnCtlState* S, ArnCtlState* H, const double* red,
                                double* red_host, double* prm, uint32_t* status, int t,
                                double (*G)[kArnMaxNV + 1]) {
  const int lane = threadIdx.x & 63;
  // the same field of H as p of S
  auto mirror = [&](auto* p) {
    return reinterpret_cast<decltype(p)>(reinterpret_cast<char*>(H) +
                                         (reinterpret_cast<char*>(p) - reinterpret_cast<char*>(S)));
  };
  auto put = [&](auto* p, auto v) {
    *p = v;
    *mirror(p) = v;
  };
  // every load up front (one latency, not a chain): the step is t, and anything that says
  // otherwise hands it back
  const int j = t;
  const int np = j + 1;
  const int32_t halted = S->halt, sj = S->j, pending = S->hn_pending, nvm = S->nv_max, m = S->m;
  const bool on = lane <= j;
  const double rv = on ? red[lane] : 0.0;       // w_j . V_i
  const double rg = on ? red[np + lane] : 0.0;  // V_j . V_i (lane j: |V_j|^2)
  const double ww_raw = red[2 * np];            // |w_j|^2
  double sig = (lane <= j) ? S->sig[lane] : 0.0;
  const double hprev = (lane < j) ? S->h[lane] : 0.0;  // MGS coefficients of step j - 1
  const double csl = (lane < j) ? S->cs[lane] : 0.0;
  const double snl = (lane < j) ? S->sn[lane] : 0.0;
  const double wn_i = S->wnorm[j > 0 ? j - 1 : 0], gvi = S->gv[j > 0 ? j - 1 : 0];
  const double se = S->sig_est[j], ptol = S->ptol, omega = S->omega, lr2 = S->lag_ratio2;
  const int32_t steps = S->steps;
  if (halted) return;  // an earlier step was handed back: the host takes over from there
  if (red_host) {  // the results of step t for the host (read if this step is handed back)
    for (int i = lane; i <= 2 * np; i += 64) red_host[i] = red[i];
  }
  // hand step j back to the host unchanged (the host loop redoes it from the same state)
  auto hand_back = [&] {
    if (lane == 0) {
      put(&S->halt, int32_t(1 + j));
      prm[kArnMaxNV + 3] = 1.0;  // the fused step queued behind this control does nothing
    }
    __threadfence_system();
    if (lane == 0) __hip_atomic_store(status + t, 2u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  };
  if (sj != t || !pending || j < 1 || j + 1 > nvm || j + 1 >= m) {
    hand_back();
    return;
  }

  // -- finish step i = j - 1 with hn = |V_j| (lgmres.cpp `finish`)
  const int i = j - 1;
  const double hn = std::sqrt(ctl_bcast(rg, j));
  const double alpha = 1.0 / hn;
  const double sig_j = std::isfinite(alpha) ? alpha : 1.0;
  const bool breakdown = !(hn > DBL_EPSILON * wn_i);
  // Givens sweep over hcur[0..i+1] = (h_0 .. h_i, hn): hcur[k] settles at sweep k
  double a = ctl_bcast(hprev, 0);
  double rcol = 0.0;  // lane k: R[k][i]
  for (int k = 0; k < i; ++k) {
    const double b = ctl_bcast(hprev, k + 1);
    const double c = ctl_bcast(csl, k), s = ctl_bcast(snl, k);
    const double tk = c * a + s * b;
    a = -s * a + c * b;
    if (lane == k) rcol = tk;
  }
  // givens(hcur[i], hn) (nk_solver.cpp detail::givens)
  double ci = 1.0, si = 0.0;
  if (hn != 0.0) {
    const double r = std::hypot(a, hn);
    ci = a / r;
    si = hn / r;
  }
  const double rii = ci * a + si * hn;
  if (lane == i) rcol = rii;
  const double gv_next = -si * gvi, gv_i = ci * gvi;
  if (std::fabs(gv_next) < ptol || breakdown) {
    hand_back();
    return;
  }
  double tau = 1.0;
  if (se > 0.0) tau = sig_j / se;  // JVP_j saw V_j scaled by the estimate, not sig_j
  if (lane == j) sig = sig_j;

  // -- step j: |w|, Gram row, MGS coefficients (I + L) h = V^T w
  const double ww = tau * tau * ww_raw;
  if (!std::isfinite(ww)) {
    hand_back();
    return;
  }
  const double gj = (lane < j) ? sig_j * sig * rg : 0.0;  // gram[j][lane]
  // Gram rows 0..j (k < row) in LDS for the column sweep (one wave: LDS keeps its order).  Every
  // load is issued before the first LDS store (one row per unrolled iteration, no index
  // division): one memory latency for the whole matrix instead of one per row.
  {  // lane k takes column k of rows k+1 .. j-1
    double gl[kArnMaxNV];
#pragma unroll
    for (int r = 1; r < kArnMaxNV; ++r) gl[r] = (r < j && lane < r) ? S->gram[r][lane] : 0.0;
#pragma unroll
    for (int r = 1; r < kArnMaxNV; ++r)
      if (r < j && lane < r) G[r][lane] = gl[r];
  }
  if (lane < j) G[j][lane] = gj;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  double acc = on ? tau * sig * rv : 0.0;
  double hh = 0.0;
  for (int k = 0; k <= j; ++k) {
    const double hk = ctl_bcast(acc, k);  // final: every k' < k has been subtracted
    hh += hk * hk;
    if (lane > k && on) acc -= G[lane][k] * hk;
  }
  const double est = ww - hh;  // |v_{j+1}|^2 = |w|^2 - |h|^2
  if (!(est > lr2 * ww)) {
    hand_back();
    return;
  }
  const double e = std::sqrt(est);
  const double zs = 1.0 / e;
  const double zn = zs * e;
  if (zn == 0.0) {
    hand_back();
    return;
  }
  const double sc = omega / zn;

  // -- commit step i's Hessenberg column and step j, then the fused step's parameters
  if (lane <= i) put(&S->R[lane][i], rcol);
  if (lane < j) put(&S->gram[j][lane], gj);
  if (on) put(&S->h[lane], acc);
  if (lane < kArnMaxNV) prm[lane] = on ? -acc * sig : 0.0;
  if (lane == 0) {
    put(&S->cs[i], ci);
    put(&S->sn[i], si);
    put(&S->gv[i], gv_i);
    put(&S->gv[i + 1], gv_next);
    put(&S->sig[j], sig_j);
    put(&S->rn[j], hn);
    if (se > 0.0) put(&S->zs[j], sig_j);
    put(&S->wnorm[j], std::sqrt(ww));
    put(&S->sig_est[j + 1], zs);
    put(&S->zs[j + 1], zs);
    put(&S->j, int32_t(j + 1));
    put(&S->hn_pending, int32_t(1));
    put(&S->steps, steps + 1);
    prm[kArnMaxNV] = tau;
    prm[kArnMaxNV + 1] = sc * zs;
    prm[kArnMaxNV + 2] = sc;
    prm[kArnMaxNV + 3] = 0.0;
  }
  // no fence: the host reads nothing on a continued step (it reads the mirror after a hand-back,
  // whose release fence follows these writes in stream order)
  if (lane == 0) __hip_atomic_store(status + t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}


// The control launches' form of ctl_body (arnctl.hip): the same arithmetic in the same order
// (bitwise the same results), split in two.  ctl_load issues every load of the step's state --
// the scalars, the lane arrays and, for lane l < j, Gram row l -- and is run by the first wave of
// every reducing block, so the loads are in registers when the last block gets the values;
// ctl_run is the control itself, with the MGS forward substitution on the Gram row in registers
// (ctl_body stages the rows through LDS and reads G[lane][k] inside the serial loop).  Round 6:
// the launch's control part went from two load latencies and an LDS-latency chain (5.3 us,
// scripts/dbg/ctl_probe.py) to 3.2 us; staging the rows through LDS once instead (coalesced
// column loads, one batch of row reads) measured 4.3 us.  (The fused launch's tail keeps
// ctl_body: its code is part of every fused kernel.)
struct CtlPre {
  int32_t halted, sj, pending, nvm, m, steps;
  double sig, hprev, csl, snl;             // lane values (0 beyond their ranges)
  double wn_i, gvi, se, ptol, omega, lr2;  // uniform
  double grow[kArnMaxNV];                  // lane l < j: gram[l][k] for k < l (else 0)
};
__device__ __forceinline__ void ctl_load(const ArnCtlState* S, int t, CtlPre& P) {
  const int lane = threadIdx.x & 63;
  const int j = t;
  P.halted = S->halt;
  P.sj = S->j;
  P.pending = S->hn_pending;
  P.nvm = S->nv_max;
  P.m = S->m;
  P.steps = S->steps;
  P.sig = (lane <= j) ? S->sig[lane] : 0.0;
  P.hprev = (lane < j) ? S->h[lane] : 0.0;
  P.csl = (lane < j) ? S->cs[lane] : 0.0;
  P.snl = (lane < j) ? S->sn[lane] : 0.0;
  P.wn_i = S->wnorm[j > 0 ? j - 1 : 0];
  P.gvi = S->gv[j > 0 ? j - 1 : 0];
  P.se = S->sig_est[j];
  P.ptol = S->ptol;
  P.omega = S->omega;
  P.lr2 = S->lag_ratio2;
  const bool row = lane < j && lane < kArnMaxNV;
#pragma unroll
  for (int k = 0; k < kArnMaxNV; ++k) P.grow[k] = (row && k < lane) ? S->gram[lane][k] : 0.0;
}

__device__ inline void ctl_run(ArnCtlState* S, ArnCtlState* H, const double* red,
                               double* red_host, double* prm, uint32_t* status, int t,
                               const CtlPre& P) {
  const int lane = threadIdx.x & 63;
  auto mirror = [&](auto* p) {
    return reinterpret_cast<decltype(p)>(reinterpret_cast<char*>(H) +
                                         (reinterpret_cast<char*>(p) - reinterpret_cast<char*>(S)));
  };
  auto put = [&](auto* p, auto v) {
    *p = v;
    *mirror(p) = v;
  };
  const int j = t;
  const int np = j + 1;
  const bool on = lane <= j;
  const double rv = on ? red[lane] : 0.0;       // w_j . V_i
  const double rg = on ? red[np + lane] : 0.0;  // V_j . V_i (lane j: |V_j|^2)
  const double ww_raw = red[2 * np];            // |w_j|^2
  double sig = P.sig;
  const double hprev = P.hprev, csl = P.csl, snl = P.snl;
  const double wn_i = P.wn_i, gvi = P.gvi, se = P.se, ptol = P.ptol, omega = P.omega,
               lr2 = P.lr2;
  const int32_t steps = P.steps;
  if (P.halted) return;
  if (red_host) {
    for (int i = lane; i <= 2 * np; i += 64) red_host[i] = red[i];
  }
  auto hand_back = [&] {
    if (lane == 0) {
      put(&S->halt, int32_t(1 + j));
      prm[kArnMaxNV + 3] = 1.0;
    }
    __threadfence_system();
    if (lane == 0) __hip_atomic_store(status + t, 2u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  };
  if (P.sj != t || !P.pending || j < 1 || j + 1 > P.nvm || j + 1 >= P.m) {
    hand_back();
    return;
  }

  // -- finish step i = j - 1 with hn = |V_j| (as ctl_body)
  const int i = j - 1;
  const double hn = std::sqrt(ctl_bcast(rg, j));
  const double alpha = 1.0 / hn;
  const double sig_j = std::isfinite(alpha) ? alpha : 1.0;
  const bool breakdown = !(hn > DBL_EPSILON * wn_i);
  double a = ctl_bcast(hprev, 0);
  double rcol = 0.0;
  for (int k = 0; k < i; ++k) {
    const double b = ctl_bcast(hprev, k + 1);
    const double c = ctl_bcast(csl, k), s = ctl_bcast(snl, k);
    const double tk = c * a + s * b;
    a = -s * a + c * b;
    if (lane == k) rcol = tk;
  }
  double ci = 1.0, si = 0.0;
  if (hn != 0.0) {
    const double r = std::hypot(a, hn);
    ci = a / r;
    si = hn / r;
  }
  const double rii = ci * a + si * hn;
  if (lane == i) rcol = rii;
  const double gv_next = -si * gvi, gv_i = ci * gvi;
  if (std::fabs(gv_next) < ptol || breakdown) {
    hand_back();
    return;
  }
  double tau = 1.0;
  if (se > 0.0) tau = sig_j / se;
  if (lane == j) sig = sig_j;

  // -- step j: |w|, Gram row, MGS coefficients (I + L) h = V^T w
  const double ww = tau * tau * ww_raw;
  if (!std::isfinite(ww)) {
    hand_back();
    return;
  }
  const double gj = (lane < j) ? sig_j * sig * rg : 0.0;  // gram[j][lane]
  double acc = on ? tau * sig * rv : 0.0;
  double hh = 0.0;
#pragma unroll
  for (int k = 0; k < kArnMaxNV; ++k) {  // k <= j <= kArnMaxNV - 1 (j + 1 <= nv_max)
    if (k <= j) {  // (a guard, not a break: the loop stays unrolled, P.grow in registers)
      const double hk = ctl_bcast(acc, k);
      hh += hk * hk;
      const double g = (lane == j) ? ctl_bcast(gj, k) : P.grow[k];
      if (lane > k && on) acc -= g * hk;
    }
  }
  const double est = ww - hh;
  if (!(est > lr2 * ww)) {
    hand_back();
    return;
  }
  const double e = std::sqrt(est);
  const double zs = 1.0 / e;
  const double zn = zs * e;
  if (zn == 0.0) {
    hand_back();
    return;
  }
  const double sc = omega / zn;

  // -- commit (as ctl_body)
  if (lane <= i) put(&S->R[lane][i], rcol);
  if (lane < j) put(&S->gram[j][lane], gj);
  if (on) put(&S->h[lane], acc);
  if (lane < kArnMaxNV) prm[lane] = on ? -acc * sig : 0.0;
  if (lane == 0) {
    put(&S->cs[i], ci);
    put(&S->sn[i], si);
    put(&S->gv[i], gv_i);
    put(&S->gv[i + 1], gv_next);
    put(&S->sig[j], sig_j);
    put(&S->rn[j], hn);
    if (se > 0.0) put(&S->zs[j], sig_j);
    put(&S->wnorm[j], std::sqrt(ww));
    put(&S->sig_est[j + 1], zs);
    put(&S->zs[j + 1], zs);
    put(&S->j, int32_t(j + 1));
    put(&S->hn_pending, int32_t(1));
    put(&S->steps, steps + 1);
    prm[kArnMaxNV] = tau;
    prm[kArnMaxNV + 1] = sc * zs;
    prm[kArnMaxNV + 2] = sc;
    prm[kArnMaxNV + 3] = 0.0;
  }
  if (lane == 0) __hip_atomic_store(status + t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace nk

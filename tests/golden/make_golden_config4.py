"""Reference-pinned fixtures for config 4 and for the time loop (survey container only).

Two cases, both driven through the reference's own prologue (``sh_scipy_nk.py:1-49`` executed by
``make_golden.reference_namespace``) and SciPy 1.15.3's ``newton_krylov`` exactly as the loop body
does (``sh_scipy_nk.py:53-61``):

``nk_n4096_h0625_sampled.npz``  (config 4: 4096^2, d = 0.625 N = 2560, SURVEY 7 hard part 2)
    ONE implicit step from ``U0 = default_rng(2020).standard_normal(4096^2)`` at SciPy's default
    tolerances.  A 4096^2 state is 134 MB, so only a sample is stored: 64 strided rows of U1
    (rows 0, 64, 128, ...; 2 MB), the sum of every row of U1 (4096 values), max|U1| and the
    reference's Newton-iteration and F-eval counts.  The GPU test regenerates U0 from the seed.

``nk_n64_traj100.npz``  (the reference defaults: N = 64, d = 40, sh_scipy_nk.py:15-16)
    100 consecutive steps of the loop from ``U0 = default_rng(2020).standard_normal(64^2)``
    (the reference draws ``np.random.randn``; a seeded generator makes it reproducible), every
    10th state stored, the Newton-iteration / F-eval counts of all 100 steps.

Only arrays are written; no reference source text.  Run (about 3-4 minutes, ~12 GB of RAM for
the 4096^2 CSR matrices):  MPLBACKEND=Agg python tests/golden/make_golden_config4.py
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import OUT, nk_step, reference_namespace  # noqa: E402

SAMPLE_STRIDE = 64


def config4_case():
    N, d = 4096, 2560.0
    t0 = time.time()
    ns = reference_namespace(N, d)
    print(f"4096^2 prologue (CSR Lap, L): {time.time() - t0:.1f} s", flush=True)
    U0 = np.random.default_rng(2020).standard_normal(N * N)
    t0 = time.time()
    U1, nit, nfev, fin = nk_step(ns, U0)
    print(f"4096^2 step: {time.time() - t0:.1f} s, nit {nit}, nfev {nfev}, |F|inf {fin:.3e}",
          flush=True)
    G = U1.reshape(N, N)
    rows = np.arange(0, N, SAMPLE_STRIDE)
    return dict(N=N, d=d, h=ns["h"], r=0.01, k=0.2, g=1.0, seed=2020, f_tol=np.nan,
                rows=rows, U1_rows=G[rows].copy(), U1_rowsum=G.sum(axis=1),
                U1_absmax=float(np.abs(U1).max()), nit=np.array([nit]),
                nfev=np.array([nfev]), fnorm=np.array([fin]))


def traj_case(nsteps=100, every=10):
    N, d = 64, 40.0
    ns = reference_namespace(N, d)
    U = np.random.default_rng(2020).standard_normal(N * N)
    saved, at, nits, nfevs, fins = [U.copy()], [0], [], [], []
    for s in range(1, nsteps + 1):
        U, nit, nfev, fin = nk_step(ns, U)
        nits.append(nit)
        nfevs.append(nfev)
        fins.append(fin)
        if s % every == 0:
            saved.append(U.copy())
            at.append(s)
    print(f"64^2 trajectory: {nsteps} steps, nit {sum(nits)}, nfev {sum(nfevs)}", flush=True)
    return dict(N=N, d=d, h=ns["h"], r=0.01, k=0.2, g=1.0, seed=2020, f_tol=np.nan,
                steps=np.array(at), traj=np.array(saved), nit=np.array(nits),
                nfev=np.array(nfevs), fnorm=np.array(fins))


def main():
    cases = {"nk_n64_traj100": traj_case()}
    if "--traj-only" not in sys.argv:
        cases["nk_n4096_h0625_sampled"] = config4_case()
    for name, arrs in cases.items():
        np.savez_compressed(os.path.join(OUT, name + ".npz"),
                            **{k: np.asarray(v) for k, v in arrs.items()})
        print("wrote", name, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""Generate the golden parity fixtures from the reference itself (survey container only).

The reference ``python_work/sh_scipy_nk.py`` is a top-to-bottom script whose module level runs a
2500-step plotting loop (:51-69).  Following SURVEY.md section 8c, this script executes ONLY its
prologue (lines 1-49: imports, parameters, the assembled CSR ``Lap`` and ``L``, and ``residual``)
in a private namespace, with ``N`` / ``d`` substituted per case, then drives
``scipy.optimize.newton_krylov(residual, Uo)`` exactly as the loop body does (:56-61).

Only the resulting arrays (inputs and outputs) are written to ``tests/golden/*.npz``; no reference
source text is stored.  ``/root/reference`` does not exist on the GPU box, so the tests there read
only these fixtures.  Run:  MPLBACKEND=Agg python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import re
import sys

import numpy as np

REF = "/root/reference/python_work/sh_scipy_nk.py"
OUT = os.path.dirname(os.path.abspath(__file__))


def reference_namespace(N: int, d: float):
    """exec sh_scipy_nk.py:1-49 with N and d substituted."""
    os.environ.setdefault("MPLBACKEND", "Agg")
    with open(REF) as fh:
        src = "\n".join(fh.read().splitlines()[:49])
    src, n1 = re.subn(r"^N = 64", f"N = {N}", src, flags=re.M)
    src, n2 = re.subn(r"^d = 40", f"d = {d!r}", src, flags=re.M)
    assert n1 == 1 and n2 == 1, "reference prologue changed"
    ns: dict = {}
    exec(compile(src, REF, "exec"), ns)
    import matplotlib.pyplot as plt
    plt.close("all")
    return ns


def set_old(ns, uo):
    ns["Uo"] = uo.copy()
    ns["UoUo"] = np.multiply(uo, uo)
    ns["UoUoUo"] = np.multiply(uo, ns["UoUo"])


def nk_step(ns, uo, steps=None, **kw):
    """One step of the reference loop (sh_scipy_nk.py:56-61), counting F evals and Newton its.
    `steps` (a list) receives the Armijo step size s of every Newton iteration: scipy's own
    scalar_search_armijo (scipy/optimize/_linesearch.py:684-739) is wrapped, not replaced."""
    import scipy.optimize._nonlin as nonlin
    from scipy.optimize import newton_krylov
    set_old(ns, uo)
    nfev = [0]
    nit = [0]
    res = ns["residual"]

    def F(u):
        nfev[0] += 1
        return res(u)

    def cb(x, f):
        nit[0] += 1

    orig = nonlin.scalar_search_armijo

    def armijo(*a, **k):
        out = orig(*a, **k)
        if steps is not None:
            steps.append(np.nan if out[0] is None else float(out[0]))
        return out

    nonlin.scalar_search_armijo = armijo
    try:
        u = newton_krylov(F, uo, callback=cb, **kw)
    finally:
        nonlin.scalar_search_armijo = orig
    set_old(ns, uo)
    fin = float(np.abs(res(u)).max())
    return u, nit[0], nfev[0], fin


def ops_case(N, d, seed=2020):
    ns = reference_namespace(N, d)
    rng = np.random.default_rng(seed)
    v = rng.standard_normal(N * N)
    return dict(N=N, d=d, h=ns["h"], r=float(ns["r"]), k=ns["k"], g=float(ns["g"]), v=v,
                lap_v=ns["Lap"] @ v, L_v=ns["L"] @ v, L_nnz=ns["L"].nnz)


def backtrack_case():
    """(4) A Newton step whose Armijo line search backtracks (s < 1, including the cubic branch
    of scalar_search_armijo): the reference geometry (N = 61, d = 40) from a large-amplitude
    start U0 = 3 * default_rng(2020).standard_normal(N^2), default f_tol.  Records scipy's step
    sizes per Newton iteration and its F-eval count."""
    N, d = 61, 40.0
    ns = reference_namespace(N, d)
    U0 = 3.0 * np.random.default_rng(2020).standard_normal(N * N)
    steps = []
    U, nit, nfev, fin = nk_step(ns, U0, steps=steps)
    print("nk_n61_amp3_backtrack nit", nit, "nfev", nfev, "steps", np.round(steps, 4))
    return dict(N=N, d=d, h=ns["h"], r=0.01, k=0.2, g=1.0, f_tol=np.nan,
                traj=np.array([U0, U]), nit=np.array([nit]), nfev=np.array([nfev]),
                fnorm=np.array([fin]), steps=np.array(steps))


def main():
    if "--only-backtrack" in sys.argv:
        z = backtrack_case()
        np.savez_compressed(os.path.join(OUT, "nk_n61_amp3_backtrack.npz"),
                            **{k: np.asarray(v) for k, v in z.items()})
        return 0
    cases = {"nk_n61_amp3_backtrack": backtrack_case()}
    # (1) operator fixtures: L@v and Lap@v at N = 5 (C++ twin geometry d=2, main.cpp:3-5),
    #     61 and 64 (reference domain d=40), plus an h = 0.625 grid at N = 128.
    for name, (N, d) in {"ops_n5_d2": (5, 2.0), "ops_n61": (61, 40.0), "ops_n64": (64, 40.0),
                         "ops_n128_h0625": (128, 80.0)}.items():
        cases[name] = ops_case(N, d)

    # (2) residual(u) at N=61 with the reference globals (sh_scipy_nk.py:47-49)
    ns = reference_namespace(61, 40.0)
    rng = np.random.default_rng(2020)
    uo = rng.standard_normal(61 * 61)
    u = uo + 0.1 * rng.standard_normal(61 * 61)
    set_old(ns, uo)
    cases["residual_n61"] = dict(N=61, d=40.0, h=ns["h"], r=0.01, k=0.2, g=1.0, uo=uo, u=u,
                                 F=ns["residual"](u))

    # (3) Newton-Krylov steps (sh_scipy_nk.py:56-61), U0 = default_rng(2020).standard_normal(N^2)
    for name, (N, d, ftol, nsteps) in {
        "nk_n61_default": (61, 40.0, None, 2),
        "nk_n61_tight": (61, 40.0, 1e-10, 1),
        "nk_n64_default": (64, 40.0, None, 1),
        "nk_n64_h0625_tight": (64, 40.0, 1e-10, 1),
        "nk_n96_h0625_tight": (96, 60.0, 1e-10, 1),
        "nk_n5_d2_tight": (5, 2.0, 1e-10, 3),
    }.items():
        ns = reference_namespace(N, d)
        U = np.random.default_rng(2020).standard_normal(N * N)
        traj, nits, nfevs, fins = [U.copy()], [], [], []
        kw = {} if ftol is None else {"f_tol": ftol}
        for _ in range(nsteps):
            U, nit, nfev, fin = nk_step(ns, U, **kw)
            traj.append(U.copy())
            nits.append(nit)
            nfevs.append(nfev)
            fins.append(fin)
        cases[name] = dict(N=N, d=d, h=ns["h"], r=0.01, k=0.2, g=1.0,
                           f_tol=np.nan if ftol is None else ftol, traj=np.array(traj),
                           nit=np.array(nits), nfev=np.array(nfevs), fnorm=np.array(fins))
        print(name, "nit", nits, "nfev", nfevs, "|F|inf", fins)

    for name, arrs in cases.items():
        np.savez_compressed(os.path.join(OUT, name + ".npz"),
                            **{k: np.asarray(v) for k, v in arrs.items()})
    print("wrote", len(cases), "fixtures to", OUT)


if __name__ == "__main__":
    sys.exit(main())

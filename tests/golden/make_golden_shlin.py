"""Generate sh_linearised (python_work/sh_linearised.py) golden fixtures from the reference itself
(survey container only).

``main()`` is one function: it draws ``U = np.random.randn(N**2)`` (unseeded), builds Lap and L,
and runs ``ceil(Tf/k)`` semi-implicit steps, each a sparse direct solve

    U[s+1] = spsolve(I + D - L k/2, (I + L k/2) U[s]),  D = diag((5U[s] - U[s-1])^2 k/16 - g k U[s])

(:48-56), plotting as it goes.  This script seeds NumPy's global generator (2020), caps the step
count by handing the module a ``math`` whose ``ceil`` returns STEPS, runs ``main()`` headless
(Agg), and records every ``spsolve`` right-hand side and solution through a wrapper around the
module's ``linalg``.

Writes tests/golden/shlin_steps.npz: U0 and U[s] for s = 1..STEPS (N = 64, d = 40, k = 0.2,
r = 0.2, g = 0 -- main()'s values).
Run:  MPLBACKEND=Agg python tests/golden/make_golden_shlin.py
"""
import os
import sys
from types import SimpleNamespace

import numpy as np

REF_DIR = "/root/reference/python_work"
OUT = os.path.dirname(os.path.abspath(__file__))
STEPS = 6


def main():
    os.environ.setdefault("MPLBACKEND", "Agg")
    import matplotlib
    matplotlib.use("Agg")
    sys.path.insert(0, REF_DIR)
    import sh_linearised as sl

    rec = {"rhs": [], "U": []}
    real = sl.linalg

    def spsolve(A, b):
        x = real.spsolve(A, b)
        rec["rhs"].append(np.asarray(b).copy())
        rec["U"].append(x.copy())
        return x

    sl.linalg = SimpleNamespace(spsolve=spsolve)
    sl.math = SimpleNamespace(ceil=lambda v: STEPS)
    np.random.seed(2020)
    U0 = np.random.randn(64 * 64)
    np.random.seed(2020)
    sl.main()
    assert len(rec["U"]) == STEPS
    np.savez_compressed(os.path.join(OUT, "shlin_steps.npz"), U0=U0, U=np.array(rec["U"]),
                        rhs=np.array(rec["rhs"]), N=64, d=40.0, k=0.2, r=0.2, g=0.0)
    print("saved", STEPS, "steps; max |U|", float(np.abs(rec["U"][-1]).max()))


if __name__ == "__main__":
    main()

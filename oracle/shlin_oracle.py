"""TEST INFRASTRUCTURE ONLY -- restatement of the semi-implicit Swift-Hohenberg stepper
(python_work/sh_linearised.py).

    D = diag((5 U[s] - U[s-1])^2 k/16 - g k U[s])                       (:50)
    U[s+1] = spsolve(I + D - L k/2, (I + L k/2) U[s])                      (:56)

with L = -Lap*Lap - 2 Lap + (r - 1) I the same 13-point periodic operator as sh_scipy_nk.py
(:31-39; sh_oracle.csr_L).  main() starts from U[-1] = U[0] (:25-26).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
from scipy.sparse import linalg

from .sh_oracle import csr_L


def step(L, U, Uo, k, g):
    """One pass of main()'s loop body (:48-56); returns U[s+1]."""
    nn = U.size
    I = sp.identity(nn, format="csc")
    D = sp.diags(np.multiply(5 * U - Uo, 5 * U - Uo) * k / 16 - g * k * U, 0, shape=(nn, nn),
                 format="csc")
    return linalg.spsolve((I + D - L * k / 2), np.transpose((I + L * k / 2) @ U))


def run(U0, nsteps, N=64, d=40.0, k=0.2, r=0.2, g=0.0):
    """main() (:14-65) without plotting; returns the list of U[1..nsteps]."""
    L = csr_L(N, d / N, r).tocsc()
    U, Uo, out = U0.copy(), U0.copy(), []
    for _ in range(nsteps):
        U, Uo = step(L, U, Uo, k, g), U
        out.append(U)
    return out

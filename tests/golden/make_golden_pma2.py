"""Generate PMA2 (MEMS moving-mesh, python_work/PMA2_nk.py) golden fixtures from the reference
itself (survey container only).

``PMA2_nk.py`` builds a 3-D plot at import time with ``fig.gca(projection='3d')`` (:56), which
matplotlib >= 3.5 no longer accepts; the shim routes ``gca(**kw)`` with keywords to
``add_subplot(**kw)``.  ``main()`` plots every step, so this script drives the
loop body of ``main`` (:77-106) itself, with plotting off, exactly as ``main`` orders it:

    U.val = U.new; compute_Q_spatial_ders; J = ...; compute_u_spatial_ders
    dt = compute_g()*k                  (local: residual() keeps using the global dt = k)
    solve_PMA(); CN_term = compute_rhs_pde()
    U.new = newton_krylov(residual, U.val, verbose=0)
    Q.val += dt*Q.dt

Writes tests/golden/pma2_*.npz (inputs and outputs only, no reference source):
  pma2_steps    Q0, U0 and, per step s < STEPS: U_new[s], Q_val[s], dt[s], nit[s], nfev[s]
  pma2_fields   the derived fields at the start of step FIELD_STEP (nonzero U): Q derivatives, J,
                U_dx/U_dy/U_xx/U_yy, the smoothed monitor, Q.dt, CN_term, plus residual(u1) at a
                perturbed u1 with that step's U.val / CN_term
Run:  MPLBACKEND=Agg python tests/golden/make_golden_pma2.py
"""
import os
import sys

import numpy as np

REF_DIR = "/root/reference/python_work"
OUT = os.path.dirname(os.path.abspath(__file__))
STEPS = 4
FIELD_STEP = 2


def load_reference():
    os.environ.setdefault("MPLBACKEND", "Agg")
    import matplotlib
    matplotlib.use("Agg")
    from matplotlib.figure import FigureBase
    gca = FigureBase.gca

    def gca_shim(self, **kw):
        return self.add_subplot(**kw) if kw else gca(self)

    FigureBase.gca = gca_shim
    sys.path.insert(0, REF_DIR)
    import PMA2_nk as pm
    pm.plot_bool = False
    return pm


def main():
    pm = load_reference()
    from scipy.optimize import newton_krylov
    # main() initialisation (:65-71)
    pm.Q.val = np.reshape(0.5 * pm.ksiksi ** 2 + 0.5 * pm.etaeta ** 2, pm.NN_)
    pm.make_Ibdy()
    pm.make_M()
    pm.U.new = np.zeros(pm.NN_, dtype=float)
    Q0, U0 = pm.Q.val.copy(), pm.U.new.copy()

    calls = [0]
    resid = pm.residual

    def counted(u):
        calls[0] += 1
        return resid(u)

    out = {"U_new": [], "Q_val": [], "dt": [], "nit": [], "nfev": []}
    fields = None
    for s in range(STEPS):
        pm.U.val = pm.U.new.copy()
        pm.compute_Q_spatial_ders()
        pm.J = pm.Q.d2ksi * pm.Q.d2eta - pm.Q.dksideta ** 2
        pm.compute_u_spatial_ders()
        dt = pm.compute_g() * pm.k
        pm.solve_PMA()
        pm.CN_term = pm.compute_rhs_pde()
        if s == FIELD_STEP:
            rng = np.random.default_rng(2020)
            u1 = pm.U.val + 1e-3 * rng.standard_normal(pm.NN_)
            fields = dict(
                U_val=pm.U.val.copy(), Q_val=pm.Q.val.copy(), Q_dksi=pm.Q.dksi, Q_deta=pm.Q.deta,
                Q_d2ksi=pm.Q.d2ksi, Q_d2eta=pm.Q.d2eta, Q_dksideta=pm.Q.dksideta, J=pm.J,
                U_dx=pm.U.dx, U_dy=pm.U.dy, U_xx=pm.U.xx, U_yy=pm.U.yy,
                mon=pm.compute_and_smooth_monitor(), Q_dt=pm.Q.dt, CN=pm.CN_term, dt=dt, u1=u1,
                R1=pm.residual(u1))
        calls[0] = 0
        its = [0]
        pm.U.new = newton_krylov(counted, pm.U.val, verbose=0,
                                 callback=lambda x, f: its.__setitem__(0, its[0] + 1))
        pm.Q.val += dt * pm.Q.dt
        out["U_new"].append(pm.U.new.copy())
        out["Q_val"].append(pm.Q.val.copy())
        out["dt"].append(dt)
        out["nit"].append(its[0])
        out["nfev"].append(calls[0])
        print(f"step {s}: dt {dt:.6e} nit {its[0]} nfev {calls[0]} u_min {pm.U.new.min():.6e}")
    np.savez_compressed(os.path.join(OUT, "pma2_steps.npz"), Q0=Q0, U0=U0,
                        **{k: np.array(v) for k, v in out.items()})
    np.savez_compressed(os.path.join(OUT, "pma2_fields.npz"), **fields)


if __name__ == "__main__":
    main()

"""Generate droplet (config 3) golden fixtures from the reference itself (survey container only).

``python_work/droplet.py`` is importable once two matplotlib incompatibilities are shimmed
(SURVEY.md 8c): ``Axes3D.w_zaxis`` (removed in matplotlib 3.8, used at :87) is aliased to
``zaxis``; plotting is then disabled with ``plot3d_bool = False``.  ``read_from_file`` cannot be
used (Windows path separator, :568), so the coal init state is read with ``np.loadtxt``.

Writes tests/golden/droplet_*.npz (inputs and outputs only, no reference source):
  droplet_init        U0, Q0 from initdrop_coal_1_91-61_100_0.01_0.01_0.1_0.15.txt
  droplet_fields      the per-step derived fields of evolve_with_PDE step 1 (:371-381) and a
                      residual(u, F, dt) evaluation (:435-450)
  droplet_nk          newton_krylov(lambda u: residual(u, F, dt), U.val, maxiter=20, f_tol=1e-7)
                      at the fixed step-1 mesh (:383), with Newton-iteration / F-eval counts
  droplet_pma         Q.val after loop_pma(3e-9, 5) and after loop_pma(3e-9, 400) (:589-599)
  droplet_evolve      U.new, Q.val, scale after evolve_with_PDE(1e-4, 3, 1e-2, 3e-9, 400) (2 steps)
  droplet_evolve10    config 3 over its SURVEY 8(d) length: evolve_with_PDE(1e-4, 11, 1e-2, 3e-9,
                      400) (S = 10 steps), U.new / Q.val / dt_n / Newton its after EVERY step,
                      recorded by wrapping the module's loop_pma (called once per step, :384)
Run:  MPLBACKEND=Agg python tests/golden/make_golden_droplet.py [evolve10]
"""
import contextlib
import io
import os
import sys

import numpy as np

REF_DIR = "/root/reference/python_work"
OUT = os.path.dirname(os.path.abspath(__file__))
INIT = "initdrop_coal_1_91-61_100_0.01_0.01_0.1_0.15.txt"


def load_reference():
    os.environ.setdefault("MPLBACKEND", "Agg")
    import matplotlib
    matplotlib.use("Agg")
    from mpl_toolkits.mplot3d import axes3d
    axes3d.Axes3D.w_zaxis = property(lambda s: s.zaxis)
    sys.path.insert(0, REF_DIR)
    import droplet as dr
    dr.plot3d_bool = False
    dr.make_Ibdy()
    dr.make_M()
    return dr


def reset(dr, U0, Q0):
    dr.U.new = U0.copy()
    dr.U.val = U0.copy()
    dr.Q.val = Q0.copy()


def step_fields(dr):
    """The derivative block of evolve_with_PDE (:371-381)."""
    dr.U.val = dr.U.new.copy()
    dr.compute_Q_spatial_ders()
    dr.J = dr.Q.d2ksi * dr.Q.d2eta - dr.Q.dksideta ** 2
    dr.compute_u_spatial_ders()
    dr.P.val = dr.pressure(dr.U.val, dr.U.xx, dr.U.yy)
    dr.compute_P_spatial_ders()
    return dr.pde_rhs(dr.U.val, dr.U.xx, dr.U.yy)


def main():
    dr = load_reference()
    d = np.loadtxt(os.path.join(REF_DIR, INIT))
    U0, Q0 = d[:, 0].copy(), d[:, 1].copy()
    np.savez_compressed(os.path.join(OUT, "droplet_init.npz"), U0=U0, Q0=Q0)

    reset(dr, U0, Q0)
    F = step_fields(dr)
    rng = np.random.default_rng(2020)
    u1 = U0 * (1 + 0.01 * rng.standard_normal(U0.size))
    dt = 1e-4
    R1 = dr.residual(u1, F, dt)
    np.savez_compressed(
        os.path.join(OUT, "droplet_fields.npz"),
        Q_dksi=dr.Q.dksi, Q_deta=dr.Q.deta, Q_d2ksi=dr.Q.d2ksi, Q_d2eta=dr.Q.d2eta,
        Q_dksideta=dr.Q.dksideta, J=dr.J, U_dx=dr.U.dx, U_dy=dr.U.dy, U_xx=dr.U.xx, U_yy=dr.U.yy,
        P_val=dr.P.val, P_dx=dr.P.dx, P_dy=dr.P.dy, F=F, u1=u1, dt=dt, R1=R1)

    # one NK solve at the fixed step-1 mesh (:383)
    from scipy.optimize import newton_krylov
    nfev = [0]
    nit = [0]

    def Fres(u):
        nfev[0] += 1
        return dr.residual(u, F, dt)

    with contextlib.redirect_stdout(io.StringIO()):
        Unk = newton_krylov(Fres, dr.U.val, verbose=1, maxiter=20, f_tol=1e-7,
                            callback=lambda x, f: nit.__setitem__(0, nit[0] + 1))
    np.savez_compressed(os.path.join(OUT, "droplet_nk.npz"), U=Unk, nit=nit[0], nfev=nfev[0],
                        fnorm=np.abs(dr.residual(Unk, F, dt)).max())
    print("droplet NK: nit", nit[0], "nfev", nfev[0])

    # PMA mesh loop from the step-1 state (U/J of step_fields are the ones the first solve uses)
    out = {}
    for loops in (5, 400):
        reset(dr, U0, Q0)
        step_fields(dr)
        dr.loop_pma(3e-9, loops)
        out[f"Q_{loops}"] = dr.Q.val.copy()
    np.savez_compressed(os.path.join(OUT, "droplet_pma.npz"), **out)

    # two full time steps
    reset(dr, U0, Q0)
    log = io.StringIO()
    with contextlib.redirect_stdout(log):
        dr.evolve_with_PDE(1e-4, 3, 1e-2, 3e-9, 400)
    np.savez_compressed(os.path.join(OUT, "droplet_evolve.npz"), U=dr.U.new, Q=dr.Q.val,
                        Uval=dr.U.val, log=np.array(log.getvalue()))
    print(log.getvalue())


def evolve10():
    """S = 10 steps of evolve_with_PDE from the coal init state, every step recorded."""
    dr = load_reference()
    d = np.loadtxt(os.path.join(REF_DIR, INIT))
    U0, Q0 = d[:, 0].copy(), d[:, 1].copy()
    reset(dr, U0, Q0)
    rec = {"U": [], "Q": [], "nit": []}
    inner = dr.loop_pma
    real_nk = dr.newton_krylov
    nits = [0]

    def nk(*a, **kw):  # counts the Newton iterations of each step's solve
        cb = kw.pop("callback", None)
        nits[0] = 0

        def count(x, f):
            nits[0] += 1
            if cb:
                cb(x, f)
        return real_nk(*a, callback=count, **kw)

    def pma(dtmesh, loops):  # evolve_with_PDE calls it once per step, after the solve (:384)
        rec["nit"].append(nits[0])
        inner(dtmesh, loops)
        rec["U"].append(dr.U.new.copy())
        rec["Q"].append(dr.Q.val.copy())

    dr.loop_pma = pma
    dr.newton_krylov = nk
    log = io.StringIO()
    with contextlib.redirect_stdout(log):
        dr.evolve_with_PDE(1e-4, 11, 1e-2, 3e-9, 400)
    # "<it> 0.0001 * <scale> = <dt_n> . T = ..." per step (:408-409)
    dts = [float(ln.split("=")[1].split()[0]) for ln in log.getvalue().splitlines()
           if " * " in ln and ". T = " in ln]
    assert len(dts) == 10 and len(rec["U"]) == 10, (len(dts), len(rec["U"]))
    np.savez_compressed(os.path.join(OUT, "droplet_evolve10.npz"), U=np.array(rec["U"]),
                        Q=np.array(rec["Q"]), dt=np.array(dts), nit=np.array(rec["nit"]))
    print("dt", dts, "nit", rec["nit"])


if __name__ == "__main__":
    if sys.argv[1:] == ["evolve10"]:
        evolve10()
    else:
        main()

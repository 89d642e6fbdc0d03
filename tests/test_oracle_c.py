"""CPU: the C restatement of the SH arithmetic (oracle/c/sh_oracle.c) against the reference's
golden vectors, and its AddressSanitizer + UBSan self-check build.

The C restatement builds L as the reference does (two applications of Lap, sh_scipy_nk.py:38-39),
so matching the CSR fixtures pins that construction; the sanitizer build then checks it against
the closed-form 13-point coefficients the kernels use, on odd, rectangular and tiny grids."""
import ctypes as C
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import ROOT, load_golden
from oracle import sh_oracle

CDIR = os.path.join(ROOT, "oracle", "c")
BUILD = os.path.join(ROOT, "oracle", "_build")

pytestmark = pytest.mark.skipif(shutil.which("gcc") is None and shutil.which("cc") is None,
                                reason="no C compiler")


@pytest.fixture(scope="module")
def lib():
    subprocess.run(["make", "-s", "-C", CDIR, "all"], check=True)
    lib = C.CDLL(os.path.join(BUILD, "libsh_oracle.so"))
    P, I, D = C.c_void_p, C.c_int64, C.c_double
    lib.sho_lap5.argtypes = [P, P, I, I, D]
    lib.sho_lap5.restype = None
    lib.sho_sh13.argtypes = [P, P, I, I, D, D]
    lib.sho_residual.argtypes = [P, P, P, I, I, D, D, D, D]
    lib.sho_fd_closed.argtypes = [P, P, D, D, P, I, I, D, D, D, D]
    return lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


@pytest.mark.parametrize("name", ["ops_n5_d2", "ops_n61", "ops_n64", "ops_n128_h0625"])
def test_c_operators_match_reference_csr(lib, name):
    z = load_golden(name)
    N, h, r = int(z["N"]), float(z["h"]), float(z["r"])
    v = np.ascontiguousarray(z["v"])
    y = np.empty_like(v)
    lib.sho_lap5(_p(v), _p(y), N, N, 1.0 / h ** 2)
    assert np.abs(y - z["lap_v"]).max() <= 1e-13 * max(1.0, np.abs(z["lap_v"]).max())
    assert lib.sho_sh13(_p(v), _p(y), N, N, h, r) == 0
    assert np.abs(y - z["L_v"]).max() <= 1e-13 * max(1.0, np.abs(z["L_v"]).max())


def test_c_residual_matches_reference(lib):
    z = load_golden("residual_n61")
    N = int(z["N"])
    u, uo = np.ascontiguousarray(z["u"]), np.ascontiguousarray(z["uo"])
    F = np.empty_like(u)
    assert lib.sho_residual(_p(u), _p(uo), _p(F), N, N, float(z["h"]), float(z["r"]),
                            float(z["k"]), float(z["g"])) == 0
    assert np.abs(F - z["F"]).max() <= 1e-12 * max(1.0, np.abs(z["F"]).max())


def test_c_fd_closed_form_matches_numpy_oracle(lib):
    rng = np.random.default_rng(5)
    ny, nx, h = 24, 40, 0.625
    x0, zv = rng.standard_normal(ny * nx), rng.standard_normal(ny * nx)
    w = np.empty_like(x0)
    assert lib.sho_fd_closed(_p(x0), _p(zv), 1e-4, 0.3, _p(w), ny, nx, h, 0.01, 0.2, 1.0) == 0
    ref = sh_oracle.fd_quotient_closed_form(x0, zv, 1e-4, 0.3, ny, nx, h, 0.01, 0.2, 1.0)
    assert np.abs(w - ref).max() <= 1e-12 * max(1.0, np.abs(ref).max())


def test_c_restatement_clean_under_asan_ubsan():
    """The sanitizer build exits 0 with no report: no out-of-bounds access or undefined
    behaviour on 61x61, 5x5, 3x7, 1x1, 2x9, 64x48 and 17x128 periodic grids."""
    subprocess.run(["make", "-s", "-C", CDIR, "asan"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    out = subprocess.run([os.path.join(BUILD, "check_asan")], capture_output=True, text=True,
                         env=env, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.strip() == "ok"
    assert "ERROR: AddressSanitizer" not in out.stderr and "runtime error" not in out.stderr

"""The ARN_OPQ=2 question (round 5: the bounds-checked build with the stencil coefficients and x0
pinned through "+s" asm constraints returned NaN at nv 25-30 on the mailbox instantiation).  Under
the library NKHIP_LIB names and the mailbox mode NKHIP_ARN_MBOX (1: records, 2: every consumer
recomputes, so no record is ever polled), every fused instantiation nv 19..35 once on 32 x 1024
(the mailbox geometry of test_fused_kernel_mailbox_every_length) against an fp64 torch reference,
then one f_tol = 1e-10 solve per grid: non-finite outputs, the largest error, the solve's status
and the bounds counters (check builds).
    NKHIP_LIB=.../libnkhip_check_opq2.so python3 scripts/dbg/opq2_probe.py"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "iterative-solvers-summer-2020_amd"))
import nkhip  # noqa: E402
from nkhip import _lib  # noqa: E402


def G(y, h, r, k, g):
    e = 1.0 / h ** 2

    def lap(a):
        return e * (torch.roll(a, 1, 0) + torch.roll(a, -1, 0) + torch.roll(a, 1, 1)
                    + torch.roll(a, -1, 1) - 4 * a)
    la = lap(y)
    return y / k - ((-lap(la) - 2 * la + (r - 1) * y) + g * y * y - y * y * y) / 2


def bounds():
    n, line = C.c_int64(0), C.c_int32(0)
    rc = _lib.lib.nk_debug_bounds(C.byref(n), C.byref(line), 1)
    return None if rc != 0 else [n.value, line.value]


out = {"lib": os.path.basename(os.environ.get("NKHIP_LIB", "libnkhip.so")),
       "mbox": os.environ.get("NKHIP_ARN_MBOX", "1"), "kernel": {}, "solve": {}}
ny, nx = 32, 1024
h, r, k, g, tau, zs, sc = 0.625, 0.01, 0.2, 1.0, 0.75, 0.5, 1e-3
gen = torch.Generator(device="cpu").manual_seed(11)
Vall = [torch.randn(ny, nx, generator=gen, dtype=torch.float64).cuda() for _ in range(35)]
w = torch.randn(ny, nx, generator=gen, dtype=torch.float64).cuda()
x0 = torch.randn(ny, nx, generator=gen, dtype=torch.float64).cuda()
G0 = G(x0, h, r, k, g)
for nv in range(19, 36):
    V = Vall[:nv]
    coef = [0.3 / nv * (1 + (i % 3)) for i in range(nv)]
    v, wo, d = nkhip.sh_arnoldi_fused(V, coef, w, tau, x0, G0, h, r, k, g, zs, sc)
    vr = tau * w
    for c, Vi in zip(coef, V):
        vr = vr + c * Vi
    wr = (G(x0 + sc * zs * vr, h, r, k, g) - G0) / sc
    out["kernel"][nv] = {"nonfinite": int((~torch.isfinite(v)).sum() + (~torch.isfinite(wo)).sum()),
                         "dots_nonfinite": int(sum(not np.isfinite(x) for x in d)),
                         "v_err": float((v - vr).abs().max() / vr.abs().max()),
                         "w_err": float((wo - wr).abs().max() / wr.abs().max())}
out["kernel_bounds"] = bounds()
for gy, gx in ((64, 1024), (128, 1024), (40, 512)):
    m = nkhip.SwiftHohenberg(N=gx, ny=gy, d=0.625 * gx, f_tol=1e-10)
    U = torch.as_tensor(np.random.default_rng(2020).standard_normal((gy, gx)), device="cuda")
    try:
        U1 = m.step(U)
        out["solve"][f"{gy}x{gx}"] = {"status": 0, "nit": m.last_stats["nit"],
                                      "nonfinite": int((~torch.isfinite(U1)).sum())}
    except Exception as e:  # noqa: BLE001
        out["solve"][f"{gy}x{gx}"] = {"error": str(e)[:200]}
    m.close()
out["solve_bounds"] = bounds()
print(json.dumps(out), flush=True)

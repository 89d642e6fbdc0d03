"""Where the round-5 ARN_OPQ=2 check build's fused kernel goes wrong (scripts/dbg/opq2_probe.py
found w' wrong and v right at nv 25 on 32 x 1024, identical with NKHIP_ARN_MBOX 1 and 2): the
error pattern of w' against the library's own product build -- which rows / columns / lanes,
and whether w' is off by a factor (a wrong scalar: the FD step, a stencil coefficient) or
locally (a wrong row or register).
    NKHIP_LIB=.../libnkhip_r05_check_opq2.so python3 scripts/dbg/opq2_pattern.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "iterative-solvers-summer-2020_amd"))
import nkhip  # noqa: E402


def G(y, h, r, k, g):  # G(y) = y/k - (L y + g y^2 - y^3)/2 by periodic rolls (opq2_probe.py)
    e = 1.0 / h ** 2

    def lap(a):
        return e * (torch.roll(a, 1, 0) + torch.roll(a, -1, 0) + torch.roll(a, 1, 1)
                    + torch.roll(a, -1, 1) - 4 * a)
    la = lap(y)
    return y / k - ((-lap(la) - 2 * la + (r - 1) * y) + g * y * y - y * y * y) / 2


ny, nx, nv = 32, 1024, int(os.environ.get("NV", "25"))
h, r, k, g, tau, zs, sc = 0.625, 0.01, 0.2, 1.0, 0.75, 0.5, 1e-3
gen = torch.Generator(device="cpu").manual_seed(11)
Vall = [torch.randn(ny, nx, generator=gen, dtype=torch.float64).cuda() for _ in range(35)]
w = torch.randn(ny, nx, generator=gen, dtype=torch.float64).cuda()
x0 = torch.randn(ny, nx, generator=gen, dtype=torch.float64).cuda()
G0 = G(x0, h, r, k, g)
V = Vall[:nv]
coef = [0.3 / nv * (1 + (i % 3)) for i in range(nv)]
v, wo, d = nkhip.sh_arnoldi_fused(V, coef, w, tau, x0, G0, h, r, k, g, zs, sc)
vr = tau * w
for c, Vi in zip(coef, V):
    vr = vr + c * Vi
wr = (G(x0 + sc * zs * vr, h, r, k, g) - G0) / sc
err = (wo - wr).abs()
bad = err > 1e-9 * wr.abs().max()
rows = bad.any(dim=1).nonzero().flatten().tolist()
cols = bad.any(dim=0).nonzero().flatten().tolist()
ratio = (wo[bad] / wr[bad]) if bad.any() else torch.empty(0)
out = {"nv": nv, "bad_points": int(bad.sum()), "of": ny * nx, "bad_rows": rows,
       "bad_cols_mod128": sorted(set(c % 128 for c in cols))[:64], "n_bad_cols": len(cols),
       "ratio_min": float(ratio.min()) if ratio.numel() else None,
       "ratio_max": float(ratio.max()) if ratio.numel() else None,
       "v_err": float((v - vr).abs().max() / vr.abs().max())}
print("PATTERN " + json.dumps(out), flush=True)

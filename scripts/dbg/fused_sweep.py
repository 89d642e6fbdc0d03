"""Every basis length through the fused kernel vs an fp64 torch reference, with and
without edge arrays, twice (determinism).  Prints the worst relative errors; no asserts."""
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "iterative-solvers-summer-2020_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import nkhip  # noqa: E402
from test_gpu_fused import _torch_G  # noqa: E402

h, r, k, g, tau, zs, sc = 0.625, 0.01, 0.2, 1.0, 0.75, 0.5, 1e-3
for ny, nx in [(40, 256), (96, 130), (12, 40), (64, 64)]:
    for nv in range(1, 35):
        gen = torch.Generator(device="cpu").manual_seed(nv * 7 + nx)
        rnd = lambda: torch.randn(ny, nx, generator=gen, dtype=torch.float64).cuda()  # noqa
        V = [rnd() for _ in range(nv)]
        coef = [float(c) for c in torch.randn(nv, generator=gen, dtype=torch.float64)]
        w, x0 = rnd(), rnd()
        G0 = _torch_G(x0, h, r, k, g)
        vr = tau * w
        for c, Vi in zip(coef, V):
            vr = vr + c * Vi
        wr = (_torch_G(x0 + sc * zs * vr, h, r, k, g) - G0) / sc
        E = [nkhip.edge_gather(t) for t in V + [w]]
        out = []
        for useE in (False, True, True):
            v, wo, d = nkhip.sh_arnoldi_fused(V, coef, w, tau, x0, G0, h, r, k, g, zs, sc,
                                              E=E if useE else None)
            out.append((v, wo, d))
        ev = float((out[0][0] - vr).abs().max() / vr.abs().max())
        ew = float((out[0][1] - wr).abs().max() / wr.abs().max())
        ewE = float((out[1][1] - wr).abs().max() / wr.abs().max())
        det = torch.equal(out[1][1], out[2][1]) and out[1][2] == out[2][2]
        flag = "" if (ew < 1e-9 and ewE < 1e-9 and det) else "   <-- BAD"
        print(f"{ny}x{nx} nv={nv:2d} v {ev:.1e} w' {ew:.1e} w'(E) {ewE:.1e} det {det}{flag}",
              flush=True)

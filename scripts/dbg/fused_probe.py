import sys, os
import torch
sys.path.insert(0, "."); sys.path.insert(0, "tests"); sys.path.insert(0, "iterative-solvers-summer-2020_amd")
import nkhip
from test_gpu_fused import _torch_G
ny, nx, nv = 16, 64, 1
g = torch.Generator().manual_seed(1)
rnd = lambda: torch.randn(ny, nx, generator=g, dtype=torch.float64).cuda()
V = [rnd() for _ in range(nv)]; w = rnd(); x0 = rnd()
h, r, k, gg, tau = 0.625, 0.01, 0.2, 1.0, 0.75
G0 = _torch_G(x0, h, r, k, gg)
zs, sc = 0.5, 1e-3
for label, G0in in (("G0", G0), ("zero", torch.zeros_like(G0))):
    v, wo, d = nkhip.sh_arnoldi_fused(V, [0.3], w, tau, x0, G0in, h, r, k, gg, zs, sc)
    vr = tau * w + 0.3 * V[0]
    Gy = _torch_G(x0 + sc * zs * vr, h, r, k, gg)
    wr = (Gy - G0in) / sc
    print(label, "v err", float((v - vr).abs().max()), "w err", float((wo - wr).abs().max()))
    # what G did the kernel use? G_k = wo*sc + G0in
    Gk = wo * sc + G0in
    print("  G err", float((Gk - Gy).abs().max()), "G(x0+0) err", float((Gk - _torch_G(x0, h, r, k, gg)).abs().max()))
    print("  row0", (Gk - Gy)[0, :8].tolist())
    print("  row5", (Gk - Gy)[5, :8].tolist())

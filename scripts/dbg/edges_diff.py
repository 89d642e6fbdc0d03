"""test_fused_kernel_edges_identical's cases, every one (not stopping at the first): for each,
whether v / w' / dots of the vector path and the edge-array path agree bitwise, and where w'
differs (rows, columns, max relative difference).  Run once per library (NKHIP_LIB) to tell
which path and which build moved.  Prints one JSON line per case; the outputs are also saved
(gpurun_out/<tag>_edges.pt) for a cross-library comparison.
    NKHIP_LIB=... python3 scripts/dbg/edges_diff.py <tag>"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "iterative-solvers-summer-2020_amd"))
import nkhip  # noqa: E402



def G(y, h, r, k, g):  # G(y) = y/k - (L y + g y^2 - y^3)/2 by periodic rolls (opq2_pattern.py)
    e = 1.0 / h ** 2

    def lap(a):
        return e * (torch.roll(a, 1, 0) + torch.roll(a, -1, 0) + torch.roll(a, 1, 1)
                    + torch.roll(a, -1, 1) - 4 * a)
    la = lap(y)
    return y / k - ((-lap(la) - 2 * la + (r - 1) * y) + g * y * y - y * y * y) / 2


tag = sys.argv[1] if len(sys.argv) > 1 else "x"
saved = {}
for ext in (False, True):
    for ny, nx in [(64, 64), (40, 130), (24, 600), (16, 4), (8, 512)]:
        nv = 7
        gen = torch.Generator(device="cpu").manual_seed(nx + ny)
        rnd = lambda: torch.randn(ny, nx, generator=gen, dtype=torch.float64).cuda()  # noqa: E731
        V = [rnd() for _ in range(nv)]
        coef = [float(c) for c in torch.randn(nv, generator=gen, dtype=torch.float64)]
        w, x0 = rnd(), rnd()
        z = rnd() if ext else None
        args = (V, coef, w, 0.75, x0, None, 0.625, 0.01, 0.2, 1.0, 0.5, 1e-3)
        v1, w1, d1 = nkhip.sh_arnoldi_fused(*args, z=z)
        E = [nkhip.edge_gather(t) for t in V + [w]]
        Ev = torch.full_like(E[0], float("nan"))
        Ew = torch.full_like(E[0], float("nan"))
        v2, w2, d2 = nkhip.sh_arnoldi_fused(*args, z=z, E=E, Ev_out=Ev, Ew_out=Ew)
        torch.cuda.synchronize()
        dw = (w1 != w2)
        u = (z if ext else None)
        if u is None:
            u = 0.75 * w
            for c, Vi in zip(coef, V):
                u = u + c * Vi
        wr = (G(x0 + 1e-3 * 0.5 * u, 0.625, 0.01, 0.2, 1.0) - G(x0, 0.625, 0.01, 0.2, 1.0)) / 1e-3
        rel = lambda a: float(((a - wr).abs().max() / wr.abs().max()).item())  # noqa: E731
        out = {"ext": ext, "ny": ny, "nx": nx, "v_eq": bool(torch.equal(v1, v2)),
               "w_eq": bool(torch.equal(w1, w2)), "d_eq": d1 == d2,
               "w_bad_rows": dw.any(dim=1).nonzero().flatten().tolist()[:40],
               "w_bad_cols": dw.any(dim=0).nonzero().flatten().tolist()[:40],
               "w_nbad": int(dw.sum()),
               "w_maxrel": float(((w1 - w2).abs().max() / w1.abs().max()).item()),
               "w1_err": rel(w1), "w2_err": rel(w2)}
        print("EDGES " + json.dumps(out), flush=True)
        saved[f"{ext}-{ny}-{nx}"] = (v1.cpu(), w1.cpu(), torch.tensor(d1), v2.cpu(), w2.cpu(),
                                     torch.tensor(d2))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
torch.save(saved, os.path.join(ROOT, "gpurun_out", f"{tag}_edges.pt"))

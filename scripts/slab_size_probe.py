"""Per-rank work of the strong-scaling line at N GPUs, measured on one: a periodic ny x 4096 grid
(ny = 4096 / N rows, the rank's slab without its exchange) stepped from default_rng(2020), ms per
Arnoldi step and that time per row against the full grid's -- how much the fused kernel loses on
short slabs (short bands, ramp, tail), which bounds the N = 8 efficiency before any xGMI cost.
    python3 scripts/slab_size_probe.py [ny ...]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "iterative-solvers-summer-2020_amd"))
import nkhip  # noqa: E402


def run(ny, nx=4096, warmup=2, steps=4):
    U0 = np.random.default_rng(2020).standard_normal((ny, nx))
    m = nkhip.SwiftHohenberg(N=nx, ny=ny, d=0.625 * nx, profile=8)
    a = torch.as_tensor(U0, device="cuda")
    b = torch.empty_like(a)
    for _ in range(warmup):
        m.step(a, out=b)
        a, b = b, a
    m.reset_profile()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    narn = 0
    for _ in range(steps):
        m.step(a, out=b)
        narn += m.last_stats["njvp"]
        a, b = b, a
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    prof = m.kernel_profile()
    m.close()
    f = prof.get("arnoldi_fused", {})
    us = 1e3 * f["ms"] / f["timed"] if f.get("timed") else None
    gbs = f["timed_bytes"] / (f["ms"] * 1e-3) / 1e9 if f.get("timed") else None
    return {"ny": ny, "ms_per_arnoldi": round(1e3 * dt / max(narn, 1), 4),
            "us_per_arnoldi_per_1k_rows": round(1e6 * dt / max(narn, 1) / ny * 1024, 2),
            "fused_avg_us": round(us, 1) if us else None,
            "fused_frac": round(gbs / 8000, 4) if gbs else None}


if __name__ == "__main__":
    for ny in [int(a) for a in sys.argv[1:]] or [4096, 2048, 1024, 512]:
        print(json.dumps(run(ny)), flush=True)

"""Does the fused kernel's speed depend on where the solver's vector pool lands in HBM?  Several
steppers (each with its own pool) in ONE process, stepped alternately from the same state;
prints the fused kernel's fraction of 8 TB/s per stepper and round (profiles/
r03_pool_placement.md).

POOLS: comma list, one stepper per entry: "m" = a hipMalloc pool (NKHIP_POOL_ALLOC=malloc),
"v" = the default chunk-mapped pool.  MODES: comma list of "<mbox>/<edges>" settings cycled
over the rounds (NKHIP_ARN_MBOX, NKHIP_EDGES; both are read per call)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "iterative-solvers-summer-2020_amd")]
import nkhip  # noqa: E402

n = int(os.environ.get("N", "4096"))
pools = os.environ.get("POOLS", "m,v,m,v").split(",")
U0 = torch.as_tensor(np.random.default_rng(2020).standard_normal((n, n)), device="cuda")
os.environ["NKHIP_DEBUG_POOL"] = "1"
models = []
for kind in pools:
    if kind == "m":
        os.environ["NKHIP_POOL_ALLOC"] = "malloc"
    else:
        os.environ.pop("NKHIP_POOL_ALLOC", None)
    models.append(nkhip.SwiftHohenberg(N=n, d=0.625 * n, profile=8))
os.environ.pop("NKHIP_POOL_ALLOC", None)
U1 = models[0].step(U0)
U2 = models[0].step(U1)
modes = os.environ.get("MODES", "1/1").split(",")
for rnd in range(3 * len(modes)):
    mbx, edg = modes[rnd % len(modes)].split("/")
    os.environ["NKHIP_ARN_MBOX"] = mbx
    os.environ["NKHIP_EDGES"] = edg
    for i, m in enumerate(models):
        m.reset_profile()
        torch.cuda.synchronize()
        t = time.perf_counter()
        a = m.step(U2)
        b = m.step(a)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        prof = m.kernel_profile()
        p = prof["arnoldi_fused"]
        frac = p["timed_bytes"] / (p["ms"] * 1e-3) / 8e12
        c = prof["krylov_combo"]
        cf = c["timed_bytes"] / (c["ms"] * 1e-3) / 8e12 if c["ms"] > 0 else 0.0
        print(f"round {rnd} mbox/edges {modes[rnd % len(modes)]} model {i} ({pools[i]}): "
              f"{dt * 1e3:.1f} ms for 2 steps, fused frac {frac:.4f}, combo {cf:.4f}", flush=True)

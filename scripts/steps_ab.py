"""Wall time of K implicit 4096^2 steps without kernel events (NKHIP_BENCH_PROFILE-free), for A/B
of solver switches in one process:  python scripts/steps_ab.py VAR=0,VAR=1 ...
Each comma-separated spec sets environment variables for one pass; passes alternate twice over
the same starting state.  Prints one JSON line per pass (ms per step, per Arnoldi step)."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-solvers-summer-2020_amd"))
import nkhip  # noqa: E402


def main():
    specs = sys.argv[1:] or ["NKHIP_DEVCTL=1", "NKHIP_DEVCTL=0"]
    n, steps, warm = int(os.environ.get("N", "4096")), int(os.environ.get("STEPS", "12")), 2
    h, k, r, g = 0.625, 0.2, 0.01, 1.0
    U0 = torch.as_tensor(np.random.default_rng(2020).standard_normal((n, n)), device="cuda")
    model = nkhip.SwiftHohenberg(N=n, d=h * n, k=k, r=r, g=g, profile=0)
    a, b = U0.clone(), torch.empty_like(U0)
    for _ in range(warm):
        model.step(a, out=b)
        a, b = b, a
    start = a.clone()
    for rep in range(2):
        for spec in specs:
            for kv in spec.split(","):
                key, val = kv.split("=")
                os.environ[key] = val
            a.copy_(start)
            arn = 0
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                model.step(a, out=b)
                arn += model.last_stats["n_arnoldi"]
                a, b = b, a
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(json.dumps({"rep": rep, "spec": spec, "ms_per_step": round(1e3 * dt / steps, 3),
                              "ms_per_arnoldi_step": round(1e3 * dt / arn, 4), "arnoldi": arn,
                              "device_steps": model.last_stats.get("n_device_steps")}), flush=True)


if __name__ == "__main__":
    main()

"""BASELINE config 2 alone: the 1024^2 fp64 periodic 5-point Laplacian (sh_scipy_nk.py:32-35),
`reps` back-to-back launches of nk_lap5_apply on resident inputs, for a kernel-only rocprofv3
trace (scripts/profile_config2.sh).  Prints one JSON line with the HIP-event average per launch
(gaps included) and the error against the oracle stencil."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-solvers-summer-2020_amd"))
sys.path.insert(0, ROOT)
import nkhip  # noqa: E402
from oracle import sh_oracle  # noqa: E402


def main():
    n, h, reps = 1024, 0.625, int(os.environ.get("REPS", "200"))
    v_np = np.random.default_rng(7).standard_normal(n * n)
    v = torch.as_tensor(v_np.reshape(n, n), device="cuda")
    y = torch.empty_like(v)
    for _ in range(5):
        nkhip.lap5_apply(v, 1 / h ** 2, out=y)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        nkhip.lap5_apply(v, 1 / h ** 2, out=y)
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / reps
    err = float(np.abs(y.cpu().numpy().reshape(-1) - sh_oracle.lap5(v_np, n, n, 1 / h ** 2)).max())
    print(json.dumps({"workload": "lap5_1024x1024_fp64", "launches": reps + 5,
                      "event_us_per_launch_incl_gap": round(us, 3),
                      "alg_bytes_per_launch": 16 * n * n, "max_abs_err_vs_oracle": err}))


if __name__ == "__main__":
    main()

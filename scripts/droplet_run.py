#!/usr/bin/env python3
"""Run N droplet steps (config 3) from the reference's coal init state; for profiling."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-solvers-summer-2020_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import nkhip  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
with np.load(os.path.join(ROOT, "tests", "golden", "droplet_init.npz")) as z:
    U0, Q0 = z["U0"], z["Q0"]
d = nkhip.Droplet(profile=True)
d.set_state(U0, Q0)
torch.cuda.synchronize()
t0 = time.perf_counter()
for s in range(steps):
    t1 = time.perf_counter()
    d.step()
    torch.cuda.synchronize()
    print("step", s, "s", round(time.perf_counter() - t1, 4), d.last_stats, flush=True)
print("total", time.perf_counter() - t0)

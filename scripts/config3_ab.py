#!/usr/bin/env python3
"""Config 3 (droplet, 91x61, 400 PMA loops per step) and PMA2 steps/s as bench.py measures them,
without the CPU legs: one line per run, for A/B of runtime switches (NKHIP_DEVCTL ...)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "iterative-solvers-summer-2020_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import nkhip  # noqa: E402

with np.load(os.path.join(ROOT, "tests", "golden", "droplet_init.npz")) as z:
    U0, Q0 = z["U0"], z["Q0"]
d = nkhip.Droplet()
d.set_state(U0, Q0)
d.step()
d.set_state(U0, Q0)
torch.cuda.synchronize()
t0 = time.perf_counter()
nits, narn = 0, 0
for _ in range(5):
    d.step(1e-4, 3e-9, 400)
    nits += d.last_stats["nit"]
    narn += d.last_stats["n_arnoldi"]
torch.cuda.synchronize()
drop = 5 / (time.perf_counter() - t0)
Uend = d.get_state()[0] if hasattr(d, "get_state") else None
d.close()
m = nkhip.Mems()
m.step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    m.step()
torch.cuda.synchronize()
pma2 = 20 / (time.perf_counter() - t0)
m.close()
print(json.dumps({"env": sys.argv[1:] or os.environ.get("NKHIP_DEVCTL", "default"),
                  "config3_steps_per_s": round(drop, 2), "newton_its": nits, "arnoldi": narn,
                  "pma2_steps_per_s": round(pma2, 1)}), flush=True)

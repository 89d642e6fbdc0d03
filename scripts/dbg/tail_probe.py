"""Stage times of the fused launch's tail (ARN_TAIL_PROBE build, scripts/arn_variant_build.sh
tprobe -DARN_TAIL_PROBE): a few device-controlled 4096^2 steps, then the summed wall-clock ticks
(100 MHz) of each stage per tail."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "iterative-solvers-summer-2020_amd"))
os.environ["NKHIP_DEVCTL"] = "1"
import nkhip  # noqa: E402
from nkhip import _lib  # noqa: E402

n = int(os.environ.get("N", "4096"))
U = torch.as_tensor(np.random.default_rng(2020).standard_normal((n, n)), device="cuda")
m = nkhip.SwiftHohenberg(N=n, d=0.625 * n, k=0.2, r=0.01, g=1.0, profile=0)
out = (C.c_ulonglong * 8)()
U = m.step(U)
_lib.lib.nk_debug_tail_probe(out)
for _ in range(3):
    U = m.step(U)
assert _lib.lib.nk_debug_tail_probe(out) == 0
cnt = max(out[0], 1)
names = ["first arrival -> controller's arrival", "-> all arrived", "-> all reduced",
         "-> all-reduced", "-> control done"]
print(f"tails {out[0]}")
for i, nm in enumerate(names):
    print(f"{nm:40s} {out[i + 1] / cnt / 100:.2f} us")

"""One fused solve under the bounds-checked library (NKHIP_LIB=.../libnkhip_check.so), then the
first out-of-range source line nk_debug_bounds recorded.  python3 scripts/dbg/bounds_probe.py ny nx"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "iterative-solvers-summer-2020_amd"))
os.environ.setdefault("NKHIP_LIB", os.path.join(ROOT, "iterative-solvers-summer-2020_amd", "nkhip",
                                                "libnkhip_check.so"))
import nkhip  # noqa: E402
from nkhip import _lib  # noqa: E402

ny, nx = int(sys.argv[1]), int(sys.argv[2])
m = nkhip.SwiftHohenberg(N=nx, ny=ny, d=0.625 * nx, f_tol=1e-10)
U = torch.as_tensor(np.random.default_rng(2020).standard_normal((ny, nx)), device="cuda")
try:
    U = m.step(U)
    print("step ok", m.last_stats)
except Exception as e:  # noqa: BLE001
    print("step failed:", e)
n, line = C.c_int64(), C.c_int32()
print("nk_debug_bounds rc", _lib.lib.nk_debug_bounds(C.byref(n), C.byref(line), 1),
      "violations", n.value, "first line", line.value)

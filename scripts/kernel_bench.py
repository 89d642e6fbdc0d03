#!/usr/bin/env python3
"""Per-kernel microbenchmarks (configs 2 and 4 kernels) with HIP events on torch's stream.

* config 2: 1024^2 fp64 periodic 5-point Laplacian SpMV (sh_scipy_nk.py:32-35), 16 B/pt
* 13-point L apply (sh_scipy_nk.py:38-39) and the analytic JVP at 1024^2 .. 8192^2
Prints one JSON line per kernel/size: avg us, algorithmic GB/s, fraction of 8 TB/s.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "iterative-solvers-summer-2020_amd"))

import torch  # noqa: E402

import nkhip  # noqa: E402

PEAK = 8000.0


def timeit(fn, reps):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps  # us


def main():
    sizes = [int(s) for s in (sys.argv[1:] or ["1024", "2048", "4096", "8192"])]
    only = os.environ.get("KB_ONLY")
    h, r, k, g = 0.625, 0.01, 0.2, 1.0
    for n in sizes:
        gen = torch.Generator(device="cuda").manual_seed(7)
        v = torch.randn(n, n, dtype=torch.float64, device="cuda", generator=gen)
        u = torch.randn(n, n, dtype=torch.float64, device="cuda", generator=gen)
        y = torch.empty_like(v)
        g0 = torch.randn(n, n, dtype=torch.float64, device="cuda", generator=gen)
        reps = max(5, int(2e9 / (n * n * 16)))
        cases = [
            ("lap5", 16, lambda: nkhip.lap5_apply(v, 1 / h ** 2, out=y)),
            ("sh13", 16, lambda: nkhip.sh13_apply(v, h, r, out=y)),
            ("sh_jvp_analytic", 24, lambda: nkhip.sh_jvp(u, v, h, r, k, g, out=y)),
            ("sh_residual_ref", 24, lambda: nkhip.sh_residual(u, v, h, r, k, g, out=y)),
            ("sh_fdjvp", 32, lambda: nkhip.sh_fdjvp(u, g0, v, h, r, k, g, 1.0, 1e-7, out=y)),
            ("torch_copy", 16, lambda: y.copy_(v)),
            # same traffic mix as the FD JVP (3 streams read, 1 written): the practical roofline
            ("torch_addcmul_3r1w", 32, lambda: torch.addcmul(u, v, g0, out=y)),
            ("torch_add_2r1w", 24, lambda: torch.add(u, v, out=y)),
        ]
        for name, bpp, fn in cases:
            if only and name not in only.split(","):
                continue
            us = timeit(fn, reps)
            gbs = bpp * n * n / (us * 1e-6) / 1e9
            print(json.dumps({"kernel": name, "n": n, "avg_us": round(us, 2),
                              "alg_GBps": round(gbs, 1), "frac_peak": round(gbs / PEAK, 4)}),
                  flush=True)


if __name__ == "__main__":
    main()

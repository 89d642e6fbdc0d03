"""Microbenchmark of the fused Arnoldi step (csrc/arnoldi.hip) at 4096^2 over the basis length.

Prints one line per (nv, ext): average kernel time (HIP events around 20 launches, no reduction)
and the algorithmic rate 8 n (nv + 4 + ext) bytes / time against the 8 TB/s HBM peak.  Tuning
knobs are environment variables read once per process (NKHIP_ARN_PF, NKHIP_ARN_NT,
NKHIP_ARN_ROUNDS), so compare configurations in separate processes.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "iterative-solvers-summer-2020_amd"))
import nkhip  # noqa: E402


def main():
    N = int(os.environ.get("ARN_N", "4096"))
    nvs = [int(x) for x in os.environ.get("ARN_NVS", "1,4,8,12,16,20,24,28,32,35").split(",")]
    n = N * N
    torch.manual_seed(0)
    V = [torch.randn(N, N, dtype=torch.float64, device="cuda") for _ in range(max(nvs))]
    w, x0, z, G0 = (torch.randn(N, N, dtype=torch.float64, device="cuda") for _ in range(4))
    vo = torch.empty_like(w)
    wo = torch.empty_like(w)
    # ARN_EDGES=1: block halos from edge arrays (the solver's default), the outputs' written
    edges = os.environ.get("ARN_EDGES", "1") == "1"
    EV = [nkhip.edge_gather(t) for t in V] if edges else None
    Ew = nkhip.edge_gather(w) if edges else None
    Evo, Ewo = (torch.empty_like(Ew), torch.empty_like(Ew)) if edges else (None, None)
    out = []
    for ext in (False, True):
        for nv in nvs:
            coef = [0.01] * nv
            args = (V[:nv], coef, w, 1.0, x0, G0, 0.625, 0.01, 0.2, 1.0, 1.0, 1e-7)
            kw = dict(z=z if ext else None, v_out=vo, w_out=wo, reduce=False)
            if edges:
                kw.update(E=EV[:nv] + [Ew], Ev_out=Evo, Ew_out=Ewo)
            for _ in range(3):
                nkhip.sh_arnoldi_fused(*args, **kw)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 20
            a.record()
            for _ in range(reps):
                nkhip.sh_arnoldi_fused(*args, **kw)
            b.record()
            torch.cuda.synchronize()
            us = a.elapsed_time(b) * 1e3 / reps
            byt = 8.0 * n * (nv + 4 + (1 if ext else 0))
            out.append({"nv": nv, "ext": ext, "us": round(us, 2),
                        "GBps": round(byt / us / 1e3, 1), "frac": round(byt / us / 1e3 / 8000, 3)})
            print(json.dumps(out[-1]), flush=True)
    tag = os.environ.get("ARN_TAG", "")
    if tag:
        os.makedirs("gpurun_out", exist_ok=True)
        with open(f"gpurun_out/arn_{tag}.json", "w") as f:
            json.dump(out, f)


if __name__ == "__main__":
    main()

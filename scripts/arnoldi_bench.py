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
    # vectors carved from one pool with the solver's stride (Engine::pad: an odd multiple of
    # 128 KiB, which spreads the vectors' rows over the HBM channels); separately allocated torch
    # tensors sit at 2-MiB-aligned strides and stream very differently (ARN_POOL=0)
    nvec = max(nvs) + 6
    if os.environ.get("ARN_POOL", "1") == "1":
        p = (n + 255) // 256 * 256
        stride = (p + 32767) // 32768 * 32768 + 16384
        pool = torch.randn(nvec * stride, dtype=torch.float64, device="cuda")
        vecs = [pool[i * stride:i * stride + n].view(N, N) for i in range(nvec)]
    else:
        vecs = [torch.randn(N, N, dtype=torch.float64, device="cuda") for _ in range(nvec)]
    V = vecs[:max(nvs)]
    w, x0, z, G0, c1, c2 = vecs[max(nvs):]
    if os.environ.get("ARN_POOL", "1") == "1":
        out = torch.empty(2 * stride, dtype=torch.float64, device="cuda")
        vo, wo = out[:n].view(N, N), out[stride:stride + n].view(N, N)
    else:
        vo = torch.empty_like(w)
        wo = torch.empty_like(w)
    # ARN_EDGES=1: block halos from edge arrays (the solver's default), the outputs' written
    edges = os.environ.get("ARN_EDGES", "1") == "1"
    EV = [nkhip.edge_gather(t) for t in V] if edges else None
    Ew = nkhip.edge_gather(w) if edges else None
    Evo, Ewo = (torch.empty_like(Ew), torch.empty_like(Ew)) if edges else (None, None)
    Ec = [nkhip.edge_gather(t) for t in (vo, wo, c1, c2)] if edges else None
    out = []
    for ext in (False, True):
        for nv in nvs:
            coef = [0.01] * nv
            args = (V[:nv], coef, w, 1.0, x0, G0, 0.625, 0.01, 0.2, 1.0, 1.0, 1e-7)
            kw = dict(z=z if ext else None, v_out=vo, w_out=wo, reduce=False)
            if edges:
                kw.update(E=EV[:nv] + [Ew], Ev_out=Evo, Ew_out=Ewo)
            chain = os.environ.get("ARN_CHAIN", "1") == "1"
            # ARN_CHAIN=1 (default): as in the solver, each launch reads the previous launch's
            # outputs -- w = its w', the newest basis vector = its v (the buffers rotate; edge
            # arrays follow); 0: the same inputs every time
            bufs = [vo, wo, c1, c2] if chain else None

            def one(i):
                if not chain:
                    nkhip.sh_arnoldi_fused(*args, **kw)
                    return
                iv, iw, ov, ow = ((2 * i + k) % 4 for k in (0, 1, 2, 3))
                Vl = V[:nv - 1] + [bufs[iv]]
                a2 = (Vl,) + args[1:2] + (bufs[iw],) + args[3:]
                k2 = dict(kw, v_out=bufs[ov], w_out=bufs[ow])
                if edges:
                    k2.update(E=EV[:nv - 1] + [Ec[iv], Ec[iw]], Ev_out=Ec[ov], Ew_out=Ec[ow])
                nkhip.sh_arnoldi_fused(*a2, **k2)

            for i in range(3):
                one(i)
            torch.cuda.synchronize()
            mbstat = os.environ.get("ARN_MBSTAT") == "1"  # the mailbox statistics build
            if mbstat:
                import ctypes as C
                from nkhip import _lib
                cnt = (C.c_int64 * 4)()
                _lib.lib.nk_debug_mailbox(cnt, 1)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 20
            a.record()
            for i in range(reps):
                one(i)
            b.record()
            torch.cuda.synchronize()
            us = a.elapsed_time(b) * 1e3 / reps
            byt = 8.0 * n * (nv + 4 + (1 if ext else 0))
            out.append({"nv": nv, "ext": ext, "us": round(us, 2),
                        "GBps": round(byt / us / 1e3, 1), "frac": round(byt / us / 1e3 / 8000, 3)})
            if mbstat:
                rc = _lib.lib.nk_debug_mailbox(cnt, 1)
                out[-1]["mailbox_per_launch"] = (
                    {k: cnt[i] / reps for i, k in enumerate(("needed", "late", "extra_polls",
                                                             "recomputed"))} if rc == 0 else rc)
            print(json.dumps(out[-1]), flush=True)
    tag = os.environ.get("ARN_TAG", "")
    if tag:
        os.makedirs("gpurun_out", exist_ok=True)
        with open(f"gpurun_out/arn_{tag}.json", "w") as f:
            json.dump(out, f)


if __name__ == "__main__":
    main()

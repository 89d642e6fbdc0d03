"""Rehearse the driver's N-GPU decomposition of the bench workload on ONE GPU.

bench.py --gpus N cuts the 4096^2 grid into N row slabs, one process per GPU over RCCL.  Here the
same N slabs run on one GPU through the loopback communicator (one host thread per slab, the same
halo/all-reduce protocol and the same fused-kernel slab path), so the decomposition at the real
size is checked before the 8-GPU job: every slab takes the same Newton decisions, and the
assembled state is a root of the oracle residual, as close to the single periodic slab as the
changed summation order allows.  Timing here is NOT a scaling number (all slabs share one GPU).

Usage on the GPU box: python scripts/loopback_rehearsal.py [N] [slabs,...]
"""
import json
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "iterative-solvers-summer-2020_amd"))
sys.path.insert(0, ROOT)
import nkhip  # noqa: E402
from oracle import sh_oracle  # noqa: E402  (checker only)


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    slabs = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "2,4,8").split(",")]
    h, k, r, g = 0.625, 0.2, 0.01, 1.0
    U0 = np.random.default_rng(2020).standard_normal((N, N))
    single = nkhip.SwiftHohenberg(N=N, d=h * N, k=k, r=r, g=g)
    ref = single.step(torch.as_tensor(U0, device="cuda")).cpu().numpy()
    ref_st = dict(single.last_stats)
    single.close()
    print(json.dumps({"slabs": 1, "nit": ref_st["nit"], "njvp": ref_st["njvp"]}), flush=True)
    for P in slabs:
        comms = nkhip.loopback_comms(P)
        out, stats, profs, errs = [None] * P, [None] * P, [None] * P, []

        def run(p):
            try:
                stream = torch.cuda.Stream()
                with torch.cuda.stream(stream):
                    row0, ny = nkhip.slab_rows(N, p, P)
                    m = nkhip.SwiftHohenberg(N=N, d=h * N, k=k, r=r, g=g, comm=comms[p],
                                             ny_local=ny, stream=stream)
                    u = torch.as_tensor(U0[row0:row0 + ny].copy(), device="cuda")
                    out[p] = m.step(u).cpu().numpy()
                    stats[p] = dict(m.last_stats)
                    profs[p] = m.kernel_profile()
                    stream.synchronize()
                    m.close()
            except BaseException as e:  # noqa: BLE001
                errs.append(repr(e))
                comms[p].abort()  # peers leave their collectives instead of blocking

        t0 = time.perf_counter()
        th = [threading.Thread(target=run, args=(p,)) for p in range(P)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=600)
        dt = time.perf_counter() - t0
        if any(t.is_alive() for t in th):
            print(json.dumps({"slabs": P, "errors": ["slab thread still running"]}), flush=True)
            os._exit(1)  # a blocked thread may still touch the comms: do not close them
        for c in comms:
            c.close()
        if errs:
            print(json.dumps({"slabs": P, "errors": errs}), flush=True)
            sys.exit(1)
        got = np.concatenate(out, axis=0)
        F = sh_oracle.residual(got.reshape(-1), U0.reshape(-1), N, N, h, r, k, g)
        res = {"slabs": P, "rows_per_slab": [int(o.shape[0]) for o in out],
               "nit": [s["nit"] for s in stats], "njvp": [s["njvp"] for s in stats],
               "fused_launches": [pr.get("arnoldi_fused", {}).get("launches", 0) for pr in profs],
               "max_abs_diff_vs_single": float(np.abs(got - ref).max()),
               "residual_maxnorm": float(np.abs(F).max()), "wall_s_one_gpu": round(dt, 2)}
        print(json.dumps(res), flush=True)
        ok = (len(set(res["nit"])) == 1 and abs(res["nit"][0] - ref_st["nit"]) <= 1
              and res["residual_maxnorm"] <= 6.06e-6 * 1.01 and min(res["fused_launches"]) > 0)
        if not ok:
            sys.exit(1)


if __name__ == "__main__":
    main()

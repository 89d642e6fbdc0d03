#!/usr/bin/env python3
"""Headline benchmark: implicit Swift-Hohenberg Newton-Krylov time steps on a 4096^2 grid.

Metric (BASELINE.json): "Newton-steps/sec + JVP SpMV HBM GB/s (% peak), 4096^2 grid, 1/2/4/8 GPU".
A *step* is one implicit Crank-Nicolson time step = one full ``newton_krylov`` solve, exactly the
loop body of the reference (sh_scipy_nk.py:56-61), on the config-4 workload: N = 4096,
h = 0.625 (d = 0.625 N, SURVEY.md section 7 hard part 2), k = 0.2, r = 0.01, g = 1,
U0 = default_rng(2020).standard_normal(N^2), scipy-default tolerances, FD (scipy-faithful) JVP.

    python bench.py [--gpus N --steps K --warmup W]       (N > 1: starts N rank processes itself)
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

N > 1: the same 4096^2 grid is cut into N row slabs (strong scaling); halo exchange and
all-reduce through the peer-memory communicator over xGMI (default) or RCCL (--comm rccl).
value = time steps per second of the whole job (max over ranks of the timed region).
Rank 0 prints ONE JSON line.  The kernel roofline comes from HIP events recorded around every
kernel on the solver's stream inside the timed region (nk_sh_kernel_profile); roofline.traffic
from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over a short child run of this bench on
the same box after the timed region (N=1; --pmc off: the last committed profile's ratios).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "iterative-solvers-summer-2020_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "Newton-steps/sec + JVP SpMV HBM GB/s (% peak), 4096^2 grid, 1/2/4/8 GPU"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=4096, help="grid points per side")
    ap.add_argument("--jvp", choices=["fd", "analytic"], default="fd")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--comm", choices=["peer", "rccl"], default="peer",
                    help="slab communicator for N > 1: peer-memory kernels over xGMI (default) "
                         "or RCCL send/recv + all-reduce")
    ap.add_argument("--rccl-self", action="store_true",
                    help="testing: build the RCCL communicator even at world size 1")
    ap.add_argument("--peer-self", action="store_true",
                    help="testing: build the peer-memory communicator even at world size 1")
    ap.add_argument("--extra", choices=["on", "off"], default="on",
                    help="also measure configs 2 (1024^2 Lap SpMV) and 3 (91x61 droplet)")
    ap.add_argument("--pmc", choices=["auto", "off"], default="auto",
                    help="HBM traffic of this box: two rocprofv3 --pmc passes (FETCH_SIZE, "
                         "WRITE_SIZE) over a short child run of this bench, N=1 only")
    ap.add_argument("--probes", choices=["on", "off"], default="on",
                    help="the isolated-JVP and copy-bandwidth probes after the timed region")
    ap.add_argument("--slab-ab", type=int, default=2,
                    help="N > 1: time steps of each slab-exchange variant after the warmup; the "
                         "fastest is the one the timed region runs (slab_exchange_ab; 0: off)")
    return ap.parse_args()


def pmc_traffic(args):
    """roofline.traffic measured on THIS box in THIS run: the bench itself, 1 warmup + 1 timed
    step at the same grid, run twice as a child process under rocprofv3 -- one --pmc FETCH_SIZE
    pass and one --pmc WRITE_SIZE pass (separate passes, MI355X_MICROARCH.md: read bytes =
    2 x FETCH_SIZE KiB, write bytes = WRITE_SIZE KiB on gfx950) -- each with the solver's launch
    log, matched dispatch by dispatch (scripts/traffic_match.py).  None when rocprofv3 is absent
    or a pass fails (the line then falls back to profiles/latest_traffic.json)."""
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None
    d = tempfile.mkdtemp(prefix="nkhip_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    child = [sys.executable, os.path.abspath(__file__), "--steps", "1", "--warmup", "1",
             "--n", str(args.n), "--jvp", args.jvp, "--extra", "off", "--cpu-baseline", "off",
             "--pmc", "off", "--probes", "off"]
    t0 = time.perf_counter()
    try:
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            env = dict(os.environ, NKHIP_LAUNCH_LOG=os.path.join(d, c + ".launches"),
                       TMPDIR=os.environ.get("TMPDIR", "/tmp"))
            r = subprocess.run([prof, "--pmc", c, "-d", os.path.join(d, c), "-o", c,
                                "--output-format", "csv", "--"] + child, env=env,
                               stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=150)
            if r.returncode != 0:
                return None
        logs = [open(os.path.join(d, c + ".launches")).read() for c in ("FETCH_SIZE", "WRITE_SIZE")]
        if logs[0] != logs[1]:  # the two passes must be the same deterministic program
            return None
        sys.path.insert(0, os.path.join(ROOT, "scripts"))
        import traffic_match as tm
        res = tm.match(tm.find(os.path.join(d, "FETCH_SIZE"), "counter_collection.csv"),
                       tm.find(os.path.join(d, "WRITE_SIZE"), "counter_collection.csv"), None,
                       os.path.join(d, "FETCH_SIZE.launches"), "bench")
        res["source"] = ("this run, this box: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE "
                         "passes over a child run of this bench (1 warmup + 1 step, same grid), "
                         "matched dispatch by dispatch to the solver's launch log; HBM bytes = "
                         "2 x FETCH_SIZE KiB + WRITE_SIZE KiB (gfx950)")
        res["seconds"] = round(time.perf_counter() - t0, 1)
        return res
    except (OSError, ValueError, subprocess.SubprocessError):
        return None
    finally:
        shutil.rmtree(d, ignore_errors=True)


def trace_durations(args):
    """Kernel-only durations on THIS box: `rocprofv3 --kernel-trace --stats` over a child run of
    this bench (1 warmup + 1 step, same grid).  An event pair around a launch that starts on an
    idle queue (the first JVP of every LGMRES call follows the host's line-search round trip)
    also times the dispatch of the launch; the trace does not.  {kernel name: (calls, avg_us)},
    or None without rocprofv3 or when the pass fails."""
    import csv
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None
    d = tempfile.mkdtemp(prefix="nkhip_kt_", dir=os.environ.get("TMPDIR", "/tmp"))
    child = [sys.executable, os.path.abspath(__file__), "--steps", "1", "--warmup", "1",
             "--n", str(args.n), "--jvp", args.jvp, "--extra", "off", "--cpu-baseline", "off",
             "--pmc", "off", "--probes", "off"]
    try:
        r = subprocess.run([prof, "--kernel-trace", "--stats", "-d", d, "-o", "kt",
                            "--output-format", "csv", "--"] + child,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=150,
                           env=dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp")))
        if r.returncode != 0:
            return None
        for root, _, files in os.walk(d):
            for f in files:
                if f.endswith("kernel_stats.csv"):
                    return {row["Name"]: (int(row["Calls"]), float(row["AverageNs"]) / 1e3)
                            for row in csv.DictReader(open(os.path.join(root, f)))}
        return None
    except (OSError, ValueError, KeyError, subprocess.SubprocessError):
        return None
    finally:
        shutil.rmtree(d, ignore_errors=True)


# the trace name of a kernel class the solver's launch log names (stencil modes: nk::SMode)
TRACE_NAMES = {"sh_fdjvp": "march_kernel<(nk::SMode)5,", "sh_ajvp": "march_kernel<(nk::SMode)6,"}


def cpu_baseline(n, h, k, r, g, u_start, gpu_fevals_per_step):
    """The reference's CPU path (scipy CSR L + scipy.optimize.newton_krylov on the reference
    residual, oracle/sh_oracle.py) timed on ONE full implicit step at the full grid size, from
    the same state the GPU's first timed step started from (so the same step of the trajectory).
    The first Newton iteration's time, extrapolated with the GPU run's F evals per step, is
    reported beside it (round-1 method).  Returns (record, the CPU's next state)."""
    import numpy as np
    from scipy.optimize import newton_krylov

    from oracle import sh_oracle

    L = sh_oracle.csr_L(n, h, r)
    cnt = [0]
    f = sh_oracle.make_csr_residual(L, u_start, k, g, cnt)
    marks = []
    t0 = time.perf_counter()
    u_next = newton_krylov(f, u_start, callback=lambda x, fx: marks.append(
        (time.perf_counter() - t0, cnt[0])))
    dt = time.perf_counter() - t0
    t1, f1 = marks[0] if marks else (dt, cnt[0])
    try:
        import threadpoolctl
        blas_threads = max(i.get("num_threads", 1) for i in threadpoolctl.threadpool_info()) or 1
    except Exception:
        blas_threads = os.cpu_count() or 1
    rec = {
        "value": 1.0 / dt,
        "unit": "steps/s",
        "cores": int(blas_threads),
        "kind": "port",
        "sample": (f"ONE full implicit step at {n}^2 timed (scipy CSR L, {L.nnz} nnz, + "
                   f"scipy.optimize.newton_krylov on the reference residual): {dt:.1f} s, "
                   f"{len(marks)} Newton its, {cnt[0]} F evals, from the state the GPU's first "
                   f"timed step started from. csr_matvec and NumPy element-wise are "
                   f"single-threaded; OpenBLAS BLAS-1 uses {blas_threads} threads; "
                   f"os.cpu_count()={os.cpu_count()}"),
        "step_s": round(dt, 2),
        "newton_its": len(marks),
        "fevals": cnt[0],
        "first_iteration_extrapolated": {
            "value": 1.0 / (t1 / max(f1, 1) * gpu_fevals_per_step),
            "first_iteration_s": round(t1, 2), "first_iteration_fevals": f1,
            "method": "s per F eval of the first Newton iteration x the GPU run's F evals per "
                      "step (round-1 estimate)"},
    }
    return rec, u_next


def config2_lap5(n=1024, reps=200, rocprof=True):
    """Config 2: 1024^2 fp64 periodic 5-point Laplacian SpMV (sh_scipy_nk.py:32-35), 16 B/pt,
    timed with HIP events on torch's stream; the reference's CSR `Lap @ v` timed beside it."""
    import numpy as np
    import torch

    import nkhip
    from oracle import sh_oracle
    h = 0.625
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
    # the kernel alone: an event pair around each launch (no inter-launch gap in the average)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for e0, e1 in ev:
        e0.record()
        nkhip.lap5_apply(v, 1 / h ** 2, out=y)
        e1.record()
    torch.cuda.synchronize()
    ev_us = sum(e0.elapsed_time(e1) for e0, e1 in ev) * 1e3 / reps
    # the kernel-only duration from a rocprofv3 trace of the same launches (an event pair around
    # a ~5 us kernel measures mostly the events), else the event pairs
    rp = config2_rocprof() if rocprof else None
    k_us = rp["avg_us"] if rp else ev_us
    k_gbs = 16 * n * n / (k_us * 1e-6) / 1e9
    err = float(np.abs(y.cpu().numpy().reshape(-1) - sh_oracle.lap5(v_np, n, n, 1 / h ** 2)).max())
    L = sh_oracle.csr_lap(n, h)
    best = 1e9
    for _ in range(20):
        t0 = time.perf_counter()
        L @ v_np
        best = min(best, time.perf_counter() - t0)
    return {"workload": f"lap5_{n}x{n}_fp64", "avg_us_per_launch_incl_gap": round(us, 2),
            "alg_GBps": round(16 * n * n / (us * 1e-6) / 1e9, 1), "max_abs_err_vs_oracle": err,
            "cpu_scipy_csr_ms": round(best * 1e3, 3),
            "roofline": {"kernel": "tile_kernel<LAP5>", "bound": "hbm",
                         "achieved": round(k_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(k_gbs / HBM_PEAK_GBS, 4), "avg_us": round(k_us, 2),
                         "alg_bytes_per_launch": 16 * n * n,
                         "launches": rp["calls"] if rp else reps,
                         "duration_source": ("rocprofv3 --kernel-trace --stats over "
                                             "scripts/config2_kernel.py on this box" if rp else
                                             "HIP event pair around each launch"),
                         "event_pair_us": round(ev_us, 2),
                         "mall_resident": True,
                         "note": "the 16.8 MB working set (v, y) stays on chip between "
                                 "launches (each XCD's 2 MB slice in its 4 MB L2, the rest in "
                                 "the 256 MB Infinity Cache), so HBM is not what bounds it"},
            "note": "back-to-back launches; rocprofv3 durations in profiles/r02_config2.md"}


def config2_rocprof():
    """Config 2's kernel duration without launch gaps or event overhead: `rocprofv3
    --kernel-trace --stats` over scripts/config2_kernel.py (205 back-to-back launches of the
    1024^2 Laplacian, ~10 s), the average duration of march_kernel<LAP5>.  None without
    rocprofv3 or when the pass fails."""
    import csv
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None
    d = tempfile.mkdtemp(prefix="nkhip_c2_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        r = subprocess.run([prof, "--kernel-trace", "--stats", "-d", d, "-o", "c2",
                            "--output-format", "csv", "--", sys.executable,
                            os.path.join(ROOT, "scripts", "config2_kernel.py")],
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=150,
                           env=dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp")))
        if r.returncode != 0:
            return None
        for root, _, files in os.walk(d):
            for f in files:
                if f.endswith("kernel_stats.csv"):
                    for row in csv.DictReader(open(os.path.join(root, f))):
                        if "tile_kernel" in row["Name"] or "march_kernel" in row["Name"]:
                            return {"avg_us": float(row["AverageNs"]) / 1e3,
                                    "calls": int(row["Calls"])}
        return None
    except (OSError, ValueError, KeyError, subprocess.SubprocessError):
        return None
    finally:
        shutil.rmtree(d, ignore_errors=True)


def config3_droplet(steps=5, cpu_steps=2):
    """Config 3: 91x61 droplet time-march (droplet.py evolve_with_PDE, 400 PMA loops per step)
    from the reference's coal init state; the restated reference path (scipy) timed beside it."""
    import numpy as np
    import torch

    import nkhip
    from oracle import droplet_oracle
    with np.load(os.path.join(ROOT, "tests", "golden", "droplet_init.npz")) as z:
        U0, Q0 = z["U0"], z["Q0"]
    d = nkhip.Droplet()
    d.set_state(U0, Q0)
    d.step()  # warm-up (compiles nothing, but pages in the kernels)
    d.set_state(U0, Q0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nits = 0
    for _ in range(steps):
        d.step(1e-4, 3e-9, 400)
        nits += d.last_stats["nit"]
    torch.cuda.synchronize()
    gpu = time.perf_counter() - t0
    d.close()
    t0 = time.perf_counter()
    droplet_oracle.evolve(U0, Q0, cpu_steps)
    cpu = time.perf_counter() - t0
    return {"workload": "droplet_91x61_coal_evolve_with_PDE", "steps": steps,
            "gpu_steps_per_s": round(steps / gpu, 2), "newton_its_per_step": nits / steps,
            "cpu_reference_path_steps_per_s": round(cpu_steps / cpu, 3), "cpu_steps": cpu_steps,
            "pma_loops_per_step": 400}


def config_pma2(steps=20, cpu_steps=2):
    """the PMA2 MEMS moving-mesh stepper (PMA2_nk.py main() loop, 51^2, one PMA
    mesh step + one Newton-Krylov solve per time step), GPU vs the restated reference path."""
    import torch

    import nkhip
    from oracle import pma2_oracle
    m = nkhip.Mems()
    m.step()  # warm-up
    m.set_state(*m.initial_state())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nit = 0
    for _ in range(steps):
        m.step()
        nit += m.last_stats["nit"]
    torch.cuda.synchronize()
    gpu = time.perf_counter() - t0
    m.close()
    u, q = pma2_oracle.initial_state()
    t0 = time.perf_counter()
    for _ in range(cpu_steps):
        u, q, _ = pma2_oracle.step(u, q)
    cpu = time.perf_counter() - t0
    return {"workload": "pma2_mems_51x51_step", "steps": steps,
            "gpu_steps_per_s": round(steps / gpu, 2), "newton_its_per_step": nit / steps,
            "cpu_reference_path_steps_per_s": round(cpu_steps / cpu, 3), "cpu_steps": cpu_steps}


def config_shlin(sizes=((64, 30, 30), (512, 20, 2))):
    """sh_linearised.py's semi-implicit step (r = 0.2, g = 0, k = 0.2,
    h = 0.625): GPU matrix-free CG vs the reference's scipy spsolve on the assembled matrix."""
    import numpy as np
    import torch

    import nkhip
    from oracle import shlin_oracle
    from oracle.sh_oracle import csr_L
    out = {}
    for n, steps, cpu_steps in sizes:
        U0 = np.random.default_rng(2020).standard_normal(n * n)
        s = nkhip.SHLinearised(N=n, d=0.625 * n, k=0.2, r=0.2, g=0.0)
        U = torch.as_tensor(U0, device="cuda")
        s.step(U, U)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        Uo, its = U, 0
        for _ in range(steps):
            U, Uo = s.step(U, Uo), U
            its += s.last_iters
        torch.cuda.synchronize()
        gpu = time.perf_counter() - t0
        s.close()
        L = csr_L(n, 0.625, 0.2).tocsc()
        t0 = time.perf_counter()
        u, uo = U0.copy(), U0.copy()
        for _ in range(cpu_steps):
            u, uo = shlin_oracle.step(L, u, uo, 0.2, 0.0), u
        cpu = time.perf_counter() - t0
        out[f"{n}x{n}"] = {"gpu_steps_per_s": round(steps / gpu, 2),
                           "cg_iters_per_step": its / steps,
                           "cpu_spsolve_steps_per_s": round(cpu_steps / cpu, 3)}
    return {"workload": "sh_linearised_semi_implicit_step", **out}


def config5_one_gpu(n=16384, warmup=1, steps=1):
    """Config 5's grid (16384^2, d = 0.625 N, the same parameters and seed) on ONE GPU: the
    single-GPU point of the 1/2/4/8 strong-scaling series the driver's 8-GPU job measures (the
    workspace pool is 58 vectors of 2.1 GB = 125 GB of HBM).  steps/s and ms per Arnoldi step."""
    import numpy as np
    import torch

    import nkhip
    U0 = np.random.default_rng(2020).standard_normal((n, n))
    U = torch.as_tensor(U0, device="cuda")
    del U0
    m = nkhip.SwiftHohenberg(N=n, d=0.625 * n, k=0.2, r=0.01, g=1.0)
    out = torch.empty_like(U)
    for _ in range(warmup):
        m.step(U, out=out)
        U, out = out, U
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    narn = nit = 0
    for _ in range(steps):
        m.step(U, out=out)
        narn += m.last_stats["n_arnoldi"]
        nit += m.last_stats["nit"]
        U, out = out, U
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    m.close()
    del U, out
    torch.cuda.empty_cache()
    return {"workload": f"swift_hohenberg_cn_newton_krylov_{n}x{n}_1gpu", "steps": steps,
            "warmup": warmup, "gpu_steps_per_s": round(steps / dt, 4),
            "ms_per_arnoldi_step": round(1e3 * dt / max(narn, 1), 3),
            "newton_its_per_step": nit / steps, "arnoldi_steps_per_step": narn / steps}


def config4_trajectory(n=4096, steps=100):
    """Config 4 over its stated length (BASELINE.json: "100 implicit time steps"): the
    reference's time loop (sh_scipy_nk.py:53-61) from U0 = default_rng(2020).standard_normal(N^2)
    at N = n (d = 0.625 N, k = 0.2, r = 0.01, g = 1, scipy-default tolerances, FD JVP), all `steps`
    steps timed from the first (no warmup step skipped: the headline's window starts later on the
    same trajectory), on a stepper of its own.  steps/s over the whole trajectory, Newton /
    Arnoldi counts, and the last step's oracle residual (sh_scipy_nk.py:47-49) on the host."""
    import numpy as np
    import torch

    import nkhip
    from oracle import sh_oracle
    h, k, r, g = 0.625, 0.2, 0.01, 1.0
    a = torch.as_tensor(np.random.default_rng(2020).standard_normal((n, n)), device="cuda")
    b = torch.empty_like(a)
    m = nkhip.SwiftHohenberg(N=n, d=h * n, k=k, r=r, g=g)
    tot = {"nit": 0, "njvp": 0, "nfev": 0}
    nit_first = nit_last = None
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(steps):
        m.step(a, out=b)
        st = m.last_stats
        for key in tot:
            tot[key] += st[key]
        nit_first = st["nit"] if s == 0 else nit_first
        nit_last = st["nit"]
        a, b = b, a
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    m.close()
    u1, u0 = a.cpu().numpy().reshape(-1), b.cpu().numpy().reshape(-1)
    del a, b
    torch.cuda.empty_cache()
    F = sh_oracle.residual(u1, u0, n, n, h, r, k, g)
    return {"workload": f"swift_hohenberg_cn_newton_krylov_{n}x{n}_{steps}_steps",
            "steps": steps, "gpu_steps_per_s": round(steps / dt, 4), "seconds": round(dt, 3),
            "newton_its_per_step": tot["nit"] / steps,
            "newton_its_first_last": [nit_first, nit_last],
            "arnoldi_steps_per_step": tot["njvp"] / steps,
            "ms_per_arnoldi_step": round(1e3 * dt / max(tot["njvp"], 1), 4),
            "final_step_residual": float(np.abs(F).max()),
            "f_tol": float(np.finfo(float).eps ** (1 / 3)), "state_max_abs": float(np.abs(u1).max()),
            "what": "steps 1..%d of the reference's time loop from U0, every step timed; "
                    "final_step_residual = oracle residual of the last step on the host" % steps}


def config_droplet_init():
    """initialise_coalescing_droplets(1000, [[0,0,1,1],[3,0,1,1]], 5e-9, 20) on
    the GPU (20 000 PMA loops); checked against the reference's initdrop_coal_* file."""
    import numpy as np
    import torch

    import nkhip
    with np.load(os.path.join(ROOT, "tests", "golden", "droplet_init.npz")) as z:
        U0 = z["U0"]
    d = nkhip.Droplet()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    U, _ = d.initialise_coalescing()
    torch.cuda.synchronize()
    gpu = time.perf_counter() - t0
    d.close()
    err = float(np.abs(U.cpu().numpy() - U0).max() / np.abs(U0).max())
    return {"workload": "droplet_initialise_coalescing_1000x20", "gpu_s": round(gpu, 3),
            "rel_err_vs_reference_init_file": err,
            "cpu_reference_path_s": "64.3 (NumPy restatement, one core, measured in the build "
                                    "container; tests/test_oracle_droplet.py)"}


def jvp_isolated(n, h, r, k, g, x0, jvp, reps=20):
    """The JVP stencil the metric names, alone: `reps` back-to-back launches on resident n^2
    inputs (after the timed region), HIP events on the launch stream.  FD: reads x0, z, G0 and
    writes w (32 B/pt); analytic: reads u, z, writes Jz (24 B/pt)."""
    import torch

    import nkhip
    gen = torch.Generator(device="cuda").manual_seed(11)
    z = torch.randn(n, n, dtype=torch.float64, device="cuda", generator=gen)
    g0 = torch.randn(n, n, dtype=torch.float64, device="cuda", generator=gen)
    w = torch.empty_like(z)
    x = x0.reshape(n, n)
    if jvp == "fd":
        fn, bpp, name = (lambda: nkhip.sh_fdjvp(x, g0, z, h, r, k, g, 1.0, 1e-7, out=w)), 32, "sh_fdjvp"
    else:
        fn, bpp, name = (lambda: nkhip.sh_jvp(x, z, h, r, k, g, out=w)), 24, "sh_ajvp"
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / reps
    gbs = bpp * n * n / (us * 1e-6) / 1e9
    return {"kernel": name, "bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4), "avg_us": round(us, 2),
            "alg_bytes_per_launch": bpp * n * n, "launches": reps,
            "source": f"{reps} back-to-back launches on resident {n}^2 inputs after the timed region"}


def copy_bandwidth(n, reps=20, scale=4):
    """This box's streaming rate, measured after the timed region so roofline fractions can be
    compared across boxes (their HBM spread is ~15 %): fp64 device-to-device copies of scale x n^2
    elements (read one vector, write one: 16 B/pt) by nk_stream_copy (16-KB chunks per block,
    non-temporal; the guide's float4-copy pattern, ~6.3 TB/s) and, for reference, torch's copy_;
    alternating between two buffer pairs so the working set (2.1 GB at 4096^2) exceeds the 256 MB
    Infinity Cache; HIP events on the current stream around back-to-back launches.  Copies of
    4 x 4096^2 (~175 us each) keep the launch gaps to ~1 % of the time (round 5,
    scripts/micro/copy_bench.hip: 1 x 4096^2 copies, ~44 us, lose ~3 % to them).
    peak_measured = the faster of the two."""
    import torch

    import nkhip
    n2 = n * n * scale
    bufs = [torch.empty(n2, dtype=torch.float64, device="cuda") for _ in range(4)]
    for b_ in bufs:
        b_.normal_()

    def rate(fn):
        for i in range(4):
            fn(bufs[2 * (i % 2)], bufs[2 * (i % 2) + 1])
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        for i in range(reps):
            fn(bufs[2 * (i % 2)], bufs[2 * (i % 2) + 1])
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) * 1e3 / reps
        return round(16.0 * n2 / (us * 1e-6) / 1e9, 1), round(us, 2)

    lib_gbs, lib_us = rate(lambda s_, d_: nkhip.stream_copy(s_, out=d_))
    torch_gbs, _ = rate(lambda s_, d_: d_.copy_(s_))
    del bufs
    return {"GB/s": max(lib_gbs, torch_gbs), "nk_stream_copy_GB/s": lib_gbs,
            "nk_stream_copy_avg_us": lib_us, "torch_copy_GB/s": torch_gbs,
            "what": f"{scale} x {n}^2 fp64 copies (16 B/pt), {reps} reps over two buffer pairs, "
                    "HIP events around the back-to-back launches, after the timed region"}


_PUSH_FALLBACK = {"set": False}  # peer_or_rccl set NKHIP_SLAB_PUSH=0 itself


def effective_slab_path(slots, one_device):
    """The slab path the solver takes on a peer-memory group under the current environment (the
    switches the library reads per call): in_kernel (NKHIP_SLAB_XK, sh_problem.cpp push_mode),
    edge_halo (no halo slots, or NKHIP_SLAB_PUSH=0), pushed_tail (NKHIP_ARN_TAIL, one rank per
    GPU only, lgmres.cpp), else pushed."""
    xk = os.environ.get("NKHIP_SLAB_XK", "")
    if xk[:1] == "1" or (xk[:1] == "2" and not one_device):
        return "in_kernel"
    if not slots or os.environ.get("NKHIP_SLAB_PUSH", "1")[:1] == "0":
        return "edge_halo"
    if os.environ.get("NKHIP_ARN_TAIL", "")[:1] in ("1", "2") and not one_device:
        return "pushed_tail"
    return "pushed"


def peer_or_rccl(nkhip, dist, torch, max_nx, coll_dev="cpu", allow_rccl=True):
    """The peer-memory communicator, verified before it is used, at the full row width, with
    bounded device waits.  Two collectives, each agreed on over the gloo side channel:
      1. nk_comm_selftest -- one all-reduce and one halo exchange of known values.  If any rank
         cannot create, map or verify the group, every rank falls back to RCCL (stderr says so)
         -- or fails, when the ranks share a device (RCCL takes one rank per GPU);
      2. nk_comm_selftest_push -- the pushed-halo-rows protocol the slab solver uses by default
         (push into the neighbours' halo slots, system-scope fence, no flag, one all-reduce, read
         back, host check).  If it fails on any rank, every rank runs the edge + halo exchange
         path instead (NKHIP_SLAB_PUSH=0), which step 1 verified.
    Returns (comm, check): check records both outcomes and the slab path taken."""
    def agree(v):
        t = torch.tensor([int(v)], dtype=torch.int32, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return int(t.item())

    comm, ok = None, 1
    try:
        comm = nkhip.PeerComm.from_torch_distributed(max_nx=max_nx)
        ok = int(comm.selftest(max_nx))
    except Exception as e:  # noqa: BLE001 - any failure means: use RCCL instead
        print(f"peer-memory communicator unavailable: {e}", file=sys.stderr)
        ok = 0
    if agree(ok) == 1:
        push = comm.selftest_push(max_nx)  # True / False / None (no slots: nothing to check)
        push_ok = agree(push is not False)
        check = {"selftest": "ok"}
        if push is None:
            check["pushed_rows_selftest"] = "n/a (no halo slots)"
        elif push_ok == 1:
            check["pushed_rows_selftest"] = "ok"
            # a fallback an earlier group of this run set is not this group's (config 5 builds a
            # second group): only the switch this function set itself is taken back
            if _PUSH_FALLBACK["set"]:
                os.environ.pop("NKHIP_SLAB_PUSH", None)
                _PUSH_FALLBACK["set"] = False
        else:
            print("pushed-halo-rows self-test failed on some rank: every rank takes the edge + "
                  "halo exchange path (NKHIP_SLAB_PUSH=0)", file=sys.stderr)
            os.environ["NKHIP_SLAB_PUSH"] = "0"
            _PUSH_FALLBACK["set"] = True
            check["pushed_rows_selftest"] = "failed on some rank"
        # the path the solver takes: from the effective switches, not from the test alone
        check["slab_path"] = effective_slab_path(push is not None, not allow_rccl)
        return comm, check
    print("peer-memory communicator failed its self-test on some rank"
          + (": using RCCL" if allow_rccl else ""), file=sys.stderr)
    if comm is not None:
        comm.abort()
        comm.close()
    if not allow_rccl:
        raise RuntimeError("peer-memory communicator failed and the ranks share a device")
    return nkhip.RcclComm.from_torch_distributed(), {"selftest": "failed on some rank: RCCL",
                                                     "slab_path": "edge_halo"}


def slab_residual_max(nkhip, dist, torch, u1, u0, n, rank, world, h, r, k, g):
    """The oracle residual (sh_scipy_nk.py:47-49) of a row-slab state, max over the whole grid,
    without gathering it: each rank pads its slab of U[s+1] and U[s] with the ring neighbours'
    two edge rows (gloo all_gather of 4 rows per rank), evaluates the oracle's periodic stencil
    on the padded block -- exact on its interior rows -- on the host, and the max goes over the
    ranks (every rank gets it)."""
    import numpy as np

    from oracle import sh_oracle
    ny = u1.shape[0]
    out = []
    for x in (u1, u0):
        x = x.cpu()
        edge = torch.cat([x[:2], x[-2:]]).to(torch.float64)
        parts = [torch.empty_like(edge) for _ in range(world)]
        dist.all_gather(parts, edge)
        prev, nxt = parts[(rank - 1) % world], parts[(rank + 1) % world]
        out.append(torch.cat([prev[2:], x, nxt[:2]]).numpy())
    F = sh_oracle.residual(out[0].reshape(-1), out[1].reshape(-1), ny + 4, n, h, r, k, g)
    worst = torch.tensor([float(np.abs(F.reshape(ny + 4, n)[2:-2]).max())], dtype=torch.float64)
    del F, out
    dist.all_reduce(worst, op=dist.ReduceOp.MAX)
    return float(worst.item())


def slab_of_seeded_grid(seed, n, row0, ny, chunk=256):
    """Rows [row0, row0 + ny) of default_rng(seed).standard_normal((n, n)) without materialising
    the rows before them: the generator's draws are sequential, so drawing and discarding the
    leading rows in chunks of `chunk` rows gives the same numbers in bounded host memory."""
    import numpy as np
    rng = np.random.default_rng(seed)
    for r0 in range(0, row0, chunk):
        rng.standard_normal((min(chunk, row0 - r0), n))
    return rng.standard_normal((ny, n))


def config5_slabs(nkhip, dist, torch, comm, check, n5, rank, world, one_device, steps=1,
                  warmup=1):
    """Config 5 on the N ranks of this job: the 16384^2 grid (d = 0.625 N, k, r, g and seed as the
    headline) cut into the same row slabs over the same kind of communicator (a peer-memory group
    of the full 16384-column width, verified as the headline's), ``warmup`` untimed + ``steps``
    timed time steps, max over ranks; the whole grid's oracle residual of the last step
    (slab_residual_max).  One point of the 1/2/4/8-GPU curve per driver run.  Returns (record,
    comm): the communicator the caller closes."""
    import numpy as np
    if comm is not None and type(comm).__name__ == "PeerComm":
        comm.close()  # the headline's group is 4096 columns wide
        dist.barrier()
        comm, check = peer_or_rccl(nkhip, dist, torch, n5, "cpu", allow_rccl=not one_device)
    h, k, r, g = 0.625, 0.2, 0.01, 1.0
    row0, ny = nkhip.slab_rows(n5, rank, world)
    U = slab_of_seeded_grid(2020, n5, row0, ny)
    a = torch.as_tensor(U, device="cuda")
    del U
    b = torch.empty_like(a)
    dist.barrier()
    m = nkhip.SwiftHohenberg(N=n5, d=h * n5, k=k, r=r, g=g, comm=comm, ny_local=ny)
    for _ in range(warmup):
        m.step(a, out=b)
        a, b = b, a
    tot = {"nit": 0, "njvp": 0}
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        m.step(a, out=b)
        for key in tot:
            tot[key] += m.last_stats[key]
        a, b = b, a
    torch.cuda.synchronize()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    dt = float(dt.item())
    res = slab_residual_max(nkhip, dist, torch, a, b, n5, rank, world, h, r, k, g)
    dist.barrier()
    m.close()
    del a, b
    torch.cuda.empty_cache()
    rec = {"workload": f"swift_hohenberg_cn_newton_krylov_{n5}x{n5}", "grid": n5,
           "n_gpus": world, "steps": steps, "warmup": warmup,
           "steps_per_s": round(steps / dt, 4),
           "ms_per_arnoldi_step": round(1e3 * dt / max(tot["njvp"], 1), 4),
           "newton_its_per_step": tot["nit"] / steps,
           "arnoldi_steps_per_step": tot["njvp"] / steps,
           "final_step_residual": res, "f_tol": float(np.finfo(float).eps ** (1 / 3)),
           "comm": type(comm).__name__, "comm_check": check,
           "what": "row slabs of the 16384^2 grid on this job's ranks after the headline; "
                   "final_step_residual = oracle residual of the last step over the whole grid "
                   "(padded slabs on the host, max over ranks)"}
    if one_device:
        rec["ranks_on_one_device"] = True
    return rec, comm


def load_traffic():
    path = os.path.join(ROOT, "profiles", "latest_traffic.json")
    try:
        with open(path) as fh:
            return json.load(fh)
    except (OSError, ValueError):
        return {}


def self_launch(n):
    """``--gpus N`` started without a launcher (no WORLD_SIZE in the environment): start N rank
    processes of this same command line, one per GPU (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR=127.0.0.1 / MASTER_PORT set as torch.distributed.run sets them), forward rank 0's
    JSON line as this process's only stdout line and return the exit code (non-zero when any rank
    failed; the survivors are killed 60 s after the first failure, their peer waits being bounded).
    Runs before this process imports anything that touches the GPU, and it execs nothing: the
    ranks are children.  NKHIP_BENCH_ONE_DEVICE=1 puts every rank on device 0 (testing on a
    one-GPU box: the ranks' side channel is then gloo, as RCCL takes one rank per device)."""
    import socket
    import subprocess
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    cmd = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        # rank 0's stdout carries the JSON line; the other ranks print nothing there
        procs.append(subprocess.Popen(cmd, env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr))
    out0 = []
    import threading
    reader = threading.Thread(target=lambda: out0.extend(procs[0].stdout.read().decode()
                                                         .splitlines()), daemon=True)
    reader.start()
    failed_at = None
    while any(p.poll() is None for p in procs):
        if failed_at is None and any(p.poll() not in (None, 0) for p in procs):
            failed_at = time.monotonic()
            print("bench: a rank failed; stopping the others in 60 s", file=sys.stderr)
        if failed_at is not None and time.monotonic() - failed_at > 60:
            for p in procs:
                if p.poll() is None:
                    p.kill()
        time.sleep(0.2)
    reader.join(30)
    rcs = [p.returncode for p in procs]
    lines = [ln for ln in out0 if ln.startswith("{")]
    for ln in out0:
        if not ln.startswith("{"):
            print(ln, file=sys.stderr)
    if any(rcs) or len(lines) != 1:
        print(f"bench: rank exit codes {rcs}, {len(lines)} JSON line(s) from rank 0",
              file=sys.stderr)
        return next((c for c in rcs if c), 1)
    print(lines[0], flush=True)
    return 0


def slab_exchange_ab(model, a, b, rounds, one_device, dist, coll_dev, torch, pushed_ok=True):
    """N > 1, after the timed region: the slab paths of the fused Arnoldi step, rotating one time
    step each (``rounds`` of each), as ms per Arnoldi step (max over ranks of each step's wall
    time / its Arnoldi steps).  pushed (the default): every producer writes its edge rows into the
    neighbours' halo slots, the fused pass forms u on its halo rows itself, nothing is exchanged
    in between; edge_halo (NKHIP_SLAB_PUSH=0): a 4-row edge kernel exchanges u on the slab's edge
    rows before the fused pass; in_kernel (NKHIP_SLAB_XK=2, =1 when the ranks share a GPU): the
    fused pass's edge bands exchange them themselves; pushed_tail (NKHIP_ARN_TAIL=1): pushed,
    with each step's reduction + all-reduce + control in the fused launch's last blocks (one rank
    per GPU only: with ranks sharing a GPU it is the pushed path; its waits bounded by 3 s,
    NKHIP_ARN_TAIL_TIMEOUT_S, so a stall fails the variant within seconds).  Returns (record, a,
    b), the trajectory advanced."""
    names = ("pushed", "edge_halo", "in_kernel", "pushed_tail")
    if not pushed_ok:  # the pushed-halo-rows self-test failed (or there are no slots)
        names = ("edge_halo", "in_kernel")
    env = {"pushed": {"NKHIP_SLAB_PUSH": "1", "NKHIP_SLAB_XK": "0", "NKHIP_ARN_TAIL": "0"},
           "edge_halo": {"NKHIP_SLAB_PUSH": "0", "NKHIP_SLAB_XK": "0", "NKHIP_ARN_TAIL": "0"},
           "in_kernel": {"NKHIP_SLAB_PUSH": "1", "NKHIP_SLAB_XK": "1" if one_device else "2",
                         "NKHIP_ARN_TAIL": "0"},
           "pushed_tail": {"NKHIP_SLAB_PUSH": "1", "NKHIP_SLAB_XK": "0", "NKHIP_ARN_TAIL": "1",
                           "NKHIP_ARN_TAIL_TIMEOUT_S": "3"}}
    keys = ("NKHIP_SLAB_PUSH", "NKHIP_SLAB_XK", "NKHIP_ARN_TAIL", "NKHIP_ARN_TAIL_TIMEOUT_S")
    old = {k_: os.environ.get(k_) for k_ in keys}
    acc = {n_: [0.0, 0] for n_ in names}
    failed = failed_name = None
    try:
        for i in range(len(names) * rounds):
            name = names[i % len(names)]
            for k_ in keys:
                os.environ.pop(k_, None)
            os.environ.update(env[name])
            dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            err = 0.0
            try:  # a variant that fails ends the comparison on every rank, not the bench line
                model.step(a, out=b)
                torch.cuda.synchronize()
            except Exception as e:  # noqa: BLE001 (nkhip.NKError and HIP errors alike)
                err, failed = 1.0, f"{name}: {e}"
            t = torch.tensor([time.perf_counter() - t0, err], dtype=torch.float64, device=coll_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            if float(t[1].item()) > 0:
                failed = failed or f"{name}: failed on another rank"
                failed_name = name
                break
            acc[name][0] += float(t[0].item())
            acc[name][1] += model.last_stats["njvp"]
            a, b = b, a
    finally:
        for k_, v in old.items():
            if v is None:
                os.environ.pop(k_, None)
            else:
                os.environ[k_] = v
    rec = {f"{k_}_ms_per_arnoldi": round(1e3 * v[0] / max(v[1], 1), 4) for k_, v in acc.items()}
    if not pushed_ok:
        rec["skipped"] = "pushed, pushed_tail (the pushed-halo-rows self-test did not pass)"
    if failed:
        rec["failed"] = failed
        rec["failed_variant"] = failed_name
    rec.update({"steps_each": rounds, "arnoldi_steps": {k_: v[1] for k_, v in acc.items()},
                "what": "rotating time steps after the timed region; max over ranks of each "
                        "step's wall time / its Arnoldi steps"})
    return rec, a, b


def select_slab_path(rec, one_device, dist, torch):
    """The fastest slab path of a slab_exchange_ab record (ms per Arnoldi step, max over ranks;
    variants that failed or ran no step are out), rank 0's choice on every rank; its switches are
    set in this process's environment for everything after (the library reads them per call).
    With ranks sharing one GPU the tail is not used (lgmres.cpp), so pushed_tail there is the
    pushed path."""
    names = ("pushed", "edge_halo", "in_kernel", "pushed_tail")
    ok = [n_ for n_ in names if rec.get("arnoldi_steps", {}).get(n_, 0) > 0
          and n_ != rec.get("failed_variant")]
    best = min(ok, key=lambda n_: rec[f"{n_}_ms_per_arnoldi"]) if ok else None
    t = torch.tensor([names.index(best) if best else -1], dtype=torch.int32)
    dist.broadcast(t, 0)
    best = names[int(t.item())] if int(t.item()) >= 0 else None
    env = {"pushed": {"NKHIP_SLAB_PUSH": "1", "NKHIP_SLAB_XK": "0", "NKHIP_ARN_TAIL": "0"},
           "edge_halo": {"NKHIP_SLAB_PUSH": "0", "NKHIP_SLAB_XK": "0", "NKHIP_ARN_TAIL": "0"},
           "in_kernel": {"NKHIP_SLAB_PUSH": "1", "NKHIP_SLAB_XK": "1" if one_device else "2",
                         "NKHIP_ARN_TAIL": "0"},
           "pushed_tail": {"NKHIP_SLAB_PUSH": "1", "NKHIP_SLAB_XK": "0", "NKHIP_ARN_TAIL": "1",
                           "NKHIP_ARN_TAIL_TIMEOUT_S": "3"}}
    if best is None:  # nothing ran: the default switches
        return effective_slab_path(True, one_device)
    os.environ.update(env[best])
    return effective_slab_path(True, one_device)


def main():
    rc = 0
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(self_launch(args.gpus))  # before anything touches the GPU
    import numpy as np
    import torch
    import torch.distributed as dist

    import nkhip

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
        sys.exit(2)
    # testing on one GPU: every rank on device 0 (peer communicator only)
    one_device = world > 1 and os.environ.get("NKHIP_BENCH_ONE_DEVICE") == "1"
    device = 0 if one_device else local
    torch.cuda.set_device(device)
    comm, comm_check = None, None
    use_dist = world > 1 or args.rccl_self or args.peer_self
    # torch.distributed is only the side channel (IPC handle / RCCL unique-id exchange, barriers,
    # the max over ranks of the timed region, the final gather): gloo on host tensors.  The
    # solver's collectives run in libnkhip (peer-memory kernels, or its own RCCL communicator),
    # and a torch NCCL group would only add its own RCCL communicator, buffers and threads.
    coll_dev = "cpu"
    if use_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1:  # --rccl-self / --peer-self without a launcher: a world of one
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
            os.environ.setdefault("MASTER_PORT", "29531")
        dist.init_process_group("gloo")
        if args.rccl_self or (world > 1 and args.comm == "rccl" and not args.peer_self):
            comm = nkhip.RcclComm.from_torch_distributed()
        else:
            comm, comm_check = peer_or_rccl(nkhip, dist, torch, args.n, coll_dev,
                                            allow_rccl=not one_device)

    n = args.n
    h, k, r, g = 0.625, 0.2, 0.01, 1.0
    row0, ny = nkhip.slab_rows(n, rank, world)
    U_full = np.random.default_rng(2020).standard_normal((n, n))
    U = torch.as_tensor(U_full[row0:row0 + ny].copy(), device="cuda")
    del U_full
    stream = torch.cuda.current_stream()
    # kernel timing: HIP events around every PROFILE-th launch of each kernel class inside the
    # timed region (an event pair costs ~5 us of GPU time; every launch timed costs ~7 %)
    profile = int(os.environ.get("NKHIP_BENCH_PROFILE", "8"))
    if use_dist:
        # the problem's first device collective runs inside its construction: no rank may reach
        # it seconds ahead of a peer still generating its state (the device waits are bounded)
        dist.barrier()
    model = nkhip.SwiftHohenberg(N=n, d=h * n, k=k, r=r, g=g, jvp=args.jvp, profile=profile,
                                 comm=comm, ny_local=ny, stream=stream)
    a, b = U, torch.empty_like(U)

    def barrier():
        if use_dist:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        model.step(a, out=b)
        a, b = b, a
    # N > 1: the slab path the timed region runs is the one that wins on THIS node -- the slab
    # A/B runs here, after the warmup, and every rank takes its fastest variant (the times are
    # maxima over ranks, so every rank computes the same winner; rank 0's is broadcast anyway).
    # The state is restored afterwards, so the timed window starts where it would without it.
    slab_ab, slab_path = None, ("edge_halo (RCCL)" if world > 1 else None)
    if world > 1 and comm_check is not None:
        slab_path = comm_check.get("slab_path")
        if args.slab_ab > 0:
            a_keep = a.clone()
            pushed_ok = comm_check.get("slab_path") == "pushed"
            slab_ab, a, b = slab_exchange_ab(model, a, b, args.slab_ab, one_device, dist,
                                             coll_dev, torch, pushed_ok=pushed_ok)
            slab_path = select_slab_path(slab_ab, one_device, dist, torch)
            a.copy_(a_keep)
            del a_keep
            if slab_ab.get("failed"):
                # a variant that failed may have left the group's error word set: a fresh group
                # and stepper for the timed region (the winner's switches are already in place)
                model.close()
                comm.abort()
                comm.close()
                dist.barrier()
                comm, comm_check = peer_or_rccl(nkhip, dist, torch, args.n, coll_dev,
                                                allow_rccl=not one_device)
                slab_path = comm_check.get("slab_path")
                dist.barrier()
                model = nkhip.SwiftHohenberg(N=n, d=h * n, k=k, r=r, g=g, jvp=args.jvp,
                                             profile=profile, comm=comm, ny_local=ny,
                                             stream=stream)
            slab_ab.update({"selected": slab_path,
                            "when": "after the warmup, before the timed region (the warmup's "
                                    "final state is restored for the timed steps)"})
    want_cpu = world == 1 and args.cpu_baseline == "auto"
    u_start = a.cpu().numpy().reshape(-1) if want_cpu else None  # outside the timed region
    model.reset_profile()
    tot = {"nit": 0, "nfev": 0, "njvp": 0, "n_arnoldi": 0}
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        model.step(a, out=b)
        for key in tot:
            tot[key] += model.last_stats[key]
        a, b = b, a
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    prof = model.kernel_profile()
    final_max = float(a.abs().max())
    # check the final step on the host (outside the timed region): a = U[s+1], b = U[s]; with
    # N > 1 the slabs are gathered to every rank and rank 0 evaluates the oracle residual
    # (sh_scipy_nk.py:47-49) of the whole grid.  Slabs differ in rows by at most one: gathered
    # padded to the largest slab, then trimmed.
    if world > 1:
        nys = [nkhip.slab_rows(n, q, world)[1] for q in range(world)]
        nymax = max(nys)

        def gather(x):
            xp = torch.zeros((nymax, n), dtype=x.dtype, device=coll_dev)
            xp[:ny] = x.to(coll_dev)
            parts = [torch.empty_like(xp) for _ in range(world)]
            dist.all_gather(parts, xp)
            if rank != 0:
                return None
            return torch.cat([p_[:nq] for p_, nq in zip(parts, nys)]).cpu().numpy()

        full_a, full_b = gather(a), gather(b)
    else:
        full_a, full_b = a.cpu().numpy(), b.cpu().numpy()
    # config 5 on this job's ranks (N > 1): the point of the 16384^2 curve; at N = 1 it runs
    # below, in other_configs.config5_1gpu
    c5 = None
    if world > 1 and args.extra == "on":
        model.close()
        model = None
        del a, b
        torch.cuda.empty_cache()
        c5, comm = config5_slabs(nkhip, dist, torch, comm, comm_check,
                                 int(os.environ.get("NKHIP_BENCH_CONFIG5_N", "16384")), rank,
                                 world, one_device)

    if rank == 0:
        steps_per_s = args.steps / elapsed
        # dominant kernel by time, and the JVP stencil the metric names
        ker = {k_: v for k_, v in prof.items() if v["timed"] > 0 and v["ms"] > 0}
        for v in ker.values():  # whole-class time extrapolated from the timed launches
            v["ms_est"] = v["ms"] * v["launches"] / v["timed"]
        # the dominant HBM-streaming class; the slab path's exchange / control launches are
        # latency-bound (their time is waiting for peers, not bytes) and are reported in
        # "kernels" beside it
        comm_classes = {"arnoldi_edge", "halo", "arnoldi_ctl", "reduce_final", "edge_gather"}
        cand = [k_ for k_ in ker if k_ not in comm_classes] or list(ker)
        dom = max(cand, key=lambda k_: ker[k_]["ms_est"]) if cand else None

        # PMC traffic of this run (two child passes under rocprofv3), else the last profile's
        live = pmc_traffic(args) if (world == 1 and args.pmc == "auto") else None
        traffic_db = live or load_traffic()
        trace = trace_durations(args) if (world == 1 and args.pmc == "auto") else None

        def roof(name):
            v = ker[name]
            gbs = v["timed_bytes"] / (v["ms"] * 1e-3) / 1e9
            alg = v["timed_bytes"] / v["timed"]
            t = traffic_db.get("classes", {}).get(name)
            traffic = None
            if t and "traffic_over_alg" in t:
                # PMC HBM bytes (FETCH_SIZE x2 + WRITE_SIZE, gfx950-corrected) per launch, measured
                # on the same kernel class by scripts/profile.sh; scaled to this run's launches by
                # the traffic/algorithmic ratio of the profiled run.
                traffic = round(t["traffic_over_alg"] * alg)
            return {"kernel": name, "bound": "hbm", "achieved": round(gbs, 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                    "traffic": traffic, "launches": v["launches"], "timed_launches": v["timed"],
                    "avg_us": round(1e3 * v["ms"] / v["timed"], 2),
                    "alg_bytes_per_launch": alg,
                    "traffic_source": (traffic_db.get("source") if live else
                                       f"N=1 profile ratios, tag {traffic_db.get('tag')} "
                                       f"(profiles/latest_traffic.json: "
                                       f"{traffic_db.get('source')}); not measured in this run")
                    if traffic else None}

        from oracle import sh_oracle
        F_last = sh_oracle.residual(full_a.reshape(-1), full_b.reshape(-1), n, n, h, r, k, g)
        final_check = {"max_abs_residual": float(np.abs(F_last).max()),
                       "f_tol": float(np.finfo(float).eps ** (1 / 3)),
                       "what": "oracle residual (sh_scipy_nk.py:47-49) of the last timed step, "
                               "evaluated on the host over the whole grid; above f_tol the "
                               "bench exits non-zero after printing its line"}
        del F_last
        jvp_name = "sh_fdjvp" if args.jvp == "fd" else "sh_ajvp"
        kernel_ms = sum(v["ms_est"] for v in ker.values())
        out = {
            "metric": METRIC,
            "value": round(steps_per_s, 4),
            "unit": "steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: U0 = numpy default_rng(2020).standard_normal(N^2)",
            "config": {"workload": f"swift_hohenberg_cn_newton_krylov_{n}x{n}", "grid": [n, n],
                       "h": h, "k": k, "r": r, "g": g, "jvp": args.jvp,
                       "f_tol": "scipy default eps^(1/3) (max-norm)", "inner_m": 30,
                       "outer_k": 10, "parallelism": f"row-slab x{world}",
                       "slab_path": slab_path,
                       "comm": (type(comm).__name__ if comm is not None else "none")},
            "comm_check": comm_check,
            "newton_its_per_s": round(tot["nit"] / elapsed, 3),
            "jvps_per_s": round(tot["njvp"] / elapsed, 2),
            "per_step": {k_: v / args.steps for k_, v in tot.items()},
            "ms_per_arnoldi_step": round(1e3 * elapsed / max(tot["njvp"], 1), 4),
            "roofline": roof(dom) if dom else None,
            "jvp_roofline": roof(jvp_name) if jvp_name in ker else None,
            "kernel_time_frac_of_wall": round(kernel_ms * 1e-3 / elapsed, 4) if ker else None,
            "kernels": {k_: {"launches": v["launches"], "timed": v["timed"],
                             "ms_est": round(v["ms_est"], 3),
                             "avg_us": round(1e3 * v["ms"] / v["timed"], 2),
                             "alg_MB_per_launch": round(v["timed_bytes"] / v["timed"] / 1e6, 3),
                             "GB/s": round(v["timed_bytes"] / (v["ms"] * 1e-3) / 1e9, 1)}
                        for k_, v in ker.items()},
            "kernel_timing": f"HIP events around every {profile}-th launch of each class",
            "state_max_abs": final_max,
            "final_step_check": final_check,
            "cpu_baseline": None,
        }
        jr = out["jvp_roofline"]
        hits = [cu for nm, cu in (trace or {}).items() if TRACE_NAMES.get(jvp_name, "\0") in nm]
        if jr and hits:
            # the JVP's kernel duration from the trace (its event pairs start on an idle queue)
            calls = sum(c for c, _ in hits)
            us = sum(c * u for c, u in hits) / calls
            gbs = jr["alg_bytes_per_launch"] / (us * 1e-6) / 1e9
            jr.update({"event_avg_us": jr["avg_us"], "event_frac": jr["frac"],
                       "avg_us": round(us, 2), "achieved": round(gbs, 1),
                       "frac": round(gbs / HBM_PEAK_GBS, 4), "trace_launches": calls,
                       "duration_source": "rocprofv3 --kernel-trace --stats over a child run of "
                                          "this bench (1 warmup + 1 step, same grid, this box); "
                                          "event_avg_us: HIP event pairs in the timed run"})
        if slab_ab is not None:
            out["slab_exchange_ab"] = slab_ab
        if one_device:
            out["config"]["ranks_on_one_device"] = True
        out["traffic_measurement"] = (
            {"live": True, "seconds": live.get("seconds"),
             "classes": {c: round(v["traffic_over_alg"], 4) for c, v in live["classes"].items()
                         if v.get("traffic_over_alg")}}
            if live else {"live": False, "file": "profiles/latest_traffic.json",
                          "tag": traffic_db.get("tag")})
        if args.probes == "on":
            if world == 1:
                out["jvp_roofline_isolated"] = jvp_isolated(n, h, r, k, g, a, args.jvp)
            # the box's measured streaming rate beside the 8 TB/s spec: frac_of_measured makes
            # the fractions comparable across boxes
            cb = copy_bandwidth(n)
            out["copy_bandwidth"] = cb
            for key in ("roofline", "jvp_roofline", "jvp_roofline_isolated"):
                rl = out.get(key)
                if rl:
                    rl["peak_measured"] = cb["GB/s"]
                    rl["frac_of_measured"] = round(rl["achieved"] / cb["GB/s"], 4)
        if want_cpu:
            fe = (tot["nfev"] + tot["njvp"]) / args.steps
            rec, u_cpu = cpu_baseline(n, h, k, r, g, u_start, fe)
            # the same step on the GPU (outside the timed region) against scipy's result
            ua = torch.as_tensor(u_start.reshape(n, n), device="cuda")
            ub = model.step(ua)
            rec["gpu_vs_scipy_same_step"] = {
                "max_abs_diff": float(np.abs(ub.cpu().numpy().reshape(-1) - u_cpu).max()),
                "state_max_abs": float(np.abs(u_cpu).max()),
                "gpu_newton_its": model.last_stats["nit"], "scipy_newton_its": rec["newton_its"],
                "bar": "1e-5 * max(1, |U|) (default f_tol)"}
            del ua, ub, u_cpu
            out["cpu_baseline"] = rec
        if c5 is not None:
            out["other_configs"] = {"config5": c5}
        if world == 1 and args.extra == "on":
            out["other_configs"] = {"config2": config2_lap5(rocprof=args.pmc == "auto"),
                                    "config4_100": config4_trajectory(n),
                                    "config3": config3_droplet(),
                                    "config5_1gpu": config5_one_gpu(),
                                    "pma2": config_pma2(), "sh_linearised": config_shlin(),
                                    "droplet_init": config_droplet_init()}
        print(json.dumps(out), flush=True)
        # a wrong answer fails the run (sh_scipy_nk.py:47-49: the step is a root to f_tol in the
        # max norm; the slack covers the oracle's own rounding, ~1e-14 at these magnitudes)
        c4 = out.get("other_configs", {}).get("config4_100") or {}
        for what, v, tol in (("headline", final_check["max_abs_residual"], final_check["f_tol"]),
                             ("config5", (c5 or {}).get("final_step_residual", 0.0),
                              final_check["f_tol"]),
                             ("config4_100", c4.get("final_step_residual", 0.0),
                              final_check["f_tol"])):
            if not v <= tol + 1e-12:
                print(f"bench: {what} final-step residual {v:.3e} exceeds f_tol {tol:.3e}",
                      file=sys.stderr)
                rc = 3
    if use_dist:
        dist.barrier()  # no rank frees its communicator buffers while a peer may still use them
    if model is not None:
        model.close()
    if comm is not None:
        comm.close()
    if use_dist:
        dist.destroy_process_group()
    return rc


if __name__ == "__main__":
    sys.exit(main())

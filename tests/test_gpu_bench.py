"""GPU: bench.py's N-GPU line produced by the driver's own command form, ``python bench.py
--gpus N`` without a launcher (bench.py self_launch: N rank processes, rank 0's JSON line
forwarded).  On the one-GPU box the ranks share device 0 (NKHIP_BENCH_ONE_DEVICE=1, gloo side
channel) and run the peer-memory communicator through IPC -- the multi-process path of the
8-GPU run minus xGMI.  Parity: the final timed step is a root of the oracle residual over the
whole gathered grid (final_step_check, sh_scipy_nk.py:47-49) within SciPy's default f_tol."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(600)
def test_bench_self_launch_four_ranks_one_gpu():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["NKHIP_BENCH_ONE_DEVICE"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--n",
                        "1024", "--steps", "2", "--warmup", "1", "--extra", "off", "--pmc", "off"],
                       env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=540)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 4 and d["steps"] == 2 and d["warmup"] == 1
    assert d["config"]["comm"] == "PeerComm", d["config"]
    assert d["comm_check"] == {"selftest": "ok", "pushed_rows_selftest": "ok",
                               "slab_path": "pushed"}, d["comm_check"]
    assert d["config"]["parallelism"] == "row-slab x4"
    fc = d["final_step_check"]
    assert fc["max_abs_residual"] <= fc["f_tol"], fc
    ab = d["slab_exchange_ab"]
    assert all(ab[f"{k}_ms_per_arnoldi"] > 0
               for k in ("pushed", "edge_halo", "in_kernel", "pushed_tail")), ab
    # the timed region ran the A/B's winner (ranks sharing a GPU take no tail: pushed_tail there
    # is the pushed path)
    assert d["config"]["slab_path"] in ("pushed", "edge_halo", "in_kernel", "pushed_tail")
    assert ab["selected"] == d["config"]["slab_path"]
    best = min(("pushed", "edge_halo", "in_kernel", "pushed_tail"),
               key=lambda k: ab[f"{k}_ms_per_arnoldi"])
    assert d["config"]["slab_path"] == ("pushed" if best == "pushed_tail" else best), ab
    # the roofline names the dominant streaming kernel (with four ranks time-sharing one GPU the
    # slab edge kernel's waits for the other processes are the largest kernel time: excluded)
    assert d["value"] > 0 and d["roofline"]["kernel"] == "arnoldi_fused"


@pytest.mark.timeout(600)
def test_bench_push_selftest_fault_falls_back_and_config5_leg():
    """Two things of the N > 1 line in one self-launched 2-rank run on this GPU:
    * fault injection: rank 1 pushes wrong rows in the pushed-halo-rows self-test
      (NKHIP_PEER_SELFTEST_BREAK_PUSH=1); every rank must then take the edge + halo exchange
      path (comm_check records it, the slab A/B skips the pushed variants) and still produce a
      root of the oracle residual;
    * config 5's leg after the headline (other_configs.config5: the grid of
      NKHIP_BENCH_CONFIG5_N, here 2048^2 instead of 16384^2, on the same ranks; its whole-grid
      oracle residual within f_tol)."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(NKHIP_BENCH_ONE_DEVICE="1", NKHIP_PEER_SELFTEST_BREAK_PUSH="1",
               NKHIP_BENCH_CONFIG5_N="2048")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--n",
                        "1024", "--steps", "1", "--warmup", "1", "--extra", "on", "--pmc", "off",
                        "--probes", "off", "--slab-ab", "1"],
                       env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=540)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["comm_check"]["pushed_rows_selftest"] == "failed on some rank", d["comm_check"]
    assert d["comm_check"]["slab_path"] == "edge_halo"
    assert "pushed_ms_per_arnoldi" not in d["slab_exchange_ab"], d["slab_exchange_ab"]
    assert d["slab_exchange_ab"]["edge_halo_ms_per_arnoldi"] > 0
    # the winner of the two exchange variants, never a pushed one
    assert d["config"]["slab_path"] in ("edge_halo", "in_kernel"), d["config"]
    fc = d["final_step_check"]
    assert fc["max_abs_residual"] <= fc["f_tol"], fc
    c5 = d["other_configs"]["config5"]
    assert c5["grid"] == 2048 and c5["n_gpus"] == 2 and c5["steps_per_s"] > 0, c5
    assert c5["ms_per_arnoldi_step"] > 0 and c5["newton_its_per_step"] >= 1
    assert c5["final_step_residual"] <= c5["f_tol"], c5
    assert c5["comm"] == "PeerComm"
    # the injected fault holds for its group: the headline's winner, never the pushed path
    assert c5["comm_check"]["slab_path"] == d["config"]["slab_path"], c5["comm_check"]


@pytest.mark.timeout(300)
def test_config4_trajectory_field():
    """bench.py's other_configs.config4_100 (BASELINE config 4 over its stated length, 100 implicit
    time steps of sh_scipy_nk.py:53-61 from default_rng(2020)) at a shrunken grid: every step a
    root of the reference residual, so the last one's oracle residual is within f_tol."""
    sys.path.insert(0, ROOT)
    import bench
    c4 = bench.config4_trajectory(n=128, steps=100)
    assert c4["steps"] == 100 and c4["gpu_steps_per_s"] > 0, c4
    assert c4["workload"] == "swift_hohenberg_cn_newton_krylov_128x128_100_steps"
    assert c4["newton_its_per_step"] >= 1 and c4["arnoldi_steps_per_step"] >= 1
    assert all(x >= 1 for x in c4["newton_its_first_last"]), c4
    assert c4["final_step_residual"] <= c4["f_tol"], c4
    assert c4["ms_per_arnoldi_step"] > 0

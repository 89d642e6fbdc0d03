"""CPU: bench.py's host-side decisions for the N > 1 line (no GPU touched).

* config 5's row slab of the seeded 16384^2 grid is drawn without materialising the rows before
  it (bench.slab_of_seeded_grid), and equals the rows of the one-shot draw;
* the slab path the timed region runs is the slab A/B's fastest variant (bench.select_slab_path),
  excluding a variant that failed, with its switches left in the environment, and the path named
  from the effective switches (bench.effective_slab_path) -- over a gloo world of one, as on the
  ranks (the choice is broadcast from rank 0).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

from conftest import ROOT  # noqa: F401 (import paths)

import bench

SWITCHES = ("NKHIP_SLAB_PUSH", "NKHIP_SLAB_XK", "NKHIP_ARN_TAIL", "NKHIP_ARN_TAIL_TIMEOUT_S")


@pytest.mark.parametrize("row0,ny,chunk", [(0, 5, 4), (7, 3, 4), (9, 4, 3), (300, 20, 256)])
def test_slab_of_seeded_grid_matches_one_draw(row0, ny, chunk):
    n = 48
    full = np.random.default_rng(2020).standard_normal((row0 + ny, n))
    got = bench.slab_of_seeded_grid(2020, n, row0, ny, chunk=chunk)
    assert np.array_equal(got, full[row0:])


@pytest.fixture
def clean_switches():
    old = {k: os.environ.get(k) for k in SWITCHES}
    for k in SWITCHES:
        os.environ.pop(k, None)
    yield
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def test_effective_slab_path(clean_switches):
    assert bench.effective_slab_path(True, False) == "pushed"
    assert bench.effective_slab_path(False, False) == "edge_halo"
    os.environ["NKHIP_SLAB_PUSH"] = "0"
    assert bench.effective_slab_path(True, False) == "edge_halo"
    os.environ["NKHIP_SLAB_PUSH"] = "1"
    os.environ["NKHIP_ARN_TAIL"] = "1"
    assert bench.effective_slab_path(True, False) == "pushed_tail"
    assert bench.effective_slab_path(True, True) == "pushed"  # ranks sharing a GPU: no tail
    os.environ["NKHIP_SLAB_XK"] = "2"
    assert bench.effective_slab_path(True, False) == "in_kernel"
    assert bench.effective_slab_path(True, True) == "pushed"  # XK=2 is off on a shared GPU
    os.environ["NKHIP_SLAB_XK"] = "1"
    assert bench.effective_slab_path(True, True) == "in_kernel"


@pytest.fixture
def gloo_world_of_one():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    yield
    dist.destroy_process_group()


def _rec(ms, steps=None, failed=None):
    rec = {f"{k}_ms_per_arnoldi": v for k, v in ms.items()}
    rec["arnoldi_steps"] = steps or {k: 10 for k in ms}
    if failed:
        rec["failed"], rec["failed_variant"] = f"{failed}: boom", failed
    return rec


def test_select_slab_path(clean_switches, gloo_world_of_one):
    rec = _rec({"pushed": 0.11, "edge_halo": 0.12, "in_kernel": 0.13, "pushed_tail": 0.10})
    assert bench.select_slab_path(rec, False, dist, torch) == "pushed_tail"
    assert os.environ["NKHIP_ARN_TAIL"] == "1" and os.environ["NKHIP_SLAB_XK"] == "0"
    # the tail failed (its time is that of the steps before the failure): out of the choice
    rec = _rec({"pushed": 0.11, "edge_halo": 0.10, "in_kernel": 0.13, "pushed_tail": 0.09},
               failed="pushed_tail")
    assert bench.select_slab_path(rec, False, dist, torch) == "edge_halo"
    assert os.environ["NKHIP_SLAB_PUSH"] == "0" and os.environ["NKHIP_ARN_TAIL"] == "0"
    # a variant that ran no step is out; the in-kernel exchange on one GPU is NKHIP_SLAB_XK=1
    rec = _rec({"pushed": 0.0, "edge_halo": 0.12, "in_kernel": 0.11},
               steps={"pushed": 0, "edge_halo": 5, "in_kernel": 5})
    assert bench.select_slab_path(rec, True, dist, torch) == "in_kernel"
    assert os.environ["NKHIP_SLAB_XK"] == "1"

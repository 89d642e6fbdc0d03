"""TEST INFRASTRUCTURE ONLY -- row-slab restatement of the SH operators over torch.distributed.

The reference is single-process.  The HIP build cuts the periodic N x N grid into row slabs
(``nkhip.dist.slab_rows``) and, before every 13-point stencil pass, fetches a 2-row halo from the
ring neighbours with the same posting order libnkhip uses on RCCL (csrc/comm.cpp RcclComm::halo):
send last 2 rows -> next, send first 2 rows -> prev, recv lo <- prev, recv hi <- next.  This
module restates that protocol with ``torch.distributed`` point-to-point calls (gloo on CPU) so the
decomposition can be checked against the single-slab oracle on world_size >= 2 without a GPU.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from .sh_oracle import sh_coeffs


def halo_exchange(v: torch.Tensor):
    """v: (ny, nx) local slab (CPU).  Returns (lo, hi), each (2, nx)."""
    rank, p = dist.get_rank(), dist.get_world_size()
    prev, nxt = (rank - 1) % p, (rank + 1) % p
    lo = torch.empty_like(v[:2])
    hi = torch.empty_like(v[:2])
    ops = [dist.P2POp(dist.isend, v[-2:].contiguous(), nxt),
           dist.P2POp(dist.isend, v[:2].contiguous(), prev),
           dist.P2POp(dist.irecv, lo, prev),
           dist.P2POp(dist.irecv, hi, nxt)]
    for req in dist.batch_isend_irecv(ops):
        req.wait()
    return lo, hi


def sh13_slab(v: torch.Tensor, lo: torch.Tensor, hi: torch.Tensor, h: float, r: float):
    """L v on one slab from its 2-row halos (x periodic)."""
    c0, c1, c2, c3 = sh_coeffs(h, r)
    ext = torch.cat([lo, v, hi], dim=0)  # rows -2 .. ny+1
    ny = v.shape[0]

    def s(dy, dx):
        return torch.roll(ext, shifts=-dx, dims=1)[2 + dy:2 + dy + ny]

    ax1 = s(0, -1) + s(0, 1) + s(-1, 0) + s(1, 0)
    dg = s(-1, -1) + s(-1, 1) + s(1, -1) + s(1, 1)
    ax2 = s(0, -2) + s(0, 2) + s(-2, 0) + s(2, 0)
    return c0 * v + c1 * ax1 + c2 * dg + c3 * ax2


def allreduce_sum_max(sums, maxes):
    t = torch.tensor(list(sums), dtype=torch.float64)
    m = torch.tensor(list(maxes), dtype=torch.float64)
    if len(sums):
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    if len(maxes):
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
    return t.numpy(), m.numpy()


def residual_slab(u, uo_lo_hi, u_lo_hi, uo, h, r, k, g):
    """Reference residual (sh_scipy_nk.py:47-49) on a slab, halos supplied."""
    Lu = sh13_slab(u, *u_lo_hi, h, r)
    Luo = sh13_slab(uo, *uo_lo_hi, h, r)
    uu = u * u
    return (u - uo) / k - (Lu + g * uu - u * uu + Luo + g * uo * uo - uo * (uo * uo)) / 2


def gather_rows(v: torch.Tensor, ny_global: int):
    """All-gather the slabs into the global (ny_global, nx) array (for checking only)."""
    p = dist.get_world_size()
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(p)]
    dist.all_gather(sizes, torch.tensor([v.shape[0]], dtype=torch.int64))
    mx = int(max(s.item() for s in sizes))
    pad = torch.zeros((mx, v.shape[1]), dtype=v.dtype)
    pad[:v.shape[0]] = v
    bufs = [torch.zeros_like(pad) for _ in range(p)]
    dist.all_gather(bufs, pad)
    out = torch.cat([b[:int(s.item())] for b, s in zip(bufs, sizes)], dim=0)
    assert out.shape[0] == ny_global
    return out


def as_np(t):
    return np.asarray(t.detach().cpu().numpy())

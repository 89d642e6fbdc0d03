"""nkhip -- MI355X-native Newton-Krylov Swift-Hohenberg time-stepper.

Drop-in for the hot path of Shiakaron/Iterative-solvers-summer-2020: ``python_work/sh_scipy_nk.py``
hands a 2-D grid state to ``scipy.optimize.newton_krylov`` once per implicit Crank-Nicolson step;
here the same surface (``newton_krylov``, ``SwiftHohenberg.step``) runs on hand-written gfx950 HIP
kernels through the C-ABI library ``libnkhip.so`` (include/nkhip.h).  There is no CPU fallback:
importing this package without the built library raises ImportError.
"""
from ._lib import NKError, lib, status_string  # noqa: F401
from .dist import PeerComm, RcclComm, loopback_comms, neighbours, peer_comms, slab_rows  # noqa: F401
from .droplet import Droplet, read_init, write_init  # noqa: F401
from .mems import Mems  # noqa: F401
from .ops import (axpy, dot, lap5_apply, maxnorm, maxpy, mdot, nrm2, scal, sh13_apply, stream_copy,  # noqa: F401
                  sh_arnoldi_fused, edge_gather, arnoldi_mbox_launches, sh_fdjvp, sh_jvp, sh_residual)
from .sh import SwiftHohenberg, sh_step  # noqa: F401
from .shlin import SHLinearised  # noqa: F401
from .solver import NoConvergence, newton_krylov  # noqa: F401

__version__ = lib.nk_version().decode()

"""ctypes binding of libnkhip.so (the C-ABI declared in include/nkhip.h).

The library is built in-tree (``make -C iterative-solvers-summer-2020_amd``) and loaded from this
directory.  There is no fallback: if the library is missing, importing ``nkhip`` raises.
"""
from __future__ import annotations

import ctypes as C
import os

# torch before the library: both need libamdhip64.so.7, and whichever loads first serves the
# process.  With libnkhip first, ROCm's runtime is bound and torch runs on it -- a fresh process
# that imported nkhip before torch then failed nk_drop_create with out-of-device-memory
# (scripts/dbg/drop_create_probe.py); torch first, both run on torch's.
import torch  # noqa: E402,F401

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libnkhip.so")
# NKHIP_LIB: an alternative build of the same C-ABI (kernel tuning builds, `make tune`)
LIB_PATH = os.environ.get("NKHIP_LIB") or LIB_PATH

NK_OK = 0
NK_NO_CONVERGENCE = 1
NK_NONFINITE = 2
NK_ZERO_STEP = 3
NK_BAD_RHS = 4
NK_EINVAL = -1
NK_EHIP = -2
NK_ECOMM = -3
NK_ENOMEM = -4
ABI_VERSION = 3  # include/nkhip.h NKHIP_ABI_VERSION: the struct layouts below
NK_JVP_FD = 0
NK_JVP_ANALYTIC = 1


class nk_opts(C.Structure):
    _fields_ = [("f_tol", C.c_double), ("f_rtol", C.c_double), ("x_tol", C.c_double),
                ("x_rtol", C.c_double), ("rdiff", C.c_double), ("maxiter", C.c_int64),
                ("inner_m", C.c_int32), ("outer_k", C.c_int32), ("line_search", C.c_int32),
                ("jvp_mode", C.c_int32), ("verbose", C.c_int32), ("profile", C.c_int32)]


class nk_stats(C.Structure):
    _fields_ = [("nit", C.c_int64), ("nfev", C.c_int64), ("njvp", C.c_int64),
                ("n_arnoldi", C.c_int64), ("fnorm_inf", C.c_double), ("fnorm_2", C.c_double),
                ("status", C.c_int32), ("pad_", C.c_int32), ("n_backtrack", C.c_int64),
                ("step_min", C.c_double), ("n_device_steps", C.c_int64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "pad_"}


class nk_kprof(C.Structure):
    _fields_ = [("name", C.c_char * 32), ("launches", C.c_int64), ("total_ms", C.c_double),
                ("alg_bytes", C.c_double), ("timed", C.c_int64), ("timed_bytes", C.c_double)]


class nk_drop_params(C.Structure):
    _fields_ = [("nx", C.c_int32), ("ny", C.c_int32), ("endl", C.c_double), ("endr", C.c_double),
                ("endb", C.c_double), ("endt", C.c_double), ("epsilon", C.c_double),
                ("n_exp", C.c_int32), ("m_exp", C.c_int32), ("Bo", C.c_double),
                ("alpha2", C.c_double), ("alpha", C.c_double), ("gamma", C.c_double),
                ("C", C.c_double), ("smoothing_iters", C.c_int32), ("pad_", C.c_int32),
                ("a", C.c_double)]


class nk_mems_params(C.Structure):
    _fields_ = [("n", C.c_int32), ("m", C.c_int32), ("smoothing_iters", C.c_int32),
                ("p", C.c_int32), ("alpha", C.c_double), ("gamma", C.c_double),
                ("epsilon", C.c_double), ("beta", C.c_double), ("lambd", C.c_double),
                ("endl", C.c_double), ("endr", C.c_double), ("k", C.c_double)]


RESIDUAL_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64)

_P = C.c_void_p
_D = C.c_double
_I64 = C.c_int64
_I32 = C.c_int32

# (name, restype, argtypes) -- exactly the entry points of include/nkhip.h
SIGNATURES = [
    ("nk_version", C.c_char_p, []),
    ("nk_abi_version", C.c_int, []),
    ("nk_opts_default", C.c_int, [C.POINTER(nk_opts)]),
    ("nk_status_string", C.c_char_p, [C.c_int]),
    ("nk_lap5_apply", C.c_int, [_P, _P, _I64, _I64, _D, _P]),
    ("nk_sh13_apply", C.c_int, [_P, _P, _I64, _I64, _D, _D, _P]),
    ("nk_sh_residual", C.c_int, [_P, _P, _P, _I64, _I64, _D, _D, _D, _D, _P]),
    ("nk_sh_jvp", C.c_int, [_P, _P, _P, _I64, _I64, _D, _D, _D, _D, _P]),
    ("nk_sh_fdjvp", C.c_int, [_P, _P, _P, _P, _I64, _I64, _D, _D, _D, _D, _D, _D, _P]),
    ("nk_sh_arnoldi_fused", C.c_int, [C.POINTER(_P), C.POINTER(_D), _I32, _P, _D, _P, _P, _P,
                                      _I64, _I64, _D, _D, _D, _D, _D, _D, _P, _P,
                                      C.POINTER(_D), _P]),
    ("nk_edge_elems", C.c_int64, [_I64, _I64]),
    ("nk_arnoldi_mbox_launches", C.c_int64, []),
    ("nk_edge_gather", C.c_int, [_P, _P, _I64, _I64, _P]),
    ("nk_sh_arnoldi_fused_edges", C.c_int, [C.POINTER(_P), C.POINTER(_P), C.POINTER(_D), _I32,
                                            _P, _D, _P, _P, _P, _I64, _I64, _D, _D, _D, _D, _D,
                                            _D, _P, _P, _P, _P, C.POINTER(_D), _P]),
    ("nk_dot", C.c_int, [_P, _P, _I64, C.POINTER(_D), _P]),
    ("nk_nrm2", C.c_int, [_P, _I64, C.POINTER(_D), _P]),
    ("nk_maxnorm", C.c_int, [_P, _I64, C.POINTER(_D), _P]),
    ("nk_axpy", C.c_int, [_D, _P, _P, _I64, _P]),
    ("nk_scal", C.c_int, [_D, _P, _I64, _P]),
    ("nk_mdot", C.c_int, [C.POINTER(_P), _I32, _P, _I64, C.POINTER(_D), _P]),
    ("nk_maxpy", C.c_int, [C.POINTER(_P), C.POINTER(_D), _I32, _P, _I64, _P]),
    ("nk_stream_copy", C.c_int, [_P, _P, _I64, _P]),
    ("nk_debug_bounds", C.c_int, [C.POINTER(_I64), C.POINTER(_I32), _I32]),
    ("nk_debug_mailbox", C.c_int, [C.POINTER(_I64), _I32]),
    ("nk_comm_unique_id_bytes", C.c_int, []),
    ("nk_comm_get_unique_id", C.c_int, [_P]),
    ("nk_comm_create_rccl", C.c_int, [C.POINTER(_P), _P, _I32, _I32]),
    ("nk_comm_create_loopback", C.c_int, [C.POINTER(_P), _I32]),
    ("nk_comm_peer_handle_bytes", C.c_int, []),
    ("nk_comm_create_peer", C.c_int, [C.POINTER(_P), _I32, _I32, _I64, _P]),
    ("nk_comm_peer_connect", C.c_int, [_P, _P]),
    ("nk_comm_destroy", C.c_int, [_P]),
    ("nk_comm_abort", C.c_int, [_P]),
    ("nk_comm_selftest", C.c_int, [_P, _I64, _P]),
    ("nk_comm_selftest_push", C.c_int, [_P, _I64, _P]),
    ("nk_sh_create", C.c_int, [C.POINTER(_P), _I64, _I64, _I64, _D, _D, _D, _D,
                               C.POINTER(nk_opts), _P, _P]),
    ("nk_sh_destroy", C.c_int, [_P]),
    ("nk_sh_step", C.c_int, [_P, _P, _P, C.POINTER(nk_stats)]),
    ("nk_sh_set_opts", C.c_int, [_P, C.POINTER(nk_opts)]),
    ("nk_sh_kernel_profile", C.c_int, [_P, C.POINTER(nk_kprof), _I32]),
    ("nk_sh_reset_profile", C.c_int, [_P]),
    ("nk_sh_step_log", C.c_int, [_P, C.POINTER(_D), _I32]),
    ("nk_sh_workspace_bytes", C.c_int64, [_P]),
    ("nk_solve_workspace_bytes", C.c_int64, [_I64, C.POINTER(nk_opts)]),
    ("nk_solve", C.c_int, [RESIDUAL_FN, _P, _P, _P, _I64, C.POINTER(nk_opts),
                           C.POINTER(nk_stats), _P, _P, _I64]),
    ("nk_drop_params_default", C.c_int, [C.POINTER(nk_drop_params)]),
    ("nk_drop_create", C.c_int, [C.POINTER(_P), C.POINTER(nk_drop_params), C.POINTER(nk_opts),
                                 _P]),
    ("nk_drop_destroy", C.c_int, [_P]),
    ("nk_drop_set_state", C.c_int, [_P, _P, _P]),
    ("nk_drop_get_state", C.c_int, [_P, _P, _P]),
    ("nk_drop_step", C.c_int, [_P, _D, _D, _I32, C.POINTER(nk_stats), C.POINTER(_D),
                               C.POINTER(_D)]),
    ("nk_drop_set_scale", C.c_int, [_P, _D]),
    ("nk_drop_prepare", C.c_int, [_P]),
    ("nk_drop_field", C.c_int, [_P, _I32, _P]),
    ("nk_drop_residual", C.c_int, [_P, _P, _D, _P]),
    ("nk_drop_solve", C.c_int, [_P, _D, _P, C.POINTER(nk_stats)]),
    ("nk_drop_pma", C.c_int, [_P, _D, _I32]),
    ("nk_drop_init_coalescing", C.c_int, [_P, _I32, C.POINTER(_D), _I32, _D, _I32]),
    ("nk_shlin_create", C.c_int, [C.POINTER(_P), _I64, _I64, _D, _D, _D, _D, _D, _I64, _P]),
    ("nk_shlin_destroy", C.c_int, [_P]),
    ("nk_shlin_step", C.c_int, [_P, _P, _P, _P, C.POINTER(_I64), C.POINTER(_D)]),
    ("nk_mems_params_default", C.c_int, [C.POINTER(nk_mems_params)]),
    ("nk_mems_create", C.c_int, [C.POINTER(_P), C.POINTER(nk_mems_params), C.POINTER(nk_opts),
                                 _P]),
    ("nk_mems_destroy", C.c_int, [_P]),
    ("nk_mems_set_state", C.c_int, [_P, _P, _P]),
    ("nk_mems_get_state", C.c_int, [_P, _P, _P]),
    ("nk_mems_step", C.c_int, [_P, C.POINTER(nk_stats), C.POINTER(_D), C.POINTER(_D)]),
    ("nk_mems_prepare", C.c_int, [_P, C.POINTER(_D)]),
    ("nk_mems_field", C.c_int, [_P, _I32, _P]),
    ("nk_mems_residual", C.c_int, [_P, _P, _P]),
]


def load(path: str = LIB_PATH) -> C.CDLL:
    if not os.path.exists(path):
        raise ImportError(
            f"nkhip: {path} is missing -- build it with `make -C iterative-solvers-summer-2020_amd` "
            "(or __graft_entry__.build()); there is no CPU fallback")
    lib = C.CDLL(path)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    got = lib.nk_abi_version()
    if got != ABI_VERSION:
        raise ImportError(f"nkhip: {path} has C-ABI version {got}, this binding expects "
                          f"{ABI_VERSION} (rebuild the library)")
    return lib


lib = load()


def status_string(code: int) -> str:
    return lib.nk_status_string(int(code)).decode()


def default_opts() -> nk_opts:
    o = nk_opts()
    lib.nk_opts_default(C.byref(o))
    return o


class NKError(RuntimeError):
    """A HIP / RCCL / argument failure inside libnkhip."""


def check(rc: int, what: str) -> int:
    if rc < 0:
        raise NKError(f"{what}: {status_string(rc)} ({rc})")
    return rc

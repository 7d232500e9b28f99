"""ctypes binding of libvihmc.so (C-ABI declared in include/vihmc.h).

The library is built in-tree (``make -C vi-hmc_amd``) next to this file. torch is imported first so
that its bundled HIP runtime (SONAME libamdhip64.so.7) is the one the library binds to -- one HIP
runtime per process. There is no CPU fallback: if the library is missing or fails to load, every
entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import re
import threading

import torch  # noqa: F401  (must be loaded before libvihmc.so, see module docstring)

# VIHMC_LIB overrides the library (A/B builds of kernel variants); default: the in-tree build
LIB_PATH = os.environ.get("VIHMC_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libvihmc.so")

c_int, c_int32, c_int64, c_float, c_double = ctypes.c_int, ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_double
c_void_p, c_char_p = ctypes.c_void_p, ctypes.c_char_p
P_float = ctypes.POINTER(ctypes.c_float)
P_int64 = ctypes.POINTER(ctypes.c_int64)


class Linear(ctypes.Structure):
    _fields_ = [("w_off", c_int64), ("b_off", c_int64), ("n_out", c_int32), ("n_in", c_int32),
                ("act", c_int32), ("_pad", c_int32)]


class LikDesc(ctypes.Structure):
    _fields_ = [("loss", c_int32), ("tau_out", c_float), ("prior_scale", c_float), ("_pad", c_int32)]


class DeepONetDesc(ctypes.Structure):
    _fields_ = [("n_branch_layers", c_int32), ("n_trunk_layers", c_int32),
                ("branch", ctypes.POINTER(Linear)), ("trunk", ctypes.POINTER(Linear)),
                ("n_params", c_int64), ("N", c_int32), ("P", c_int32), ("in_branch", c_int32),
                ("in_trunk", c_int32), ("K", c_int32), ("max_chains", c_int32), ("lik", LikDesc)]


class MLPDesc(ctypes.Structure):
    _fields_ = [("n_layers", c_int32), ("_pad0", c_int32), ("layers", ctypes.POINTER(Linear)),
                ("n_params", c_int64), ("N", c_int32), ("in_dim", c_int32), ("out_dim", c_int32),
                ("K", c_int32), ("max_chains", c_int32), ("_pad1", c_int32), ("lik", LikDesc)]


# name -> (restype, argtypes); exactly the functions include/vihmc.h declares
SIGNATURES = {
    "vihmc_deeponet_plan_create": (c_int, [ctypes.POINTER(c_void_p), ctypes.POINTER(DeepONetDesc), P_float, P_float,
                                           P_float, P_float, P_int64, P_float, P_float, c_int]),
    "vihmc_mlp_plan_create": (c_int, [ctypes.POINTER(c_void_p), ctypes.POINTER(MLPDesc), P_float, P_float, P_float,
                                      P_int64, P_float, P_float, c_int]),
    "vihmc_logp_grad": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "vihmc_grad": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "vihmc_forward": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "vihmc_hmc_accept": (c_int, [c_int, c_int, c_int, c_int] + [c_void_p] * 16 + [c_void_p, c_int64, c_void_p,
                                                                                   c_void_p, c_int64, c_void_p,
                                                                                   c_int64, c_void_p, c_void_p,
                                                                                   c_void_p]),
    "vihmc_kinetic_slices": (c_int, [c_int]),
    "vihmc_kinetic": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "vihmc_mlp_trajectory": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                     c_void_p, c_void_p, c_int, c_int, c_void_p]),
    "vihmc_trajectory": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                 c_void_p, c_void_p, c_int, c_int, c_void_p]),
    "vihmc_split_step": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, ctypes.c_float,
                                 ctypes.c_float, c_void_p, c_int, c_void_p]),
    "vihmc_sensitivity": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "vihmc_plan_set_data": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "vihmc_plan_set_trunk_rows": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    "vihmc_plan_kind": (c_int, [c_void_p]),
    "vihmc_plan_n_params": (c_int64, [c_void_p]),
    "vihmc_plan_K": (c_int, [c_void_p]),
    "vihmc_plan_max_chains": (c_int, [c_void_p]),
    "vihmc_plan_device_bytes": (c_int64, [c_void_p]),
    "vihmc_timing_enable": (c_int, [c_void_p, c_int, c_int]),
    "vihmc_graph_enable": (c_int, [c_void_p, c_int]),
    "vihmc_plan_option": (c_int, [c_void_p, c_char_p, c_int]),
    "vihmc_plan_get_option": (c_int, [c_void_p, c_char_p, ctypes.POINTER(c_int)]),
    "vihmc_timing_read": (c_int, [c_void_p, ctypes.POINTER(c_double), ctypes.POINTER(c_int64)]),
    "vihmc_timing_read_class": (c_int, [c_void_p, c_int, ctypes.POINTER(c_double), ctypes.POINTER(c_int64)]),
    "vihmc_timing_reset": (c_int, [c_void_p]),
    "vihmc_clock_stamp": (c_int, [c_void_p, c_void_p]),
    "vihmc_plan_check_canaries": (c_int, [c_void_p, ctypes.POINTER(c_int64)]),
    "vihmc_plan_debug_copy": (c_int, [c_void_p, ctypes.c_char_p, c_void_p, ctypes.POINTER(c_int64)]),
    "vihmc_plan_destroy": (None, [c_void_p]),
    "vihmc_last_error": (c_char_p, []),
    "vihmc_version": (c_char_p, []),
}

_lib = None
_lock = threading.Lock()


def lib() -> ctypes.CDLL:
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(f"libvihmc.so not built ({LIB_PATH}); run `make -C vi-hmc_amd` or "
                                   "__graft_entry__.build() -- there is no CPU fallback")
            L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            for name, (res, args) in SIGNATURES.items():
                f = getattr(L, name)
                f.restype = res
                f.argtypes = args
            ver = L.vihmc_version().decode()
            if not re.search(r"diag=0(\s|$)", ver) and os.environ.get("VIHMC_ALLOW_DIAG") != "1":
                raise RuntimeError(f"{LIB_PATH} was built with timing-only diagnostic switches ({ver}); its results "
                                   "are wrong by design. Rebuild without EXTRA=-D*_ABL/-D*_STAMP, or set "
                                   "VIHMC_ALLOW_DIAG=1 for A/B timing only")
            _lib = L
    return _lib


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().vihmc_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (code {rc}): {msg}")


def fptr(a) -> P_float:
    return a.ctypes.data_as(P_float)


def iptr(a) -> P_int64:
    return a.ctypes.data_as(P_int64)

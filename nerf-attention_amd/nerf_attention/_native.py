"""ctypes binding of the C ABI in include/nerfhip.h (libnerfhip.so).

There is no CPU fallback anywhere in this package: if the HIP library is
missing or a GPU is absent, the fit path raises.  `torch` is imported before
the library is loaded so that libnerfhip.so binds to the HIP runtime torch
already loaded (same SONAME libamdhip64.so.7) — one runtime per process, so
torch's device pointers and streams are valid handles for the engine.
"""

from __future__ import annotations

import ctypes
import os
from pathlib import Path
from ctypes import c_int32, c_int64, c_void_p, c_char_p, POINTER

import torch  # noqa: F401  (must precede the dlopen, see module docstring)

from ._build import LIB

ABI_VERSION = 5

# nerfhip_precision (include/nerfhip.h)
PRECISIONS = {"fp32": 0, "bf16x3": 1}


class NerfhipError(RuntimeError):
    pass


class NativeLibraryMissing(NerfhipError):
    pass


class NerfhipSizes(ctypes.Structure):
    _fields_ = [(name, c_int64) for name in (
        "n_pad", "params", "params_t", "scratch", "target", "stats", "loss_partial", "rows",
        "grad_split", "grad_partial", "wsplit")]


_GROUP_INTS = ("W", "D", "N", "n_fits", "L_max", "epochs", "log_every", "device",
               "precision", "reserved")
_GROUP_PTRS = ("fit_layers", "fit_omega", "positions", "target", "target_norm", "mean", "std",
               "params", "params_t", "adam_m", "adam_v", "scratch", "sched", "loss_partial",
               "probe_y", "eval_y", "row_cos", "row_sq", "probe_row_cos", "probe_row_sq",
               "grad_partial", "wsplit")


class NerfhipGroup(ctypes.Structure):
    _fields_ = [(n, c_int32) for n in _GROUP_INTS] + [(n, c_void_p) for n in _GROUP_PTRS]


SVD_MAX_RANKS = 8


class NerfhipSvdBatch(ctypes.Structure):
    _fields_ = ([(n, c_int32) for n in ("n_tensors", "N", "D", "n_ranks")]
                + [("ranks", c_int32 * SVD_MAX_RANKS), ("max_sweeps", c_int32),
                   ("reserved", c_int32)]
                + [(n, c_void_p) for n in ("x", "gram", "evec", "eval", "order", "row_cos",
                                          "stats")])


ANALYSIS_MAX_DIMS = 64


class NerfhipKvAnalysisBatch(ctypes.Structure):
    _fields_ = ([(n, c_int32) for n in ("n_tensors", "N", "D", "n_dims", "max_lag", "reserved")]
                + [("dims", c_int32 * ANALYSIS_MAX_DIMS)]
                + [(n, c_void_p) for n in ("x", "autocorr", "energy")])


class NerfhipTiming(ctypes.Structure):
    _fields_ = [("launches", c_int32), ("reserved", c_int32), ("rows_ms", ctypes.c_double),
                ("params_ms", ctypes.c_double)]


class NerfhipPlan(ctypes.Structure):
    _fields_ = [(n, c_int32) for n in ("rows_variant", "grad_split", "rows_workgroups",
                                        "params_workgroups", "launches_per_epoch", "reserved")]


ROWS_VARIANTS = {0: "regular", 1: "ksplit", 2: "rows32"}   # nerfhip_rows_variant

# every symbol include/nerfhip.h declares, with its ctypes signature
SIGNATURES = {
    "nerfhip_abi_version": (c_int32, []),
    "nerfhip_status_string": (c_char_p, [c_int32]),
    "nerfhip_group_sizes": (c_int32, [c_int32, c_int32, c_int32, c_int32, c_int32,
                                      POINTER(NerfhipSizes)]),
    "nerfhip_siren_fit": (c_int32, [POINTER(NerfhipGroup), c_int32, POINTER(c_void_p)]),
    "nerfhip_siren_fit_timed": (c_int32, [POINTER(NerfhipGroup), c_int32, POINTER(c_void_p),
                                          POINTER(NerfhipTiming)]),
    "nerfhip_siren_forward": (c_int32, [POINTER(NerfhipGroup), c_void_p]),
    "nerfhip_group_plan": (c_int32, [POINTER(NerfhipGroup), POINTER(NerfhipPlan)]),
    "nerfhip_build_flags": (c_int32, []),
    "nerfhip_svd_rank_metrics": (c_int32, [POINTER(NerfhipSvdBatch), c_void_p]),
    "nerfhip_kv_analysis": (c_int32, [POINTER(NerfhipKvAnalysisBatch), c_void_p]),
    "nerfhip_rng_uniform_segments": (c_int32, [c_void_p, POINTER(c_int32), POINTER(ctypes.c_uint32),
                                               c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                               c_void_p]),
}

_lib = None


def load(path=None) -> ctypes.CDLL:
    """Load libnerfhip.so (once).  Raises NativeLibraryMissing if absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # NERFHIP_LIB: an alternate build of the same ABI (variant A/B on the box)
    p = path or Path(os.environ.get("NERFHIP_LIB", LIB))
    if not p.exists():
        raise NativeLibraryMissing(
            f"{p} not found: build the HIP engine first "
            "(python -c 'import __graft_entry__ as g; g.build()' or "
            "python nerf-attention_amd/nerf_attention/_build.py)")
    lib = ctypes.CDLL(str(p))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.nerfhip_abi_version() != ABI_VERSION:
        raise NerfhipError(f"libnerfhip ABI {lib.nerfhip_abi_version()} != {ABI_VERSION}")
    if path is None:
        _lib = lib
    return lib


def check(rc: int) -> None:
    if rc != 0:
        msg = load().nerfhip_status_string(rc).decode()
        raise NerfhipError(f"nerfhip error {rc}: {msg}")


def group_sizes(W: int, D: int, N: int, L_max: int, epochs: int) -> NerfhipSizes:
    s = NerfhipSizes()
    check(load().nerfhip_group_sizes(W, D, N, L_max, epochs, ctypes.byref(s)))
    return s

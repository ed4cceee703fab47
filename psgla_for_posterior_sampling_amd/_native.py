"""ctypes binding of libpsgla_hip.so (C ABI declared in include/psgla_hip.h).

The library is built in-tree by :func:`psgla_for_posterior_sampling_amd.build.build_native`
(``__graft_entry__.build()``).  There is NO fallback: if the shared object is missing
or fails to load, every entry point raises :class:`NativeLibraryError`.
"""
from __future__ import annotations

import ctypes
import os

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PSGLA_LIB", os.path.join(_PKG, "libpsgla_hip.so"))
ABI_VERSION = 11
TV_MAX_FUSED_IT = 24


class NativeLibraryError(RuntimeError):
    pass


c_f = ctypes.c_float
c_i32 = ctypes.c_int32
c_i64 = ctypes.c_int64
c_u64 = ctypes.c_uint64
c_u32 = ctypes.c_uint32
c_vp = ctypes.c_void_p
c_dp = ctypes.c_void_p   # device pointers are passed as integers


class PsglaSchedule(ctypes.Structure):
    _fields_ = [
        ("d_step", c_vp), ("step_offset", c_i64), ("n_inter", c_i32), ("n_inter_mmse", c_i32),
        ("acc_coef", c_vp), ("samples", c_vp), ("samples_cap", c_i64), ("blocks", c_vp),
        ("blocks2", c_vp), ("blocks_cap", c_i64),
    ]


class PsglaTvStep(ctypes.Structure):
    _fields_ = [
        ("B", c_i32), ("C", c_i32), ("H", c_i32), ("W", c_i32),
        ("x", c_vp * 2), ("u2", c_vp * 2), ("x2", c_vp * 2), ("mean", c_vp * 2), ("sq", c_vp * 2),
        ("y", c_vp), ("y_chain_stride", c_i64), ("mask", c_vp), ("mask_chain_stride", c_i64),
        ("c1", c_f), ("c2", c_f), ("sigma2", c_f), ("alpha", c_f),
        ("tau", c_f), ("one_plus_tau", c_f), ("sigma_tv", c_f), ("rho", c_f), ("ths", c_f), ("tol", c_f),
        ("n_tv", c_i32), ("exact", c_i32), ("seed", c_u64), ("chain0", c_i32), ("advance_step", c_i32),
        ("fresh", c_vp), ("norms", c_vp), ("arrive", c_vp), ("launch_mask", c_i32),
        ("kernel_variant", c_i32), ("stream_wgs", c_i32), ("ldw", c_i32), ("norms_copies", c_i32),
        ("stream_windows", c_i32), ("redo", c_vp),
    ]


class PsglaTvProx(ctypes.Structure):
    _fields_ = [
        ("B", c_i32), ("C", c_i32), ("H", c_i32), ("W", c_i32),
        ("y", c_vp), ("x2_in", c_vp), ("u2_in", c_vp), ("x2_out", c_vp), ("u2_out", c_vp),
        ("tau", c_f), ("one_plus_tau", c_f), ("sigma_tv", c_f), ("rho", c_f), ("ths", c_f), ("tol", c_f),
        ("n_tv", c_i32), ("exact", c_i32), ("fresh", c_i32), ("norms", c_vp), ("arrive", c_vp),
        ("per_chain", c_i32), ("it0", c_i32), ("last_chunk", c_i32), ("stopped", c_vp),
    ]


_SIGNATURES = {
    "psgla_abi_version": (c_i32, []),
    "psgla_last_error": (ctypes.c_char_p, []),
    "psgla_tv_step": (c_i32, [ctypes.POINTER(PsglaTvStep), ctypes.POINTER(PsglaSchedule), c_vp]),
    "psgla_tv_prox": (c_i32, [ctypes.POINTER(PsglaTvProx), c_vp]),
    "psgla_tv_step_kernel": (c_i32, [ctypes.POINTER(PsglaTvStep)]),
    "psgla_normal_fill": (c_i32, [c_vp, c_i32, c_i64, c_i32, c_u64, c_i32, c_vp, c_i64, c_u32, c_vp]),
    "psgla_langevin_update": (c_i32, [c_vp, c_vp, c_vp, c_i32, c_i64, c_i32, c_f, c_f, c_u64, c_i32, c_vp,
                                      c_i64, c_vp]),
    "psgla_relax_accumulate": (c_i32, [c_vp, c_vp, c_vp, c_f, c_i32, c_vp, c_vp, c_i32, c_i64,
                                       ctypes.POINTER(PsglaSchedule), c_vp]),
    "psgla_relax_langevin_inpaint": (c_i32, [c_vp, c_vp, c_vp, c_f, c_i32, c_vp, c_i64, c_vp, c_i64, c_vp,
                                             c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_f, c_f, c_f, c_u64, c_i32,
                                             ctypes.POINTER(PsglaSchedule), c_vp]),
    "pnpula_update": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_f, c_f, c_f, c_f, c_f, c_vp, c_vp, c_i32, c_i64,
                              c_i32, c_u64, c_i32, ctypes.POINTER(PsglaSchedule), c_vp]),
    "pnpula_prior_update": (c_i32, [c_vp, c_vp, c_f, c_f, c_vp, c_vp, c_i64, c_vp, c_i64, c_f, c_vp, c_f, c_f, c_f,
                                    c_f, c_f, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_u64, c_i32,
                                    ctypes.POINTER(PsglaSchedule), c_vp]),
    "psgla_inpaint_grad": (c_i32, [c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_i32, c_i32, c_i32, c_i32, c_f,
                                   c_vp]),
    "psgla_blur_grad": (c_i32, [c_vp, c_vp, c_i64, c_vp, c_vp, c_i32, c_vp, c_vp, c_i32, c_i32, c_i32, c_i32,
                                c_f, c_f, c_f, c_u64, c_i32, c_vp, c_i64, c_i32, c_vp]),
    "psgla_blur_set_separable": (c_i32, [c_i32]),
    "psgla_advance_step": (c_i32, [c_vp, c_vp]),
    "psgla_bias_act": (c_i32, [c_vp, c_vp, c_i64, c_i32, c_i64, c_i32, c_vp]),
    "psgla_debug_bm_tables": (c_i32, [c_vp, c_vp, c_vp, c_u32, c_u32, c_vp]),
}

EXPORTED_SYMBOLS = tuple(_SIGNATURES)

_lib = None


def lib():
    """Load the native library (once).  Raises NativeLibraryError if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryError(
            f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    try:
        handle = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover
        raise NativeLibraryError(f"cannot load {LIB_PATH}: {e}") from e
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(handle, name)
        fn.restype = res
        fn.argtypes = args
    v = handle.psgla_abi_version()
    if v != ABI_VERSION:
        raise NativeLibraryError(f"libpsgla_hip ABI {v} != expected {ABI_VERSION}; rebuild")
    _lib = handle
    return _lib


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().psgla_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (hipError {rc}): {msg}")

"""ctypes binding of libof2d.so (include/of2d.h).

The shared library is built in-tree (``opticalflow2d_amd/libof2d.so``) by
``opticalflow2d_amd/csrc/Makefile``.  There is no CPU fallback: if the library
is missing or fails to load, :func:`lib` raises.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
# OF2D_LIB_PATH: another build of the same library (tools/ A/B runs only)
LIB_PATH = os.environ.get("OF2D_LIB_PATH") or os.path.join(PKG_DIR, "libof2d.so")

OF2D_OK = 0
OF2D_ERR_INVALID_ARGUMENT = 1
OF2D_ERR_RUNTIME = 2
OF2D_ERR_DEVICE = 3
OF2D_ERR_STATE = 4

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")

PRINT_FN = C.CFUNCTYPE(None, C.c_char_p, C.c_void_p)

# name -> (restype, argtypes); the list IS the exported surface of include/of2d.h
SIGNATURES = {
    "of2d_set_print_hook": (None, [PRINT_FN, C.c_void_p]),
    "of2d_create": (C.c_int, [C.POINTER(C.c_void_p), C.c_int, C.c_int, _i32p, C.c_int, C.c_int,
                              _f32p, C.c_uint, C.c_int, C.c_int]),
    "of2d_set_images": (C.c_int, [C.c_void_p, _f64p, _f64p]),
    "of2d_estimate": (C.c_int, [C.c_void_p]),
    "of2d_get_motion": (C.c_int, [C.c_void_p, _f64p]),
    "of2d_warp": (C.c_int, [C.c_void_p, _f64p, _f64p]),
    "of2d_destroy": (C.c_int, [C.c_void_p]),
    "of2d_last_error": (C.c_char_p, [C.c_void_p]),
    "of2d_iterations_executed": (C.c_int, [C.c_void_p, _i32p, C.c_int]),
    "of2d_last_errors": (C.c_int, [C.c_void_p, _f32p, C.c_int]),
    "of2d_set_option": (C.c_int, [C.c_void_p, C.c_char_p, C.c_double]),
    "of2d_gateway": (C.c_int, [C.c_int, C.POINTER(C.c_void_p), C.c_int, C.POINTER(C.c_void_p)]),
    "of2d_gateway_output_numel": (C.c_size_t, [C.c_int, C.c_int]),
    "of2d_gateway_output_dims": (C.c_int, [C.c_int, C.c_int, C.POINTER(C.c_size_t),
                                           C.POINTER(C.c_int)]),
    "of2d_gateway_last_error": (C.c_char_p, []),
    "of2d_slab_bounds": (C.c_int, [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int),
                                   C.POINTER(C.c_int)]),
    "of2d_rccl_unique_id_size": (C.c_int, []),
    "of2d_rccl_get_unique_id": (C.c_int, [C.c_void_p, C.c_int]),
    "of2d_slab_create": (C.c_int, [C.POINTER(C.c_void_p), C.c_int, C.c_int, C.c_float, C.c_int,
                                   C.c_int, C.c_int, C.c_void_p, C.c_int]),
    "of2d_slab_set_images": (C.c_int, [C.c_void_p, _f64p, _f64p]),
    "of2d_slab_reserve": (C.c_int, [C.c_void_p, C.c_int]),
    "of2d_slab_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.c_int]),
    "of2d_slab_run": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_int)]),
    "of2d_slab_get_motion": (C.c_int, [C.c_void_p, _f64p]),
    "of2d_slab_time_kernel": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_double)]),
    "of2d_slab_last_run_ms": (C.c_int, [C.c_void_p, C.POINTER(C.c_double)]),
    "of2d_slab_set_option": (C.c_int, [C.c_void_p, C.c_char_p, C.c_double]),
    "of2d_slab_last_run_kernel_us": (C.c_int, [C.c_void_p, C.POINTER(C.c_double),
                                                C.POINTER(C.c_int)]),
    "of2d_slab_last_run_halo_us": (C.c_int, [C.c_void_p, C.POINTER(C.c_double),
                                              C.POINTER(C.c_int)]),
    "of2d_slab_last_errors": (C.c_int, [C.c_void_p, _f32p, C.c_int]),
    "of2d_slab_destroy": (C.c_int, [C.c_void_p]),
    "of2d_slab_last_error": (C.c_char_p, [C.c_void_p]),
    "of2d_slab_group_create": (C.c_int, [C.POINTER(C.c_void_p), C.c_int]),
    "of2d_slab_group_destroy": (C.c_int, [C.c_void_p]),
    "of2d_slab_create_local": (C.c_int, [C.POINTER(C.c_void_p), C.c_int, C.c_int, C.c_float,
                                         C.c_int, C.c_int, C.c_int, C.c_void_p]),
    "of2d_motion_norms": (C.c_int, [_f32p, _f32p, C.c_int, C.c_int, C.c_int, _f32p, _i32p]),
    "of2d_motion_norms_chain": (C.c_int, [_f32p, C.c_int, C.c_int, C.c_int, C.c_int, _f32p, _i32p]),
    "of2d_version": (C.c_char_p, []),
    "of2d_device_count": (C.c_int, [C.POINTER(C.c_int)]),
}

_lib = None


def build(jobs: int = 8) -> str:
    """Compile libof2d.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    subprocess.check_call(["make", "-s", "-C", CSRC, f"-j{jobs}"])
    return LIB_PATH


def lib():
    """Load libof2d.so (raises if it is missing: there is no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"libof2d.so not found at {LIB_PATH}: build it with "
            "`make -C opticalflow2d_amd/csrc` (or __graft_entry__.build())")
    # One HIP runtime per process: when torch is importable, let it load its
    # libamdhip64.so.7 first so that ours resolves to the same soname.
    try:  # pragma: no cover - environment dependent
        import torch  # noqa: F401
    except Exception:
        pass
    L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


class Of2dError(RuntimeError):
    """Raised for a non-zero status; .status holds the OF2D_ERR_* code."""

    def __init__(self, status: int, message: str):
        super().__init__(message)
        self.status = status


class InvalidArgument(Of2dError, ValueError):
    pass


def check(status: int, message: str) -> None:
    if status == OF2D_OK:
        return
    if status == OF2D_ERR_INVALID_ARGUMENT:
        raise InvalidArgument(status, message)
    raise Of2dError(status, message)

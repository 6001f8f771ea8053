"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes front-end for oracle/liboracle.so (the C restatement of the reference,
oracle/of2d_oracle.c) and, where it was built, oracle/_ref/libref_prims.so (the
reference's own self-contained primitives compiled from /root/reference).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The product package `opticalflow2d_amd` never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
REF_LIB = os.path.join(HERE, "_ref", "libref_prims.so")

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")

_lib = None
_ref = None


def build(ref: bool | None = None) -> None:
    """Run oracle/Makefile (and the reference-primitives target when the
    reference tree is present)."""
    subprocess.check_call(["make", "-s", "-C", HERE, "all"])
    if ref is None:
        ref = os.path.isdir("/root/reference/src")
    if ref:
        subprocess.check_call(["make", "-s", "-C", HERE, "ref"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build(ref=False)
        L = C.CDLL(LIB)
        i, u, f, d = C.c_int, C.c_uint, C.c_float, C.c_double
        vp = C.c_void_p
        sig = {
            "oracle_create": (i, [C.POINTER(vp), i, i, _i32p, i, i, _f32p, u, i, i]),
            "oracle_set_images": (i, [vp, _f64p, _f64p]),
            "oracle_estimate": (i, [vp]),
            "oracle_get_motion": (i, [vp, _f64p]),
            "oracle_warp": (i, [vp, _f64p, _f64p]),
            "oracle_destroy": (None, [vp]),
            "oracle_last_error": (C.c_char_p, []),
            "oracle_iterations": (i, [vp, _i32p, i]),
            "oracle_set_fixed_iters": (None, [vp, i]),
            "oracle_last_errors": (i, [vp, _f32p, i]),
            "oracle_capture_output": (None, [i]),
            "oracle_captured_output": (C.c_char_p, []),
            "oracle_clear_output": (None, []),
            "oracle_spatial_derivative": (None, [_f32p, i, i, _f32p]),
            "oracle_temporal_derivative": (None, [_f32p, _f32p, i, _f32p]),
            "oracle_qlaplacian": (None, [_f32p, i, i, _f32p]),
            "oracle_hs_update": (i, [_f32p, _f32p, _f32p, i, i, f]),
            "oracle_hs_loop": (i, [_f32p, _f32p, _f32p, i, i, f, i, i, _f32p]),
            "oracle_hs_loop_mt": (i, [_f32p, _f32p, _f32p, i, i, f, i, i, _f32p]),
            "oracle_motion_norm": (f, [_f32p, i]),
            "oracle_motion_norm_sum": (f, [_f32p, i]),
            "oracle_motion_maxabs": (f, [_f32p, i]),
            "oracle_warp2d": (None, [_f32p, _f32p, i, i]),
            "oracle_accumulate": (None, [_f32p, _f32p, i, i]),
            "oracle_gaussian_kernel": (None, [i, f, _f64p]),
            "oracle_convolute_motion": (None, [_f32p, i, i, _f64p, i]),
            "oracle_convolute_image": (None, [_f32p, i, i, _f64p, i]),
            "oracle_downsample_image": (None, [_f32p, i, i, _f32p, i, i]),
            "oracle_upsample_image": (None, [_f32p, i, i, _f32p, i, i]),
            "oracle_downsample_motion": (None, [_f32p, i, i, _f32p, i, i]),
            "oracle_upsample_motion": (None, [_f32p, i, i, _f32p, i, i]),
            "oracle_demons_force": (i, [_f32p, _f32p, i, f, f, _f32p]),
            "oracle_jacobian": (None, [_f32p, i, i, _f32p]),
            "oracle_image_min": (f, [_f32p, i]),
            "oracle_motion_exp": (None, [_f32p, i, i]),
            "oracle_sor_sweep": (None, [_f32p, _f32p, i, i, f, f, f]),
            "oracle_get_force": (None, [_f32p, _f32p, _f32p, i, _f32p]),
            "oracle_dct2d": (None, [_f64p, i, i, i]),
            "oracle_fluid_increment": (None, [_f32p, _f32p, i, i, _f32p]),
            "oracle_set_reference_loop_order": (None, [i]),
            "oracle_set_logger_fp64": (None, [i]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def ref_lib():
    """Reference primitives (None when oracle/_ref was not built here)."""
    global _ref
    if _ref is None and os.path.exists(REF_LIB):
        L = C.CDLL(REF_LIB)
        u, f, i = C.c_uint, C.c_float, C.c_int
        L.ref_gaussian.argtypes = [u, f, _f64p]
        L.ref_spatial_derivative.argtypes = [_f32p, u, u, _f32p]
        L.ref_motion_partials.argtypes = [_f32p, u, u, _f32p, _f32p]
        L.ref_qlaplacian.argtypes = [_f32p, u, u, _f32p]
        L.ref_coord2d_div.argtypes = [f, f, f, _f32p]
        L.ref_coord2d_div.restype = i
        L.ref_hs_pointwise.argtypes = [_f32p, _f32p, _f32p, u, f, _f32p]
        L.ref_hs_pointwise.restype = i
        L.ref_norm_probe.argtypes = [_f32p, u]
        L.ref_norm_probe.restype = f
        L.ref_maxabs_probe.argtypes = [_f32p, u]
        L.ref_maxabs_probe.restype = f
        _ref = L
    return _ref


class OracleError(RuntimeError):
    pass


class Registration:
    """The oracle's registration object, driven like the reference's MEX
    singleton: init (create) -> register (set_images + estimate) -> get motion
    -> warp -> close (WrapperOpticalFlow2d.cpp:23-147)."""

    def __init__(self, dims, niter, nscales, reg, params, nrefine=1, verbose=0,
                 fixed_iters=False):
        L = lib()
        self.dimx, self.dimy = int(dims[0]), int(dims[1])
        niter = np.ascontiguousarray(np.asarray(niter, dtype=np.int32)[: nscales + 1])
        p = np.ascontiguousarray(np.asarray(params, dtype=np.float32).reshape(-1))
        if p.size == 0:
            p = np.zeros(1, np.float32)
            npar = 0
        else:
            npar = int(np.asarray(params).size)
        h = C.c_void_p()
        rc = L.oracle_create(C.byref(h), self.dimx, self.dimy, niter, int(nscales), int(reg),
                             p, npar, int(nrefine), int(verbose))
        if rc != 0:
            raise OracleError(L.oracle_last_error().decode())
        self._h = h
        if fixed_iters:
            L.oracle_set_fixed_iters(h, 1)

    def register(self, Iref, Imov):
        L = lib()
        r = np.ascontiguousarray(np.asarray(Iref, np.float64).reshape(-1, order="F"))
        m = np.ascontiguousarray(np.asarray(Imov, np.float64).reshape(-1, order="F"))
        rc = L.oracle_set_images(self._h, r, m)
        if rc == 0:
            rc = L.oracle_estimate(self._h)
        if rc != 0:
            raise OracleError(L.oracle_last_error().decode())

    def motion(self):
        out = np.zeros(self.dimx * self.dimy * 2, np.float64)
        lib().oracle_get_motion(self._h, out)
        return out.reshape((self.dimx, self.dimy, 2), order="F")

    def warp(self, Imov):
        m = np.ascontiguousarray(np.asarray(Imov, np.float64).reshape(-1, order="F"))
        out = np.zeros_like(m)
        lib().oracle_warp(self._h, m, out)
        return out.reshape((self.dimx, self.dimy), order="F")

    def iterations(self):
        buf = np.zeros(4096, np.int32)
        n = lib().oracle_iterations(self._h, buf, buf.size)
        return buf[:n].tolist()

    def last_errors(self):
        buf = np.zeros(1 << 16, np.float32)
        n = lib().oracle_last_errors(self._h, buf, buf.size)
        return buf[:n].copy()

    def close(self):
        if self._h:
            lib().oracle_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

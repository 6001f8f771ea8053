"""ctypes front-end of tests/stub/libof2d_mex_test.so: the real MEX adapter
(opticalflow2d_amd/mex/OpticalFlow2dMex.cpp) compiled against the repository's
stub mex.h, driven the way MATLAB calls `OpticalFlow2d(...)`."""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
STUB = os.path.join(HERE, "stub")
LIB = os.path.join(STUB, "libof2d_mex_test.so")
_lib = None


class MexError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.check_call(["make", "-s", "-C", STUB])
        from opticalflow2d_amd import _lib as of2d
        of2d.lib()  # libof2d.so first (RTLD_GLOBAL), then the adapter linked against it
        L = C.CDLL(LIB)
        L.mexdrv_call.restype = C.c_int
        L.mexdrv_call.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t),
                                  C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t),
                                  C.POINTER(C.c_int)]
        L.mexdrv_last_error.restype = C.c_char_p
        L.mexdrv_printed.restype = C.c_char_p
        _lib = L
    return _lib


def call(*args, nargout=0, out_numel=0):
    """OpticalFlow2d(args...) through mexFunction; returns plhs[0] reshaped
    to its mxArray dims (column-major) when nargout == 1."""
    L = lib()
    arrs = [np.ascontiguousarray(np.asarray(a, np.float64).reshape(-1, order="F")) for a in args]
    ptrs = (C.c_void_p * max(len(arrs), 1))(*[a.ctypes.data for a in arrs])
    numel = (C.c_size_t * max(len(arrs), 1))(*[a.size for a in arrs])
    out = np.zeros(max(out_numel, 1), np.float64)
    dims = (C.c_size_t * 3)()
    nd = C.c_int(0)
    rc = L.mexdrv_call(nargout, len(arrs), ptrs, numel, out.ctypes.data, out.size, dims,
                       C.byref(nd))
    if rc != 0:
        raise MexError(L.mexdrv_last_error().decode())
    if nargout == 1:
        shape = tuple(dims[k] for k in range(nd.value))
        n = int(np.prod(shape)) if shape else 0
        assert n <= out.size, "output larger than the buffer"
        return out[:n].reshape(shape, order="F")
    return None


def printed() -> str:
    return lib().mexdrv_printed().decode()


def clear_printed() -> None:
    lib().mexdrv_clear_printed()

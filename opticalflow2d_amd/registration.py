"""Host-side mirror of the reference's operator interface.

* :class:`Regularisation`, :class:`Verbose`, :class:`MotionAccumulation` —
  ``src/SolverOptions.h:4-8`` with the same integer values.
* :func:`OpticalFlow2d` — the MEX entry point ``OpticalFlow2d(...)`` with the
  five call modes of ``WrapperOpticalFlow2d.cpp:23-151`` (keyed on nargout /
  nargin and whether the process-global singleton exists), routed through the
  C-ABI gateway ``of2d_gateway`` of libof2d.so.
* :class:`ImageRegistration` — an object-style handle on the same C-ABI
  (``of2d_create`` ... ``of2d_destroy``) for callers that want more than one
  registration per process.

Arrays follow MATLAB's convention used by the reference: an image is
``[dimx, dimy]`` in Fortran (column-major, x fastest) order and a motion field
is ``[dimx, dimy, 2]``.
"""
from __future__ import annotations

import ctypes as C
import enum
import threading
from typing import Callable, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import Of2dError, check


class Regularisation(enum.IntEnum):
    Diffusion = 0
    Curvature = 1
    Elastic = 2
    ThirionsDemons = 3
    DiffeomorphicDemons = 4
    Fluid = 5


class Verbose(enum.IntEnum):
    Off = 0
    On = 1


class MotionAccumulation(enum.IntEnum):
    Composition = 0
    Addition = 1


# ------------------------------------------------------------------ printing
_print_lock = threading.Lock()
_print_sink: Optional[Callable[[str], None]] = None
_print_cb = None


def set_print_sink(fn: Optional[Callable[[str], None]]) -> None:
    """Redirect the reference's mexPrintf text (banner, Logger and Fluid lines).
    ``None`` restores stdout."""
    global _print_sink, _print_cb
    L = _lib.lib()
    with _print_lock:
        _print_sink = fn
        if fn is None:
            _print_cb = None
            L.of2d_set_print_hook(_lib.PRINT_FN(), None)
        else:
            def _cb(text, _user):
                _print_sink(text.decode(errors="replace"))

            _print_cb = _lib.PRINT_FN(_cb)
            L.of2d_set_print_hook(_print_cb, None)


def _col(a, n: int) -> np.ndarray:
    """Column-major double copy of an array (the reference reads mxGetPr)."""
    v = np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape(-1, order="F"))
    if v.size < n:
        raise ValueError(f"array has {v.size} elements, expected {n}")
    return v


def _vec(a) -> np.ndarray:
    return np.ascontiguousarray(np.atleast_1d(np.asarray(a, dtype=np.float64)).reshape(-1))


# ------------------------------------------------------------------ gateway
def OpticalFlow2d(*args, nargout: int = 0):
    """The MEX function, mode for mode (WrapperOpticalFlow2d.cpp:23-151).

    ``OpticalFlow2d([dimx, dimy], niter, nscales, reg, params, nparams, nrefine, verbose)``
        initialise the process-global registration object (a ninth argument,
        not in the reference: the number of devices Horn-Schunck runs on);
    ``OpticalFlow2d(Iref, Imov)``      register (estimate motion);
    ``OpticalFlow2d(nargout=1)``       return the motion field ``[dimx, dimy, 2]``;
    ``OpticalFlow2d(Imov, nargout=1)`` return Imov warped by the motion;
    ``OpticalFlow2d()``                close.
    Any other combination raises, like ``mexErrMsgTxt``.  The reference reads
    its inputs with ``mxGetPr`` unchecked; here short arrays are refused before
    they reach the library.
    """
    L = _lib.lib()
    nrhs = len(args)
    keep = [np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape(-1, order="F"))
            for a in args]
    n_img = int(L.of2d_gateway_output_numel(1, 1))  # 0 when no singleton exists
    if nargout == 0 and nrhs in (8, 9) and n_img == 0:
        nscales = int(keep[2][0]) if keep[2].size else 0
        nparams = int(keep[5][0]) if keep[5].size else 0
        if keep[0].size < 2 or keep[1].size < nscales + 1 or keep[4].size < nparams:
            raise ValueError("init: [dimx dimy], niter (nscales+1) and params (nparams) sizes")
    elif n_img and ((nargout == 0 and nrhs == 2) or (nargout == 1 and nrhs == 1)):
        if any(v.size < n_img for v in keep):
            raise ValueError(f"images must have {n_img} elements")
    prhs = (C.c_void_p * max(nrhs, 1))(*[v.ctypes.data for v in keep])
    plhs = (C.c_void_p * max(nargout, 1))()
    out = shape = None
    if nargout == 1:
        dims = (C.c_size_t * 3)()
        nd = C.c_int(0)
        if L.of2d_gateway_output_dims(1, nrhs, dims, C.byref(nd)) == _lib.OF2D_OK:
            shape = tuple(int(dims[i]) for i in range(nd.value))
            out = np.zeros(int(np.prod(shape)), np.float64)
            plhs[0] = out.ctypes.data
    st = L.of2d_gateway(nargout, plhs, nrhs, prhs)
    check(st, L.of2d_gateway_last_error().decode())
    if out is not None:
        return out.reshape(shape, order="F")
    return None


# ------------------------------------------------------------------ Logger norms
def motion_norms(cur, prev, dims: Sequence[int]):
    """Motion::norm sums of (cur - prev) and of prev exactly as the reference's
    Logger takes them (src/Motion.cpp:42-49, src/Logger.cpp:32-51): float
    running sums in linear order, on the device.  ``cur`` / ``prev`` are
    float32 ``[dimx*dimy, 2]`` (interleaved x, y per pixel, idx = i + j*dimx),
    or ``[npairs, dimx*dimy, 2]`` for a sequence of Logger updates run on one
    workspace (each predicts the next).  Returns ``(sums float32[..., 2],
    stats int32[..., 8])``: stats are cost figures of the device walk
    (include/of2d.h of2d_motion_norms), not results."""
    dimx, dimy = int(dims[0]), int(dims[1])
    c = np.ascontiguousarray(np.asarray(cur, np.float32).reshape(-1))
    p = np.ascontiguousarray(np.asarray(prev, np.float32).reshape(-1))
    n = 2 * dimx * dimy
    if c.size % n or p.size != c.size or c.size == 0:
        raise ValueError("cur / prev need npairs * dimx*dimy*2 floats")
    k = c.size // n
    sums = np.zeros(2 * k, np.float32)
    res = np.zeros(8 * k, np.int32)
    L = _lib.lib()
    check(L.of2d_motion_norms(c, p, dimx, dimy, k, sums, res),
          L.of2d_gateway_last_error().decode())
    if np.asarray(cur).ndim == 3:
        return sums.reshape(k, 2), res.reshape(k, 8)
    return sums, res


def motion_norms_chain(u, dims: Sequence[int], batch: int = 3):
    """The Logger norms of each update of a chain of iterates ``u``
    (float32 ``[niter + 1, dimx*dimy, 2]``), computed in batches of ``batch``
    updates as the registration loop runs them (include/of2d.h
    of2d_motion_norms_chain).  Returns ``(sums float32[niter, 2], stats
    int32[niter, 8])``."""
    dimx, dimy = int(dims[0]), int(dims[1])
    a = np.ascontiguousarray(np.asarray(u, np.float32).reshape(-1))
    n = 2 * dimx * dimy
    if a.size % n or a.size < 2 * n:
        raise ValueError("u needs (niter + 1) * dimx*dimy*2 floats")
    niter = a.size // n - 1
    sums = np.zeros(2 * niter, np.float32)
    res = np.zeros(8 * niter, np.int32)
    L = _lib.lib()
    check(L.of2d_motion_norms_chain(a, dimx, dimy, niter, int(batch), sums, res),
          L.of2d_gateway_last_error().decode())
    return sums.reshape(niter, 2), res.reshape(niter, 8)


# ------------------------------------------------------------------ object API
class ImageRegistration:
    """Handle on one registration context (of2d_create ... of2d_destroy).

    Parameters mirror the init call: ``dims=(dimx, dimy)``, ``niter`` (nscales+1
    values, finest level first), ``nscales``, ``reg``, ``params`` (nparams
    floats), ``nrefine``, ``verbose``.  Extra keyword options map to
    ``of2d_set_option`` (``fixed_iters``, ``chunk``, ``device``,
    ``hs_gradients_from_image``, ``logger_fp64``, ``ngpus``).
    """

    def __init__(self, dims: Sequence[int], niter: Sequence[int], nscales: int, reg: int,
                 params: Sequence[float], nrefine: int = 1, verbose: int = 0, **options):
        L = _lib.lib()
        self.dimx, self.dimy = int(dims[0]), int(dims[1])
        nit = np.ascontiguousarray(np.asarray(niter, dtype=np.int32).reshape(-1)[: nscales + 1])
        if nit.size < nscales + 1:
            raise ValueError("niter needs nscales+1 entries")
        p = np.ascontiguousarray(np.asarray(params, dtype=np.float32).reshape(-1))
        npar = int(p.size)
        if npar == 0:
            p = np.zeros(1, np.float32)
        h = C.c_void_p()
        st = L.of2d_create(C.byref(h), self.dimx, self.dimy, nit, int(nscales), int(reg), p,
                           npar, int(nrefine), int(verbose))
        check(st, L.of2d_last_error(None).decode())
        self._h = h
        for k, v in options.items():
            self.set_option(k, v)

    def _chk(self, st):
        check(st, _lib.lib().of2d_last_error(self._h).decode())

    def set_option(self, key: str, value: float) -> None:
        self._chk(_lib.lib().of2d_set_option(self._h, key.encode(), float(value)))

    def register(self, Iref, Imov) -> None:
        self.set_images(Iref, Imov)
        self.estimate()

    def set_images(self, Iref, Imov) -> None:
        """Upload the image pair (the first half of register)."""
        n = self.dimx * self.dimy
        r, m = _col(Iref, n), _col(Imov, n)
        self._chk(_lib.lib().of2d_set_images(self._h, r, m))

    def estimate(self) -> None:
        """Run the pyramid on the images already on the device."""
        self._chk(_lib.lib().of2d_estimate(self._h))

    def motion(self) -> np.ndarray:
        out = np.zeros(self.dimx * self.dimy * 2, np.float64)
        self._chk(_lib.lib().of2d_get_motion(self._h, out))
        return out.reshape((self.dimx, self.dimy, 2), order="F")

    def warp(self, Imov) -> np.ndarray:
        n = self.dimx * self.dimy
        m = _col(Imov, n)
        out = np.zeros(n, np.float64)
        self._chk(_lib.lib().of2d_warp(self._h, m, out))
        return out.reshape((self.dimx, self.dimy), order="F")

    def iterations(self) -> list:
        buf = np.zeros(4096, np.int32)
        n = _lib.lib().of2d_iterations_executed(self._h, buf, buf.size)
        return buf[: max(n, 0)].tolist()

    def last_errors(self) -> np.ndarray:
        buf = np.zeros(1 << 16, np.float32)
        n = _lib.lib().of2d_last_errors(self._h, buf, buf.size)
        return buf[: max(n, 0)].copy()

    def close(self) -> None:
        if getattr(self, "_h", None):
            _lib.lib().of2d_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


__all__ = ["Regularisation", "Verbose", "MotionAccumulation", "OpticalFlow2d",
           "ImageRegistration", "set_print_sink", "Of2dError", "motion_norms"]

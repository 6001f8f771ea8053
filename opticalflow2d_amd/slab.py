"""Row-slab Horn-Schunck across GPUs (one process per GPU, RCCL halo).

Python handle on the ``of2d_slab_*`` part of the C-ABI.  The decomposition is
``of2d_slab_bounds``: rank r of N owns j-lines [row_begin, row_end) of the
global grid; the RCCL unique id is created by rank 0 with
``of2d_rccl_get_unique_id`` and handed to the other ranks by the caller (for
example over ``torch.distributed`` with the gloo backend).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Tuple

import numpy as np

from . import _lib
from ._lib import check


def slab_bounds(dimy: int, rank: int, nranks: int) -> Tuple[int, int]:
    """[row_begin, row_end) of rank's slab (contiguous j-lines, remainder to the
    lowest ranks)."""
    b, e = C.c_int(), C.c_int()
    st = _lib.lib().of2d_slab_bounds(int(dimy), int(rank), int(nranks), C.byref(b), C.byref(e))
    check(st, "slab_bounds: invalid arguments")
    return b.value, e.value


def halo_rows(dimy: int, rank: int, nranks: int) -> Tuple[int, int]:
    """Image rows a rank must supply: [row_begin-3, row_end+3) clipped (the
    fused kernels' first step covers two halo j-lines, whose gradients need one
    more)."""
    b, e = slab_bounds(dimy, rank, nranks)
    return max(b - 3, 0), min(e + 3, dimy)


def rccl_unique_id() -> bytes:
    L = _lib.lib()
    n = L.of2d_rccl_unique_id_size()
    buf = (C.c_char * n)()
    check(L.of2d_rccl_get_unique_id(buf, n), "ncclGetUniqueId failed")
    return bytes(buf)


class SlabGroup:
    """The ranks of one grid inside one process (``of2d_slab_group``): slabs
    created with ``group=`` exchange halos and Logger sums by device copies
    instead of RCCL; drive each rank's ``run`` from its own thread.  Used to run
    the decomposition on a single GPU (RCCL refuses two ranks on one device)."""

    def __init__(self, nranks: int):
        h = C.c_void_p()
        check(_lib.lib().of2d_slab_group_create(C.byref(h), int(nranks)),
              "slab group: nranks out of range")
        self.nranks = int(nranks)
        self._h = h

    def close(self) -> None:
        if getattr(self, "_h", None):
            check(_lib.lib().of2d_slab_group_destroy(self._h),
                  "slab group: destroy its slabs first")
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SlabSolver:
    """One rank's slab of a global HS registration (zero initial motion, one
    level, one refine — see opticalflow2d_amd/csrc/slab.cpp)."""

    def __init__(self, dimx: int, dimy: int, alpha: float, rank: int = 0, nranks: int = 1,
                 device: int = 0, unique_id: Optional[bytes] = None,
                 group: Optional[SlabGroup] = None):
        L = _lib.lib()
        self.dimx, self.dimy, self.rank, self.nranks = int(dimx), int(dimy), rank, nranks
        self.row_begin, self.row_end = slab_bounds(dimy, rank, nranks)
        h = C.c_void_p()
        if group is not None:
            st = L.of2d_slab_create_local(C.byref(h), self.dimx, self.dimy, float(alpha), rank,
                                          nranks, device, group._h)
        else:
            uid = None
            n = 0
            if unique_id is not None:
                uid = C.create_string_buffer(unique_id, len(unique_id))
                n = len(unique_id)
            st = L.of2d_slab_create(C.byref(h), self.dimx, self.dimy, float(alpha), rank,
                                    nranks, device, uid, n)
        check(st, L.of2d_slab_last_error(None).decode())
        self._h = h

    def _chk(self, st):
        check(st, _lib.lib().of2d_slab_last_error(self._h).decode())

    def set_images(self, Iref_rows: np.ndarray, Imov_rows: np.ndarray) -> None:
        """Rows [row_begin-3, row_end+3) (clipped, see halo_rows) of the global
        images as arrays of shape [dimx, rows] (column-major, x fastest)."""
        lo, hi = halo_rows(self.dimy, self.rank, self.nranks)
        n = self.dimx * (hi - lo)
        r = np.ascontiguousarray(np.asarray(Iref_rows, np.float64).reshape(-1, order="F"))
        m = np.ascontiguousarray(np.asarray(Imov_rows, np.float64).reshape(-1, order="F"))
        if r.size != n or m.size != n:
            raise ValueError(f"expected {n} values (rows {lo}..{hi})")
        self._chk(_lib.lib().of2d_slab_set_images(self._h, r, m))

    def reserve(self, niter: int) -> None:
        """Size the per-iteration Logger sums of a fixed_iters run of `niter`
        iterations now, so that run allocates nothing."""
        self._chk(_lib.lib().of2d_slab_reserve(self._h, int(niter)))

    def info(self) -> dict:
        """nranks, the RCCL communicator's rank count (ncclCommCount; 0 without
        one), rows, pitch, halo lines per fused launch, interior/edge split,
        whether the triple kernel derives dI from Iaux, and the Logger a
        convergence-on run takes (1: the reference's float running sums, 0:
        fp64 sums)."""
        buf = (C.c_int * 11)()
        n = _lib.lib().of2d_slab_info(self._h, buf, 11)
        if n < 0:
            self._chk(-n)
        keys = ["nranks", "rccl_ranks", "in_process_group", "row_begin", "row_end", "dimx",
                "pitch", "halo_lines", "split", "gradients_from_image", "logger_reference"]
        return {k: int(buf[i]) for i, k in enumerate(keys[:n])}

    def set_option(self, key: str, value: float) -> None:
        """Tuning switch (include/of2d.h of2d_slab_set_option), e.g.
        "hs_gradients_from_image" 0/1; results are bit-identical either way."""
        self._chk(_lib.lib().of2d_slab_set_option(self._h, key.encode(), float(value)))

    def run(self, niter: int, fixed_iters: bool = False) -> int:
        done = C.c_int(0)
        self._chk(_lib.lib().of2d_slab_run(self._h, int(niter), int(bool(fixed_iters)),
                                           C.byref(done)))
        return done.value

    def motion(self) -> np.ndarray:
        rows = self.row_end - self.row_begin
        out = np.zeros(self.dimx * rows * 2, np.float64)
        self._chk(_lib.lib().of2d_slab_get_motion(self._h, out))
        return out.reshape((self.dimx, rows, 2), order="F")

    def time_kernel(self, nlaunch: int = 50) -> float:
        us = C.c_double(0.0)
        self._chk(_lib.lib().of2d_slab_time_kernel(self._h, int(nlaunch), C.byref(us)))
        return us.value

    def last_run_kernel_us(self) -> tuple:
        """(average us per triple launch, launches averaged) inside the last run."""
        us = C.c_double(0.0)
        n = C.c_int(0)
        self._chk(_lib.lib().of2d_slab_last_run_kernel_us(self._h, C.byref(us), C.byref(n)))
        return us.value, n.value

    def last_run_halo_us(self) -> dict:
        """The halo's cost inside the last run, sampled on its first split
        triples (include/of2d.h of2d_slab_last_run_halo_us): the solver stream's
        stall on the previous edge launches, the exchange, the edge launches
        (us per sampled launch), and the launches sampled."""
        us = (C.c_double * 3)()
        n = C.c_int(0)
        self._chk(_lib.lib().of2d_slab_last_run_halo_us(self._h, us, C.byref(n)))
        return {"stall_us": us[0], "exchange_us": us[1], "edges_us": us[2],
                "sampled": n.value}

    def errors(self) -> np.ndarray:
        """The Logger errors of the last run's iterations (float32; global)."""
        L = _lib.lib()
        k = L.of2d_slab_last_errors(self._h, np.zeros(1, np.float32), 0)
        if k < 0:
            self._chk(-k)
        out = np.zeros(max(k, 1), np.float32)
        L.of2d_slab_last_errors(self._h, out, k)
        return out[:k]

    def last_run_ms(self) -> float:
        ms = C.c_double(0.0)
        self._chk(_lib.lib().of2d_slab_last_run_ms(self._h, C.byref(ms)))
        return ms.value

    def close(self) -> None:
        if getattr(self, "_h", None):
            _lib.lib().of2d_slab_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

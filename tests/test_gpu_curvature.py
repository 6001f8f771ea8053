"""Curvature (biharmonic) registration on the MI355X against the oracle.

The reference transforms with FFTW's REDFT10/REDFT01 (OpticalFlowCurvature.cpp:52-55),
which this image does not have; the oracle restates the r2r definitions as
naive sums in double and the device evaluates the same definitions as fp64
MFMA GEMMs (curvature_kernels.hip).  The fp64 rounding of the two differs
(fused MFMA accumulation vs separate multiply and add), so the bar is a
tolerance: max |du| <= 1e-5 px after the double -> float conversion, and
identical iteration counts.  (On MI355X the float results have come out
bitwise equal on every shape tried.)  Parity against FFTW itself is UNPINNED
(no FFTW here).
"""
import numpy as np
import pytest

from opticalflow2d_amd import ImageRegistration
from opticalflow2d_amd import synthetic as S

pytestmark = pytest.mark.gpu

TOL = 1e-5


def both(oracle, dims, niter, nscales, params, ref, mov, nrefine=1, **opt):
    with ImageRegistration(dims, niter, nscales, 1, params, nrefine, **opt) as r:
        r.register(ref, mov)
        g = dict(motion=r.motion(), warped=r.warp(mov), iters=r.iterations())
    o = oracle.Registration(dims, niter, nscales, 1, params, nrefine, 0,
                            fixed_iters=bool(opt.get("fixed_iters", 0)))
    o.register(ref, mov)
    w = dict(motion=o.motion(), warped=o.warp(mov), iters=o.iterations())
    o.close()
    return g, w


@pytest.mark.parametrize("dims", [(64, 64), (70, 37), (5, 4), (130, 96)])
def test_curvature_fixed_iterations(gpu, oracle, dims):
    ref, mov = S.texture_pair(max(dims), seed=5)
    ref, mov = ref[: dims[0], : dims[1]], mov[: dims[0], : dims[1]]
    g, w = both(oracle, dims, [8], 0, [0.5, 0.2], ref, mov, fixed_iters=1)
    assert g["iters"] == w["iters"] == [8]
    assert np.abs(g["motion"] - w["motion"]).max() <= TOL


def test_curvature_default_tau_pyramid_convergence(gpu, oracle):
    """nparams = 1 (tau = 1), two levels, convergence break on."""
    ref, mov = S.texture_pair(96, seed=2)
    g, w = both(oracle, (96, 96), [60, 40], 1, [2.0], ref, mov)
    assert g["iters"] == w["iters"]
    assert np.abs(g["motion"] - w["motion"]).max() <= TOL
    assert np.abs(g["warped"] - w["warped"]).max() <= 1e-4


def test_curvature_chunked_replay(gpu, oracle):
    ref, mov = S.texture_pair(48, seed=9)
    for chunk in (1, 7):
        g, w = both(oracle, (48, 48), [200], 0, [1.0, 0.5], ref, mov, chunk=chunk)
        assert g["iters"] == w["iters"]
        assert np.abs(g["motion"] - w["motion"]).max() <= TOL

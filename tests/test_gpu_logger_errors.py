"""Every solver's convergence-on loop against the oracle, Logger errors
included: with the default Logger (the reference's float running sums,
Motion.cpp:42-49 as Logger::update_error takes them, Logger.cpp:32-51) each
iteration's error is the reference's float32 value, so the break test
(`err < 0.001f && iter > 1`, ImageRegistrationOpticalFlow.cpp:131-134 and its
Demons / Fluid counterparts) falls on the same iteration.

Bar: iteration counts equal, the motion bit for bit, and the last loop's
errors bit for bit (their float32 patterns) — on ragged grids, pyramids with
refines, and each solver's own loop (HS's pipelined triples, Demons' and
Curvature's chunked loops, Elastic's and Fluid's per-iteration norms).
Curvature's DCT is fp64 MFMA against the oracle's naive sums (parity vs FFTW
unpinned, test_gpu_curvature.py), so its motion and errors take a tolerance.
"""
import numpy as np
import pytest

from opticalflow2d_amd import ImageRegistration
from opticalflow2d_amd import synthetic as S

pytestmark = pytest.mark.gpu


def both(oracle, dims, niter, nscales, reg, params, nrefine, ref, mov):
    with ImageRegistration(dims, niter, nscales, reg, params, nrefine) as r:
        r.register(ref, mov)
        g = dict(motion=r.motion(), iters=r.iterations(), errs=r.last_errors())
    o = oracle.Registration(dims, niter, nscales, reg, params, nrefine, 0)
    o.register(ref, mov)
    w = dict(motion=o.motion(), iters=o.iterations(), errs=o.last_errors())
    o.close()
    return g, w


def crop(pair, dims):
    return tuple(np.ascontiguousarray(a[: dims[0], : dims[1]]) for a in pair)


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32).tolist()


CASES = {
    # name: (dims, niter, nscales, reg, params, nrefine, inputs)
    "hs_texture_pyramid_refine": ((200, 136), [300, 200, 150], 2, 0, [0.15], 2,
                                  lambda: S.texture_pair(200, seed=11, ny=136)),
    "hs_square_ragged": ((129, 65), [800], 0, 0, [0.1], 1,
                         lambda: crop(S.translated_square(129), (129, 65))),
    "hs_texture_pow2": ((256, 128), [400], 0, 0, [0.2], 1,
                        lambda: S.texture_pair(256, seed=3, ny=128)),
    "thirion_pyramid_refine": ((128, 96), [40, 30], 1, 3, [1.0, 0.25, 2.0, 2.0, 5, 0], 2,
                               lambda: S.texture_pair(128, seed=4, ny=96)),
    "diffeomorphic": ((96, 96), [30], 0, 4, [1.0, 2.0, 1.0, 1.0, 5], 1,
                      lambda: (lambda r, m: (r, m * 3.0))(*S.texture_pair(96, seed=8))),
    "elastic_break": ((90, 77), [1000], 0, 2, [0.1, 0.0], 1,
                      lambda: S.texture_pair(90, seed=12, ny=77)),
    "fluid_regrid_pyramid": ((96, 96), [60, 40], 1, 5, [0.25, 0.0, 0.9], 1,
                             lambda: S.shifted_disk(96, shift=(9, 5))),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_logger_errors_bitwise(gpu, oracle, name):
    dims, niter, nscales, reg, params, nrefine, make = CASES[name]
    ref, mov = make()
    g, w = both(oracle, dims, niter, nscales, reg, params, nrefine, ref, mov)
    assert g["iters"] == w["iters"]
    assert np.array_equal(g["motion"], w["motion"])
    assert len(g["errs"]) == len(w["errs"]) > 0
    assert bits(g["errs"]) == bits(w["errs"])


def test_curvature_logger_errors(gpu, oracle):
    """Curvature, two levels, convergence on: iterations equal, errors within
    1e-5 relative (the DCT's fp64 rounding differs from the oracle's naive
    sums; on MI355X the floats have come out equal on every shape tried)."""
    ref, mov = S.texture_pair(96, seed=2)
    g, w = both(oracle, (96, 96), [60, 40], 1, 1, [2.0], 1, ref, mov)
    assert g["iters"] == w["iters"]
    assert np.abs(g["motion"] - w["motion"]).max() <= 1e-5
    assert len(g["errs"]) == len(w["errs"]) > 0
    np.testing.assert_allclose(np.asarray(g["errs"], np.float64),
                               np.asarray(w["errs"], np.float64), rtol=1e-5, atol=0)

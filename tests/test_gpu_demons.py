"""Thirion's and diffeomorphic Demons on the MI355X against the oracle.

Bar: bit-exact motion fields, warped images and iteration counts.  The
Gaussian smoothing is the reference's direct kw x kw convolution with its
linear-index boundary rule (Field.tpp:209-269), staged through LDS in the same
summation order, so no tolerance is needed.
"""
import numpy as np
import pytest

from conftest import golden
from opticalflow2d_amd import ImageRegistration, Of2dError
from opticalflow2d_amd import synthetic as S

pytestmark = pytest.mark.gpu


def both(oracle, dims, niter, nscales, reg, params, nrefine, ref, mov, **opt):
    with ImageRegistration(dims, niter, nscales, reg, params, nrefine, **opt) as r:
        r.register(ref, mov)
        g = dict(motion=r.motion(), warped=r.warp(mov), iters=r.iterations())
    o = oracle.Registration(dims, niter, nscales, reg, params, nrefine, 0,
                            fixed_iters=bool(opt.get("fixed_iters", 0)))
    o.register(ref, mov)
    w = dict(motion=o.motion(), warped=o.warp(mov), iters=o.iterations())
    o.close()
    return g, w


def test_demons_fixtures(gpu):
    g = golden("oracle_paths.npz")
    for name, niter, params in [("demons_texture64", [20], [1.0, 0.25, 2.0, 2.0, 5, 0]),
                                ("demons_add_texture64", [15], [1.0, 0.25, 2.0, 1.0, 3, 1])]:
        with ImageRegistration((64, 64), niter, 0, 3, params, 1) as r:
            r.register(g[f"{name}/ref"], g[f"{name}/mov"])
            assert r.iterations() == g[f"{name}/iters"].tolist(), name
            assert np.array_equal(r.motion(), g[f"{name}/motion"]), name
            assert np.array_equal(r.warp(g[f"{name}/mov"]), g[f"{name}/warped"]), name


@pytest.mark.parametrize("kw,accum", [(5, 0), (7, 0), (4, 1), (1, 0), (3, 2)])
def test_thirion_kernel_widths_and_accumulation(gpu, oracle, kw, accum):
    ref, mov = S.texture_pair(83, seed=kw * 10 + accum, ny=70)
    params = [1.0, 0.25, 1.5, 2.5, kw, accum]
    g, w = both(oracle, (83, 70), [12], 0, 3, params, 1, ref, mov, fixed_iters=1)
    assert g["iters"] == w["iters"]
    assert np.array_equal(g["motion"], w["motion"])
    assert np.array_equal(g["warped"], w["warped"])


@pytest.mark.parametrize("nx,kw,accum,sx", [(321, 5, 0, 0.25), (387, 7, 0, 0.25),
                                             (388, 3, 1, 0.25), (450, 5, 2, 0.25),
                                             (450, 5, 0, 0.3), (387, 7, 1, 0.7)])
def test_thirion_fused_tiles(gpu, oracle, nx, kw, accum, sx):
    """Widths at which the fused force + smoothing + update kernel runs on the
    x-interior tiles and the edge tile columns take the unfused kernels: two
    right edge columns (321: the last tile holds one column, so the tile before
    it also reaches past dimx), one (387, 388, 450), every accumulation mode.
    sigma_x 0.25 squares to a power of two (the kernels multiply by its
    reciprocal); 0.3 and 0.7 do not (they divide)."""
    ref, mov = S.texture_pair(nx, seed=nx + kw, ny=150)
    params = [1.0, sx, 1.5, 2.5, kw, accum]
    g, w = both(oracle, (nx, 150), [6], 0, 3, params, 1, ref, mov, fixed_iters=1)
    assert g["iters"] == w["iters"]
    assert np.array_equal(g["motion"], w["motion"])
    assert np.array_equal(g["warped"], w["warped"])


def test_diffeomorphic_demons_fused_tiles(gpu, oracle):
    """Diffeomorphic Demons on a grid wide enough for the fused update (mode 3:
    the smoothed correction itself, then exp and composition)."""
    ref, mov = S.texture_pair(330, seed=9, ny=120)
    g, w = both(oracle, (330, 120), [5], 0, 4, [1.0, 2.0, 1.0, 1.0, 5], 1, ref, mov * 3.0,
                fixed_iters=1)
    assert g["iters"] == w["iters"]
    assert np.array_equal(g["motion"], w["motion"])


def test_thirion_pyramid_refine(gpu, oracle):
    ref, mov = S.texture_pair(128, seed=4, ny=96)
    g, w = both(oracle, (128, 96), [15, 10], 1, 3, [1.0, 0.25, 2.0, 2.0, 5, 0], 2, ref, mov)
    assert g["iters"] == w["iters"]
    assert np.array_equal(g["motion"], w["motion"])


def test_diffeomorphic_demons(gpu, oracle):
    ref, mov = S.texture_pair(96, seed=8)
    for params in ([1.0, 0.25, 2.0, 2.0, 5], [1.0, 2.0, 1.0, 1.0, 5]):
        # the second set (sigma_x > sigma_i) allows |c| up to 1, i.e. real squarings
        g, w = both(oracle, (96, 96), [10], 0, 4, params, 1, ref, mov * 3.0, fixed_iters=1)
        assert g["iters"] == w["iters"]
        assert np.array_equal(g["motion"], w["motion"]), params


def test_demons_divide_by_zero(gpu):
    """A flat background (grad I = 0 and It = 0) makes Demons.cpp:57 divide by 0."""
    ref, mov = S.translated_square(32)
    with ImageRegistration((32, 32), [5], 0, 3, [1.0, 0.25, 2.0, 2.0, 5, 0]) as r:
        with pytest.raises(Of2dError, match="Divide by zero exception"):
            r.register(ref, mov)


def test_demons_config3_scale_512(gpu, oracle):
    """Config 3 parameters on a 512^2 texture, convergence on."""
    ref, mov = S.texture_pair(512, seed=0)
    g, w = both(oracle, (512, 512), [40], 0, 3, [1.0, 0.25, 2.0, 2.0, 5, 0], 1, ref, mov)
    assert g["iters"] == w["iters"]
    assert np.array_equal(g["motion"], w["motion"])


def test_demons_config3_full_size_4096(gpu, oracle):
    """BASELINE config 3 at its full size (4096^2, its parameters), two fixed
    iterations bit for bit."""
    ref, mov = S.procedural_pair(4096, 0, 4096)
    g, w = both(oracle, (4096, 4096), [2], 0, 3, [1.0, 0.25, 2.0, 2.0, 5, 0], 1, ref, mov,
                fixed_iters=1)
    assert g["iters"] == w["iters"] == [2]
    assert np.array_equal(g["motion"], w["motion"])
    assert np.array_equal(g["warped"], w["warped"])

"""Horn-Schunck on the MI355X through the C-ABI, against the oracle.

Bar: bit-exact motion fields and equal iteration counts (the HIP kernels keep
the reference's fp32 operation order with -ffp-contract=off and IEEE
division).  The default Logger reproduces the reference's sequential fp32
running sums (seqnorm_kernels.hip), so the errors and the printed error lines
are compared bit for bit too.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden
from opticalflow2d_amd import ImageRegistration, OpticalFlow2d, SlabSolver
from opticalflow2d_amd import synthetic as S

pytestmark = pytest.mark.gpu

def bits32(a):
    return np.asarray(a, np.float32).view(np.uint32).tolist()


def oracle_run(oracle, dims, niter, nscales, reg, params, nrefine, ref, mov, verbose=0,
               fixed=False):
    r = oracle.Registration(dims, niter, nscales, reg, params, nrefine, verbose,
                            fixed_iters=fixed)
    r.register(ref, mov)
    out = dict(motion=r.motion(), warped=r.warp(mov), iters=r.iterations(),
               errs=r.last_errors())
    r.close()
    return out


def test_config1_gateway_call_sequence(gpu, oracle):
    """BASELINE config 1 through the MEX-equivalent gateway, in the order of
    test_opticalflow2d.m:42-59: init -> register -> get -> warp -> close."""
    ka = json.load(open(os.path.join(GOLDEN, "reference_known_answers.json")))["hs_square256"]
    ref, mov = S.translated_square(256)
    OpticalFlow2d([256, 256], [200], 0, 0, [0.1], 1, 1, 0)
    try:
        OpticalFlow2d(ref, mov)
        motion = OpticalFlow2d(nargout=1)
        warped = OpticalFlow2d(mov, nargout=1)
    finally:
        OpticalFlow2d()
    assert motion.shape == (256, 256, 2) and warped.shape == (256, 256)
    o = oracle_run(oracle, (256, 256), [200], 0, 0, [0.1], 1, ref, mov)
    assert np.array_equal(motion, o["motion"])
    assert np.array_equal(warped, o["warped"])
    run = ka["runs"][0]
    assert round(float(motion.sum()), 6) == run["sum_motion"]
    assert round(float(np.abs(motion).max()), 6) == run["max_abs_motion"]


def test_early_exit_iteration_count(gpu, oracle):
    ref, mov = S.translated_square(256)
    with ImageRegistration((256, 256), [1000], 0, 0, [0.1]) as r:
        r.register(ref, mov)
        assert r.iterations() == [490]  # reference_known_answers.json
        m = r.motion()
        errs = r.last_errors()
    o = oracle_run(oracle, (256, 256), [1000], 0, 0, [0.1], 1, ref, mov)
    assert np.array_equal(m, o["motion"])
    assert bits32(errs) == bits32(o["errs"])


@pytest.mark.parametrize("chunk", [1, 7, 32])
def test_chunked_speculation_is_exact(gpu, oracle, chunk):
    """The break replay (registration.cpp loop_hs) lands on the same iterate
    whatever the chunk size."""
    ref, mov = S.translated_square(128)
    with ImageRegistration((128, 128), [1000], 0, 0, [0.1], chunk=chunk) as r:
        r.register(ref, mov)
        m, it = r.motion(), r.iterations()
    o = oracle_run(oracle, (128, 128), [1000], 0, 0, [0.1], 1, ref, mov)
    assert it == o["iters"]
    assert np.array_equal(m, o["motion"])


# hs_gradients_from_image: the triple kernel reads the stored gradient field
# dI (0) or derives it from Iaux in the kernel (1; the product does so once dI
# + It exceed the MALL, of2d_device.h hs3_gradients_from_image) — the same bits
GI = [0, 1]


@pytest.mark.parametrize("gi", GI)
@pytest.mark.parametrize("dims", [(37, 23), (129, 65), (255, 130), (64, 300), (3, 3)])
def test_ragged_sizes(gpu, oracle, dims, gi):
    nx, ny = dims
    rng = np.random.default_rng(nx * 1000 + ny)
    ref = rng.random((nx, ny))
    mov = np.roll(ref, 1, axis=0) * 0.9 + 0.05
    with ImageRegistration(dims, [25], 0, 0, [0.3], fixed_iters=1,
                           hs_gradients_from_image=gi) as r:
        r.register(ref, mov)
        m = r.motion()
        w = r.warp(mov)
    o = oracle_run(oracle, dims, [25], 0, 0, [0.3], 1, ref, mov, fixed=True)
    assert np.array_equal(m, o["motion"])
    assert np.array_equal(w, o["warped"])


def _bits(a):
    return np.asarray(a, dtype=np.float32).view(np.uint32)


@pytest.mark.parametrize("gi", GI)
@pytest.mark.parametrize("case", ["blob", "tiny", "static"])
def test_division_paths_bitwise(gpu, oracle, case, gi):
    """The triple Jacobi kernel divides without div_scale where that is exact
    (hs_jacobi_impl.h div2_unscaled: gradients in 0 or [2^-30, 2^20), the
    denominator in [2^-40, 2^40), sc in 0 or [2^-50, 2^30)) and takes the
    compiler's IEEE sequence in every other wave-step.  Both give the oracle's
    bits, signs of zero included.
      blob   It = 0 outside a 20 x 20 blob: the motion at the diffusion front is
             far below 2^-50 (scaled path there, fast path elsewhere);
      tiny   intensities ~1e-12: gradients below 2^-30 (scaled path everywhere);
      static mov == ref: It = 0 and the motion stays 0 (zero numerators)."""
    n = 200
    ref, mov = S.texture_pair(n, seed=3)
    if case == "blob":
        blob = mov.copy()
        mov = ref.copy()
        mov[90:110, 90:110] = blob[90:110, 90:110]
    elif case == "tiny":
        ref, mov = ref * 1e-12, mov * 1e-12
    else:
        mov = ref.copy()
    with ImageRegistration((n, n), [61], 0, 0, [0.3], fixed_iters=1,
                           hs_gradients_from_image=gi) as r:
        r.register(ref, mov)
        m = r.motion()
    o = oracle_run(oracle, (n, n), [61], 0, 0, [0.3], 1, ref, mov, fixed=True)
    assert np.array_equal(_bits(m), _bits(o["motion"]))
    if case == "blob":  # the case does reach the scaled-division range
        a = np.abs(m[m != 0])
        assert a.min() < 2.0 ** -60


def test_pyramid_and_refine_fixture(gpu):
    g = golden("oracle_paths.npz")
    for name, niter, nscales, params, nrefine in [("hs_square64", [60], 0, [0.1], 1),
                                                  ("hs_texture64_pyr", [40, 30], 1, [0.2], 2)]:
        with ImageRegistration((64, 64), niter, nscales, 0, params, nrefine) as r:
            r.register(g[f"{name}/ref"], g[f"{name}/mov"])
            assert r.iterations() == g[f"{name}/iters"].tolist(), name
            assert np.array_equal(r.motion(), g[f"{name}/motion"]), name
            assert np.array_equal(r.warp(g[f"{name}/mov"]), g[f"{name}/warped"]), name


@pytest.mark.parametrize("gi", GI)
def test_texture_three_levels_two_refines(gpu, oracle, gi):
    """Pyramid and refines: Iaux is the warped moving image on every refine
    after the first, so the in-kernel gradients are taken of a warped image."""
    ref, mov = S.texture_pair(200, seed=11, ny=136)
    args = ((200, 136), [30, 25, 20], 2, 0, [0.15], 2)
    with ImageRegistration(*args, hs_gradients_from_image=gi) as r:
        r.register(ref, mov)
        m, it = r.motion(), r.iterations()
    o = oracle_run(oracle, *args, ref, mov)
    assert it == o["iters"]
    assert np.array_equal(m, o["motion"])


def test_warm_start_second_register_call(gpu, oracle):
    """The singleton keeps motion[] across register calls
    (ImageRegistration.cpp:133-156): a second call continues from the first."""
    ref, mov = S.texture_pair(96, seed=5)
    args = ((96, 96), [20, 15], 1, 0, [0.2], 1)
    with ImageRegistration(*args) as r:
        r.register(ref, mov)
        r.register(ref, mov)
        m = r.motion()
    o = oracle.Registration(*args, 0)
    o.register(ref, mov)
    o.register(ref, mov)
    assert np.array_equal(m, o.motion())
    o.close()


def test_verbose_logger_lines(gpu, oracle):
    ref, mov = S.translated_square(64)
    gpu.clear()
    with ImageRegistration((64, 64), [40], 0, 0, [0.1], 1, 1) as r:
        r.register(ref, mov)
    text = "".join(gpu)
    lines = [l for l in text.splitlines() if l.startswith("Iteration:")]
    assert len(lines) == 40
    L = oracle.lib()
    L.oracle_clear_output()
    oracle_run(oracle, (64, 64), [40], 0, 0, [0.1], 1, ref, mov, verbose=1)
    olines = [l for l in L.oracle_captured_output().decode().splitlines()
              if l.startswith("Iteration:")]
    assert lines == olines


def test_divide_by_zero_raises(gpu):
    from opticalflow2d_amd import Of2dError
    flat = np.zeros((32, 32))
    with ImageRegistration((32, 32), [5], 0, 0, [0.0]) as r:
        with pytest.raises(Of2dError, match="Divide by zero exception"):
            r.register(flat, flat)


# ---------------------------------------------------------------- slab path
def test_slab_single_rank_equals_registration(gpu):
    ref, mov = S.texture_pair(256, seed=2)
    with ImageRegistration((256, 256), [300], 0, 0, [0.1]) as r:
        r.register(ref, mov)
        m, it = r.motion(), r.iterations()
    s = SlabSolver(256, 256, 0.1)
    s.set_images(ref, mov)
    assert s.run(300) == it[0]
    assert np.array_equal(s.motion(), m)
    s.close()


def test_time_kernel_leaves_motion_intact(gpu):
    """of2d_slab_time_kernel launches into scratch (include/of2d.h): the last
    run's motion stays readable, and a later run is unchanged by it."""
    ref, mov = S.texture_pair(256, seed=5)
    s = SlabSolver(256, 256, 0.1)
    s.set_images(ref, mov)
    for fixed, niter in ((True, 40), (False, 300)):
        done = s.run(niter, fixed_iters=fixed)
        m = s.motion()
        assert s.time_kernel(7) > 0
        assert np.array_equal(s.motion(), m)
        assert s.run(niter, fixed_iters=fixed) == done
        assert np.array_equal(s.motion(), m)
    s.close()


def test_slab_full_size_4096_bitwise(gpu, oracle):
    """BASELINE config 2 grid (4096^2): a few Jacobi iterations bit for bit
    against the oracle's HS loop on the same gradients."""
    n, iters = 4096, 4
    ref, mov = S.texture_pair(n, seed=0)
    s = SlabSolver(n, n, 0.1)
    s.set_images(ref, mov)
    assert s.run(iters, fixed_iters=True) == iters
    m = s.motion()
    s.close()
    L = oracle.lib()
    I = np.ascontiguousarray(mov.reshape(-1, order="F").astype(np.float32))
    Ir = np.ascontiguousarray(ref.reshape(-1, order="F").astype(np.float32))
    dI = np.zeros(2 * n * n, np.float32)
    It = np.zeros(n * n, np.float32)
    L.oracle_spatial_derivative(I, n, n, dI)
    L.oracle_temporal_derivative(Ir, I, n * n, It)
    u = np.zeros(2 * n * n, np.float32)
    errs = np.zeros(iters, np.float32)
    assert L.oracle_hs_loop(u, dI, It, n, n, 0.1, iters, 1, errs) == iters
    # end of the refine: motion (zero) -> accumulate(motion_est) (ImageRegistrationOpticalFlow.cpp:138)
    motion = np.zeros_like(u)
    L.oracle_accumulate(motion, u, n, n)
    got = np.stack([m[:, :, 0].reshape(-1, order="F"), m[:, :, 1].reshape(-1, order="F")], 1)
    assert np.array_equal(got.astype(np.float32).reshape(-1), motion)


def test_hs_16384_interior_matches_cropped_oracle(gpu, oracle):
    """BASELINE config 5 grid (16384^2) on one GPU.  The oracle cannot run that
    grid in test time, but a Jacobi iteration (and the gradients before it) only
    reaches one pixel further per step, so after k fixed iterations every pixel
    more than k + 2 px from a crop's cut edges equals the oracle run on the crop
    alone (edges shared with the image keep the same border rule)."""
    n, iters, c = 16384, 3, 160
    ref, mov = S.procedural_pair(n, 0, n)
    s = SlabSolver(n, n, 0.1)
    s.set_images(ref, mov)
    assert s.run(iters, fixed_iters=True) == iters
    m = s.motion()
    s.close()
    margin = iters + 2
    for x0, y0 in [(0, 0), (n // 2 - 77, 7001), (n - c, n - c), (0, n - c)]:
        w = oracle_run(oracle, (c, c), [iters], 0, 0, [0.1], 1, ref[x0:x0 + c, y0:y0 + c],
                       mov[x0:x0 + c, y0:y0 + c], fixed=True)["motion"]
        xl, xh = (0 if x0 == 0 else margin), (c if x0 + c == n else c - margin)
        yl, yh = (0 if y0 == 0 else margin), (c if y0 + c == n else c - margin)
        assert np.array_equal(m[x0 + xl:x0 + xh, y0 + yl:y0 + yh], w[xl:xh, yl:yh]), (x0, y0)

"""Viscous fluid and elastic registration on the MI355X against the oracle.

The SOR sweep runs as an exact wavefront of the reference's in-place
Gauss-Seidel order (fluid_kernels.hip), so the bar is bit-exact motion fields,
identical iteration counts and identical printed Dumax / Regridding lines.
"""
import numpy as np
import pytest

from conftest import golden
from opticalflow2d_amd import ImageRegistration
from opticalflow2d_amd import synthetic as S

pytestmark = pytest.mark.gpu


def run_both(gpu, oracle, dims, niter, nscales, reg, params, nrefine, ref, mov, calls=1,
             **opt):
    gpu.clear()
    with ImageRegistration(dims, niter, nscales, reg, params, nrefine, **opt) as r:
        for _ in range(calls):
            r.register(ref, mov)
        g = dict(motion=r.motion(), warped=r.warp(mov), iters=r.iterations())
    gtext = "".join(gpu)
    L = oracle.lib()
    L.oracle_clear_output()
    o = oracle.Registration(dims, niter, nscales, reg, params, nrefine, 0,
                            fixed_iters=bool(opt.get("fixed_iters", 0)))
    for _ in range(calls):
        o.register(ref, mov)
    w = dict(motion=o.motion(), warped=o.warp(mov), iters=o.iterations())
    o.close()
    otext = L.oracle_captured_output().decode()
    return g, w, gtext, otext


def body(text):
    """Printed lines after the banner (Dumax / Regridding / Iteration)."""
    return [l for l in text.splitlines()
            if l.startswith(("Dumax", "Regridding", "Iteration"))]


def test_fluid_and_elastic_fixtures(gpu):
    g = golden("oracle_paths.npz")
    for name, niter, nscales, reg, params in [("fluid_disk64", [30, 30], 1, 5, [0.25, 0.0]),
                                              ("elastic_texture64", [25], 0, 2, [0.5, 0.25])]:
        with ImageRegistration((64, 64), niter, nscales, reg, params, 1) as r:
            r.register(g[f"{name}/ref"], g[f"{name}/mov"])
            assert r.iterations() == g[f"{name}/iters"].tolist(), name
            assert np.array_equal(r.motion(), g[f"{name}/motion"]), name
            assert np.array_equal(r.warp(g[f"{name}/mov"]), g[f"{name}/warped"]), name


@pytest.mark.parametrize("dims", [(70, 37), (130, 50), (64, 64), (125, 300), (5, 4)])
def test_fluid_printed_lines_and_motion(gpu, oracle, dims):
    ref, mov = S.shifted_disk(max(dims))
    ref, mov = ref[: dims[0], : dims[1]], mov[: dims[0], : dims[1]]
    g, w, gt, ot = run_both(gpu, oracle, dims, [20], 0, 5, [0.25, 0.0], 1, ref, mov)
    assert g["iters"] == w["iters"]
    assert np.array_equal(g["motion"], w["motion"])
    assert body(gt) == body(ot)


def test_fluid_regridding_and_warm_start(gpu, oracle):
    """Large shift -> Jacobian drops below 0.5 -> regridding; the velocity field
    persists across register calls (OpticalFlowFluid.cpp:50)."""
    ref, mov = S.shifted_disk(96, shift=(9, 5))
    g, w, gt, ot = run_both(gpu, oracle, (96, 96), [60, 40], 1, 5, [0.25, 0.0, 0.9], 1, ref, mov,
                            calls=2)
    assert g["iters"] == w["iters"]
    assert np.array_equal(g["motion"], w["motion"])
    assert body(gt) == body(ot)


def test_fluid_many_strips_512(gpu, oracle):
    """8 wavefront strips with hand-offs; 3 pyramid levels as in config 4."""
    ref, mov = S.shifted_disk(512)
    g, w, gt, ot = run_both(gpu, oracle, (512, 512), [6, 6, 6], 2, 5, [0.25, 0.0], 1, ref, mov)
    assert g["iters"] == w["iters"]
    assert np.array_equal(g["motion"], w["motion"])
    assert body(gt) == body(ot)


def test_fluid_increment_workers_ragged(gpu, oracle):
    """Levels whose sweep carries the increment workers (fluid_kernels.hip SorInc:
    1000 x 777 -> 16 strips, 400 tiles; 500 x 388 -> 8 strips, 104 tiles): ragged
    last strip and tiles, regridding, two pyramid levels, printed lines."""
    ref, mov = S.shifted_disk(1000, shift=(30, 18))
    ref, mov = ref[:, :777], mov[:, :777]
    g, w, gt, ot = run_both(gpu, oracle, (1000, 777), [14, 10], 1, 5, [0.25, 0.0, 0.9], 1,
                            ref, mov)
    assert g["iters"] == w["iters"]
    assert np.array_equal(g["motion"], w["motion"])
    assert body(gt) == body(ot)
    assert any(l.startswith("Regridding") for l in body(gt))


@pytest.mark.parametrize("chunk", [1, 5, 32])
def test_elastic_chunked_with_break(gpu, oracle, chunk):
    ref, mov = S.texture_pair(90, seed=12, ny=77)
    g, w, _, _ = run_both(gpu, oracle, (90, 77), [1000], 0, 2, [0.1, 0.0], 1, ref, mov,
                          chunk=chunk)
    assert g["iters"] == w["iters"] == [413]
    assert np.array_equal(g["motion"], w["motion"])


def test_elastic_wide_sweep(gpu, oracle):
    """One SOR sweep over 1100 x 300 (18 strips), fixed iterations."""
    ref, mov = S.texture_pair(1100, seed=3, ny=300)
    g, w, _, _ = run_both(gpu, oracle, (1100, 300), [3], 0, 2, [0.3, 0.1], 1, ref, mov,
                          fixed_iters=1)
    assert np.array_equal(g["motion"], w["motion"])


def test_fluid_config4_full_size_8192(gpu, oracle):
    """BASELINE config 4 at its full size: 8192^2, 3-level pyramid, two fixed
    iterations per level (130 wavefront strips at the finest level; the second
    iteration sweeps the force the first one's fused step packed), bit for bit
    with identical printed Dumax lines."""
    ref, mov = S.shifted_disk(8192)
    g, w, gt, ot = run_both(gpu, oracle, (8192, 8192), [2, 2, 2], 2, 5, [0.25, 0.0], 1, ref, mov,
                            fixed_iters=1)
    assert g["iters"] == w["iters"]
    assert np.array_equal(g["motion"], w["motion"])
    assert body(gt) == body(ot)


def test_fluid_timestep_skip_and_integrate(gpu, oracle):
    """A faint difference image (mov = ref + 0.08 (texture shift - ref)) keeps
    maxabs(R) small at first: dt = 0.65 / maxabs >= 65 and the reference skips
    the integration (OpticalFlowFluid.cpp:135-137), so the fused step copies u
    unchanged; later iterations integrate, and some skip again."""
    ref, mov = S.texture_pair(96, seed=5)
    mov = ref + 0.08 * (mov - ref)
    g, w, gt, ot = run_both(gpu, oracle, (96, 96), [25], 0, 5, [0.25, 0.0], 1, ref, mov,
                            fixed_iters=1)
    assert g["iters"] == w["iters"]
    assert np.array_equal(g["motion"], w["motion"])
    assert body(gt) == body(ot)
    dts = [float(l.split("Timestep:")[1]) for l in body(gt) if "Timestep:" in l]
    assert any(t >= 65.0 for t in dts) and any(t < 65.0 for t in dts), dts


@pytest.mark.parametrize("fp64", [0, 1])
@pytest.mark.parametrize("case", ["faint", "mid", "tex"])
def test_fluid_convergence_break_on_device(gpu, oracle, case, fp64):
    """The Fluid loop takes its break and regrid decisions on the device and
    enqueues iterations ahead of the host's read (solvers.cpp loop_fluid):
    texture pairs that converge — 'faint' breaks at iteration 3 with every
    step skipped (dt >= 65), 'mid' at 5 after one regrid, 'tex' at 27 after 11
    regrids — with the reference's float Logger and with fp64 sums, two
    register calls (the velocity and the motion fields carry over), bit for
    bit with the oracle: iterations, motion, warped image, printed lines."""
    ref, mov = S.texture_pair(96, seed=5)
    mov = ref + {"faint": 0.08, "mid": 0.3, "tex": 1.0}[case] * (mov - ref)
    oracle.lib().oracle_set_logger_fp64(fp64)
    try:
        g, w, gt, ot = run_both(gpu, oracle, (96, 96), [60], 0, 5, [0.25, 0.0], 1, ref, mov,
                                calls=2, logger_fp64=fp64)
    finally:
        oracle.lib().oracle_set_logger_fp64(0)
    assert g["iters"] == w["iters"] and g["iters"][0] < 60, (g["iters"], w["iters"])
    assert np.array_equal(g["motion"], w["motion"])
    assert np.array_equal(g["warped"], w["warped"])
    assert body(gt) == body(ot)


def test_fluid_break_and_regrid_pyramid(gpu, oracle):
    """Breaks on two pyramid levels with regrids before them, then a second
    register call: the levels' motion indices and the estimate buffers the
    device decided are the host's state afterwards."""
    ref, mov = S.texture_pair(128, seed=5)
    g, w, gt, ot = run_both(gpu, oracle, (128, 128), [60, 60], 1, 5, [0.25, 0.0, 0.9], 1, ref,
                            mov, calls=2)
    assert g["iters"] == w["iters"], (g["iters"], w["iters"])
    assert np.array_equal(g["motion"], w["motion"])
    assert np.array_equal(g["warped"], w["warped"])
    assert body(gt) == body(ot)

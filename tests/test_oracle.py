"""The oracle (oracle/of2d_oracle.c) pinned against the reference.

* bitwise against the reference's own primitives (src/gradients.h,
  src/coord2d.h, src/Kernel.cpp) — committed fixture tests/golden/ref_prims.npz
  and, where oracle/_ref was built here, live on fresh random inputs;
* end to end against the reference outputs recorded in SURVEY.md §8c / §7
  (tests/golden/reference_known_answers.json);
* against its own committed path fixtures (regression).
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden
from opticalflow2d_amd import synthetic as S


def test_gaussian_kernel_matches_reference_fixture(oracle):
    g = golden("ref_prims.npz")
    for k, (kw, s) in enumerate(g["gauss_cases"]):
        w = np.zeros(int(kw) ** 2)
        oracle.lib().oracle_gaussian_kernel(int(kw), float(s), w)
        assert np.array_equal(w, g[f"gauss_{k}"]), (kw, s)


def test_gradients_qlaplacian_hs_match_reference_fixture(oracle):
    g = golden("ref_prims.npz")
    L = oracle.lib()
    dx, dy = (int(v) for v in g["dims"])
    dI = np.zeros(2 * dx * dy, np.float32)
    L.oracle_spatial_derivative(g["I"], dx, dy, dI)
    assert np.array_equal(dI, g["dI"])
    q = np.zeros_like(g["u"])
    L.oracle_qlaplacian(g["u"], dx, dy, q)
    assert np.array_equal(q, g["q"])
    u = g["u"].copy()
    assert L.oracle_hs_update(u, g["g"], g["It"], dx, dy, float(g["hs_alpha"])) == 0
    assert np.array_equal(u, g["hs"])
    assert L.oracle_motion_norm(g["u"], dx * dy) == g["norm"]
    assert L.oracle_motion_maxabs(g["u"], dx * dy) == g["maxabs"]


def test_motion_partials_match_reference_fixture(oracle):
    """Fluid increment R = v - dudx*v.x - dudy*v.y with v = (1, 0) and (0, 1)
    exposes dudx / dudy of the reference's gradients::partial_x/y on a Motion."""
    g = golden("ref_prims.npz")
    dx, dy = (int(v) for v in g["dims"])
    n = dx * dy
    R = np.zeros(2 * n, np.float32)
    v = np.tile(np.array([1.0, 0.0], np.float32), n)
    oracle.lib().oracle_fluid_increment(g["u"], v, dx, dy, R)
    assert np.array_equal(np.float32(1.0) - g["dudx"][0::2], R[0::2])
    assert np.array_equal(np.float32(0.0) - g["dudx"][1::2], R[1::2])


def test_primitives_live_against_reference_build(oracle):
    R = oracle.ref_lib()
    if R is None:
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    L = oracle.lib()
    rng = np.random.default_rng(99)
    for dx, dy in [(3, 3), (5, 17), (64, 31), (129, 66)]:
        I = rng.random(dx * dy).astype(np.float32)
        a, b = np.zeros(2 * dx * dy, np.float32), np.zeros(2 * dx * dy, np.float32)
        L.oracle_spatial_derivative(I, dx, dy, a)
        R.ref_spatial_derivative(I, dx, dy, b)
        assert np.array_equal(a, b)
        u = (4 * rng.standard_normal(2 * dx * dy)).astype(np.float32)
        L.oracle_qlaplacian(u, dx, dy, a)
        R.ref_qlaplacian(u, dx, dy, b)
        assert np.array_equal(a, b)
        assert L.oracle_motion_norm(u, dx * dy) == R.ref_norm_probe(u, dx * dy)
        assert L.oracle_motion_maxabs(u, dx * dy) == R.ref_maxabs_probe(u, dx * dy)
    out = np.zeros(2, np.float32)
    assert R.ref_coord2d_div(1.0, 2.0, 0.0, out) == 1  # the reference throws


def test_reference_known_answers_hs_square(oracle):
    ka = json.load(open(os.path.join(GOLDEN, "reference_known_answers.json")))["hs_square256"]
    n = ka["dims"][0]
    ref, mov = S.translated_square(n, shift=tuple(ka["shift"]), lo=ka["square"][0],
                                   hi=ka["square"][1])
    for run in ka["runs"]:
        r = oracle.Registration(ka["dims"], run["niter"], ka["nscales"], ka["reg"], ka["params"],
                                ka["nrefine"], 0)
        r.register(ref, mov)
        u = r.motion()
        assert r.iterations() == [run["iterations_executed"]]
        if "sum_motion" in run:
            d = run["decimals"]
            assert round(float(u.sum()), d) == run["sum_motion"]
            assert round(float(np.abs(u).max()), d) == run["max_abs_motion"]
        r.close()


def test_oracle_path_fixtures_regression(oracle):
    from golden.make_golden import PATH_CASES
    g = golden("oracle_paths.npz")
    for name, (kind, n, niter, nscales, reg, params, nrefine) in PATH_CASES.items():
        r = oracle.Registration((n, n), niter, nscales, reg, params, nrefine, 0)
        r.register(g[f"{name}/ref"], g[f"{name}/mov"])
        assert np.array_equal(r.motion(), g[f"{name}/motion"]), name
        assert np.array_equal(r.warp(g[f"{name}/mov"]), g[f"{name}/warped"]), name
        assert r.iterations() == g[f"{name}/iters"].tolist(), name
        r.close()


def test_reference_loop_order_is_result_neutral(oracle):
    ref, mov = S.texture_pair(48, seed=3)
    outs = []
    for order in (0, 1):
        oracle.lib().oracle_set_reference_loop_order(order)
        r = oracle.Registration((48, 48), [12, 10], 1, 3, [1.0, 0.25, 2.0, 2.0, 5, 0], 2, 0)
        r.register(ref, mov)
        outs.append(r.motion())
        r.close()
    oracle.lib().oracle_set_reference_loop_order(0)
    assert np.array_equal(outs[0], outs[1])


def test_divide_by_zero_semantics(oracle):
    """coord2d::operator/ throws (coord2d.h:95-100): HS with alpha = 0 on a
    flat image, Demons on a flat background."""
    n = 32
    flat = np.zeros((n, n))
    r = oracle.Registration((n, n), [5], 0, 0, [0.0], 1, 0)
    with pytest.raises(oracle.OracleError, match="Divide by zero exception"):
        r.register(flat, flat)
    r.close()
    ref, mov = S.translated_square(n)
    r = oracle.Registration((n, n), [5], 0, 3, [1.0, 0.25, 2.0, 2.0, 5, 0], 1, 0)
    with pytest.raises(oracle.OracleError, match="Divide by zero exception"):
        r.register(ref, mov)
    r.close()


def test_invalid_parameters(oracle):
    with pytest.raises(oracle.OracleError, match="Invalid number of regularisation parameters"):
        oracle.Registration((16, 16), [3], 0, 0, [0.1, 0.2], 1, 0)
    with pytest.raises(oracle.OracleError, match="invalid regularisation"):
        oracle.Registration((16, 16), [3], 0, 7, [0.1], 1, 0)


@pytest.mark.parametrize("shape", [(8, 8), (5, 4), (37, 70)])
def test_curvature_dct_matches_r2r_definitions(oracle, shape):
    """The oracle's REDFT10/REDFT01 (Curvature's FFTW plans, OpticalFlowCurvature.cpp:52-55)
    against scipy's unnormalised DCT-II/III, an independent implementation of the
    same published r2r definitions.  FFTW itself is absent, so this pins the
    definitions, not FFTW's rounding."""
    scipy_fft = pytest.importorskip("scipy.fft")
    n0, n1 = shape
    a = np.random.default_rng(n0 * 100 + n1).random(shape)
    for kind, dct_type in ((10, 2), (1, 3)):
        b = np.ascontiguousarray(a.copy())
        oracle.lib().oracle_dct2d(b, n0, n1, kind)
        want = scipy_fft.dct(scipy_fft.dct(a, type=dct_type, axis=1), type=dct_type, axis=0)
        np.testing.assert_allclose(b, want, rtol=1e-12, atol=1e-12 * np.abs(want).max())


def test_hs_loop_mt_motion_equals_single_thread(oracle):
    """bench.py's all-cores CPU baseline (oracle_hs_loop_mt, OpenMP over
    j-lines) computes the same motion bit for bit as the sequential loop: the
    Jacobi update reads only the previous iterate (OpticalFlowDiffusion.cpp:43-55)."""
    from opticalflow2d_amd import synthetic as S
    L = oracle.lib()
    n = 192
    ref, mov = S.procedural_pair(n, 0, n)
    I = np.ascontiguousarray(mov.reshape(-1, order="F").astype(np.float32))
    Ir = np.ascontiguousarray(ref.reshape(-1, order="F").astype(np.float32))
    dI = np.zeros(2 * n * n, np.float32)
    It = np.zeros(n * n, np.float32)
    L.oracle_spatial_derivative(I, n, n, dI)
    L.oracle_temporal_derivative(Ir, I, n * n, It)
    u1, e1 = np.zeros(2 * n * n, np.float32), np.zeros(12, np.float32)
    u2, e2 = np.zeros(2 * n * n, np.float32), np.zeros(12, np.float32)
    L.oracle_hs_loop(u1, dI, It, n, n, 0.1, 12, 1, e1)
    L.oracle_hs_loop_mt(u2, dI, It, n, n, 0.1, 12, 4, e2)
    assert np.array_equal(u1.view(np.uint32), u2.view(np.uint32))
    np.testing.assert_allclose(e2[1:], e1[1:], rtol=1e-4)

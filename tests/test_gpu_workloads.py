"""Each BASELINE.json GPU configuration's FULL benchmarked workload against the
oracle's record of it (tests/golden/workloads.json, made in this container by
tests/golden/make_workloads.py from oracle/of2d_oracle.c).

The other GPU tests compare with the oracle over a few iterations at config
scale; these run every iteration the benchmarks time, on their inputs and
options, and compare SHA-256 digests of the float32 results (bit-exact), the
iteration counts and, for the viscous fluid, every printed Dumax / Regridding
line:
  config 2  bench.py's step: SlabSolver 4096^2, 1000 fixed Jacobi iterations
  config 3  bench_configs.py cfg3: Thirion's Demons 4096^2, 100 iterations
  config 4  bench_configs.py cfg4: viscous fluid 8192^2, 3 levels x 200
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from opticalflow2d_amd import ImageRegistration, SlabSolver
from opticalflow2d_amd import synthetic as S

pytestmark = pytest.mark.gpu

REC = json.load(open(os.path.join(GOLDEN, "workloads.json")))


def digest_planar(m):
    f = np.asarray(m, np.float32)
    planar = np.concatenate([f[:, :, 0].reshape(-1, order="F"), f[:, :, 1].reshape(-1, order="F")])
    return hashlib.sha256(planar.tobytes()).hexdigest()


def digest_image(w):
    return hashlib.sha256(np.asarray(w, np.float32).reshape(-1, order="F").tobytes()).hexdigest()


def body(text):
    return [l for l in text.splitlines() if l.startswith(("Dumax", "Regridding", "Iteration"))]


@pytest.mark.parametrize("gradients", [-1, 1])
def test_config2_bench_workload(gpu, gradients):
    """gradients -1: bench.py's setting (auto: dI read, 4096^2 fits the MALL);
    1: the triple kernel derives dI from Iaux, as every config-5 slab does."""
    r = REC["cfg2"]
    n = r["n"]
    ref, mov = S.procedural_pair(n, 0, n)
    s = SlabSolver(n, n, r["alpha"])
    try:
        s.set_images(ref, mov)
        s.set_option("hs_gradients_from_image", gradients)
        s.reserve(r["niter"])
        assert s.run(r["niter"], fixed_iters=True) == r["niter"]
        assert digest_planar(s.motion()) == r["motion_sha256_f32_planar"]
    finally:
        s.close()


def test_config3_demons_workload(gpu):
    r = REC["cfg3"]
    n = r["n"]
    ref, mov = S.procedural_pair(n, 0, n)
    with ImageRegistration((n, n), r["niter"], 0, 3, r["params"], 1, fixed_iters=1) as g:
        g.register(ref, mov)
        assert g.iterations() == r["iterations"]
        assert digest_planar(g.motion()) == r["motion_sha256_f32_planar"]
        assert digest_image(g.warp(mov)) == r["warped_sha256_f32"]


def test_config4_fluid_workload(gpu):
    """Every iteration's Dumax line (OpticalFlowFluid.cpp:94: the timestep and
    its dt >= 65 skips) and every Regridding line (ImageRegistrationFluid.cpp:110)
    of the 600 iterations, and the final motion."""
    r = REC["cfg4"]
    n = r["n"]
    ref, mov = S.shifted_disk(n)
    gpu.clear()
    with ImageRegistration((n, n), r["niter"], r["nscales"], 5, r["params"], 1,
                           fixed_iters=1) as g:
        g.register(ref, mov)
        it = g.iterations()
        m = g.motion()
        w = g.warp(mov)
    lines = body("".join(gpu))
    assert it == r["iterations"]
    assert len(lines) == r["printed_lines"]
    assert lines[:3] == r["first_lines"]
    assert sum(l.startswith("Regridding") for l in lines) == r["regridding_lines"]
    assert hashlib.sha256("\n".join(lines).encode()).hexdigest() == r["printed_sha256"]
    assert digest_planar(m) == r["motion_sha256_f32_planar"]
    assert digest_image(w) == r["warped_sha256_f32"]

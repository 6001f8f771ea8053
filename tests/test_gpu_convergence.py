"""Default semantics (convergence on) at config scale: the registration stops
where the reference stops — the break test `err < 0.001f && iter > 1`
(ImageRegistrationOpticalFlow.cpp:131-134) on the Logger error
(Logger.cpp:32-51) — and returns the same motion, bit for bit.

Expected values are golden fixtures of the oracle (tests/golden/
make_convergence.py; the oracle is pinned to the reference's known answers in
reference_known_answers.json), so the 4096^2 cases need no CPU run here.  The
top-level records are the reference's semantics (Motion::norm's float running
sums, Motion.cpp:42-49); the "exact_norms" record of each fixture is the
oracle with the Logger norms summed in double (oracle_set_logger_fp64), which
the library's opt-in `logger_fp64` mode follows.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from opticalflow2d_amd import ImageRegistration
from opticalflow2d_amd import synthetic as S

pytestmark = pytest.mark.gpu


def fixture(name):
    return json.load(open(os.path.join(GOLDEN, f"convergence_{name}.json")))


def digest(m):
    f = np.asarray(m, np.float32)
    planar = np.concatenate([f[:, :, 0].reshape(-1, order="F"), f[:, :, 1].reshape(-1, order="F")])
    return hashlib.sha256(planar.tobytes()).hexdigest()


def inputs(fx):
    n = fx["n"]
    if fx["generator"] == "texture_pair":
        return S.texture_pair(n)
    return S.procedural_pair(n, 0, n)


def run(fx, **opts):
    ref, mov = inputs(fx)
    n = fx["n"]
    with ImageRegistration((n, n), fx["niter"], 0, fx["reg"], [fx["alpha"]], **opts) as r:
        r.register(ref, mov)
        return r.iterations(), r.motion(), r.last_errors()


@pytest.mark.parametrize("name", ["hs_texture1024", "hs_texture4096", "hs_procedural4096"])
def test_reference_break_and_motion(gpu, name):
    """The Logger norms are the reference's float running sums (seqnorm), so
    the loop breaks on the reference's iteration at every size:
      1024^2 texture     103
      4096^2 texture     102 (the exactly summed error would break at 107)
      4096^2 procedural  397 (exactly summed: 389)
    Bar: the iteration count, the motion bit for bit, and every iteration's
    error bit for bit (the float32 values of Logger::error)."""
    fx = fixture(name)
    it, m, errs = run(fx)
    assert it == fx["iterations_executed"]
    assert digest(m) == fx["motion_sha256_f32_planar"]
    want = np.asarray(fx["errors"], np.float32)
    assert errs.view(np.uint32).tolist() == want.view(np.uint32).tolist()


# GPU Logger errors in the fp64 mode against the oracle's exactly summed ones
# (fp64 sums of the same magnitudes): the GPU adds fp32 magnitudes per lane
# (<= 72 terms) and fp64 from there on, ~1e-7 relative
EXACT_RTOL = 1e-5


@pytest.mark.parametrize("name", ["hs_texture4096", "hs_procedural4096"])
def test_fp64_logger_mode(gpu, name):
    """Opt-in `logger_fp64`: the fused three-iteration kernels stay on and the
    norms are fp64 sums, so the break falls where the exactly summed error
    crosses 0.001 (107 / 389 at 4096^2).  Bar: that iteration, the oracle's
    motion at it bit for bit, errors within EXACT_RTOL, and a threshold margin
    far outside that tolerance."""
    fx = fixture(name)
    ex = fx["exact_norms"]
    it, m, errs = run(fx, logger_fp64=1)
    assert it == ex["iterations_executed"]
    assert digest(m) == ex["motion_sha256_f32_planar"]
    want = np.asarray(ex["errors"], np.float64)
    np.testing.assert_allclose(np.asarray(errs, np.float64), want, rtol=EXACT_RTOL, atol=0)
    k = it[0] - 1
    assert want[k] < 0.001 <= want[k - 1]
    margin = min(abs(want[k] - 0.001), abs(want[k - 1] - 0.001)) / 0.001
    assert margin > 10 * EXACT_RTOL, margin

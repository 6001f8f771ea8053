"""Multi-device Horn-Schunck through the drop-in boundary (of2d_set_option
"ngpus", the gateway's ninth init argument; opticalflow2d_amd/csrc/ranks.cpp).

By default at most one rank runs per device (ranks beyond the device count
merge: a device's rows in one slab); with "ngpus_share" every rank r runs on
device (device + r) mod count, so on a one-GPU box all of them share device 0,
which exercises the partition, the halo copies, the prediction offsets and
the chained Logger walks exactly as on N devices.  Bar: iterations, motion and
every Logger error bit-identical to the one-rank registration with the
default (reference-exact) Logger; with convergence on, a pyramid and refines
(ImageRegistration.cpp:133-156, ImageRegistrationOpticalFlow.cpp:97-151).
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from opticalflow2d_amd import ImageRegistration, OpticalFlow2d
from opticalflow2d_amd import synthetic as S

pytestmark = pytest.mark.gpu


def run(dims, niter, nscales, params, nrefine, ref, mov, **opts):
    with ImageRegistration(dims, niter, nscales, 0, params, nrefine, **opts) as r:
        r.register(ref, mov)
        return r.iterations(), r.motion(), r.last_errors(), r.warp(mov)


@pytest.mark.parametrize("ngpus", [2, 3, 8])
def test_pyramid_refines_convergence_bitwise(gpu, ngpus):
    ref, mov = S.texture_pair(256, seed=4, ny=200)
    args = ((256, 200), [300, 200, 200], 2, [0.1], 2, ref, mov)
    it1, m1, e1, w1 = run(*args)
    itn, mn, en, wn = run(*args, ngpus=ngpus, ngpus_share=1)
    assert itn == it1
    assert np.array_equal(mn, m1)
    assert np.array_equal(wn, w1)
    assert en.view(np.uint32).tolist() == e1.view(np.uint32).tolist()


@pytest.mark.parametrize("dims,ngpus", [((129, 67), 4), ((37, 23), 7), ((300, 9), 3)])
def test_ragged_fixed_iterations(gpu, dims, ngpus):
    rng = np.random.default_rng(dims[0])
    ref = rng.random(dims)
    mov = np.roll(ref, 1, axis=0) * 0.9 + 0.05
    a = run(dims, [25], 0, [0.3], 1, ref, mov, fixed_iters=1)
    b = run(dims, [25], 0, [0.3], 1, ref, mov, fixed_iters=1, ngpus=ngpus, ngpus_share=1)
    assert np.array_equal(a[1], b[1])


@pytest.mark.parametrize("opts", [{"fixed_iters": 1}, {"logger_fp64": 1}])
def test_ranks_split_launches(gpu, opts):
    """The ranks' triples as interior + edge launches (option "slab_split" = 1:
    the launch order of ranks on distinct devices) on 2 and 4 ranks sharing
    device 0, with a pyramid whose coarse levels are too short to split:
    iterations and motion bit-identical to one rank."""
    ref, mov = S.texture_pair(256, seed=11, ny=400)
    args = ((256, 400), [150, 100], 1, [0.1], 2, ref, mov)
    a = run(*args, **opts)
    for n in (2, 4):
        b = run(*args, ngpus=n, ngpus_share=1, slab_split=1, **opts)
        assert b[0] == a[0]
        assert np.array_equal(b[1], a[1])
        assert np.array_equal(b[3], a[3])


def test_fp64_logger_mode_motion(gpu):
    """logger_fp64: per-rank partial sums added in rank order — the errors
    differ from one rank's in the last bits, the iterates do not."""
    ref, mov = S.texture_pair(192, seed=8)
    a = run((192, 192), [400], 0, [0.1], 1, ref, mov, logger_fp64=1)
    b = run((192, 192), [400], 0, [0.1], 1, ref, mov, logger_fp64=1, ngpus=3, ngpus_share=1)
    assert a[0] == b[0]
    assert np.array_equal(a[1], b[1])
    np.testing.assert_allclose(b[2], a[2], rtol=1e-5)


def test_gateway_ninth_argument(gpu):
    """The MEX init with ngpus as a ninth input (WrapperOpticalFlow2d.cpp's
    eight plus this library's) gives the eight-argument result."""
    ref, mov = S.texture_pair(128, seed=2)
    out = []
    for extra in ([], [4]):
        OpticalFlow2d([128, 128], [500], 0, 0, [0.1], 1, 1, 0, *extra)
        try:
            OpticalFlow2d(ref, mov)
            out.append(OpticalFlow2d(nargout=1))
        finally:
            OpticalFlow2d()
    assert np.array_equal(out[0], out[1])


def test_config_scale_reference_break_8_ranks(gpu):
    """4096^2 texture pair on 8 ranks: the reference's break (102) and motion
    (tests/golden/convergence_hs_texture4096.json)."""
    fx = json.load(open(os.path.join(GOLDEN, "convergence_hs_texture4096.json")))
    ref, mov = S.texture_pair(4096)
    it, m, e, _ = run((4096, 4096), fx["niter"], 0, [fx["alpha"]], 1, ref, mov, ngpus=8,
                      ngpus_share=1)
    assert it == fx["iterations_executed"]
    f = np.asarray(m, np.float32)
    planar = np.concatenate([f[:, :, 0].reshape(-1, order="F"), f[:, :, 1].reshape(-1, order="F")])
    assert hashlib.sha256(planar.tobytes()).hexdigest() == fx["motion_sha256_f32_planar"]
    assert e.view(np.uint32).tolist() == np.asarray(fx["errors"], np.float32).view(np.uint32).tolist()


def test_ranks_on_distinct_devices(gpu):
    """With two or more devices the ranks sit on different ones ((device + r)
    mod count): the halo copies, the chained Logger's reads of the neighbour's
    memory and the fp64 mode's sums go between devices (peer access enabled
    for every pair used).  Four ranks, so some pairs are not neighbours.
    Skipped on a one-GPU box."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("one device")
    ref, mov = S.texture_pair(256, seed=6, ny=200)
    args = ((256, 200), [300], 0, [0.1], 1, ref, mov)
    for opts in ({}, {"logger_fp64": 1}, {"fixed_iters": 1}):
        a = run(*args, **opts)
        b = run(*args, ngpus=4, ngpus_share=1, **opts)
        assert a[0] == b[0]
        assert np.array_equal(a[1], b[1])


def test_ranks_beyond_devices_merge(gpu):
    """Default: ngpus above the device count runs one slab per device (on a
    one-GPU box the one-device loop), the same bits either way."""
    import torch
    ref, mov = S.texture_pair(256, seed=9, ny=200)
    args = ((256, 200), [300], 0, [0.1], 1, ref, mov)
    a = run(*args)
    b = run(*args, ngpus=torch.cuda.device_count() + 3)
    c = run(*args, ngpus=torch.cuda.device_count() + 3, ngpus_share=1)
    for x in (b, c):
        assert x[0] == a[0]
        assert np.array_equal(x[1], a[1])
        assert x[2].view(np.uint32).tolist() == a[2].view(np.uint32).tolist()

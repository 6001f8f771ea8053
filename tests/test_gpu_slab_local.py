"""The row-slab decomposition (opticalflow2d_amd/csrc/slab.cpp) on ONE GPU.

RCCL refuses two ranks on one device, so the multi-rank path runs here as an
in-process slab group (``of2d_slab_group``): N slabs of one grid, one host
thread per rank, the same launches and halo lines as over RCCL, moved by device
copies.  This checks the slab code itself — halo offsets, the K-line exchange
before every fused launch, the band split that overlaps it, the global row
index of the border rule, the halo rows of the gradients, the per-chunk
all-reduce of the Logger sums and the break replay — where the gloo tests
(test_dist_gloo.py) check the protocol on a numpy model.

Bar: the assembled motion bit-identical to the one-rank run of the same grid
(itself bit-identical to ImageRegistration and the oracle, test_gpu_hs.py) and
the same iteration count.
"""
import threading

import numpy as np
import pytest

from opticalflow2d_amd import SlabGroup, SlabSolver
from opticalflow2d_amd import synthetic as S
from opticalflow2d_amd.slab import halo_rows

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.asarray(a, dtype=np.float32).view(np.uint32)


def run_group(ref, mov, alpha, nranks, niter, fixed, gi=-1, fp64=0, errors=False):
    dimx, dimy = ref.shape
    g = SlabGroup(nranks)
    slabs = [SlabSolver(dimx, dimy, alpha, r, nranks, group=g) for r in range(nranks)]
    try:
        for s in slabs:
            s.set_option("hs_gradients_from_image", gi)
            s.set_option("logger_fp64", fp64)
            lo, hi = halo_rows(dimy, s.rank, nranks)
            s.set_images(ref[:, lo:hi], mov[:, lo:hi])
        done, errs = [None] * nranks, [None] * nranks

        def work(r):
            try:
                done[r] = slabs[r].run(niter, fixed_iters=fixed)
            except Exception as e:  # reported below
                errs[r] = e

        th = [threading.Thread(target=work, args=(r,)) for r in range(nranks)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=180)
        assert not any(t.is_alive() for t in th), "a rank did not finish"
        assert errs == [None] * nranks, errs
        m = np.concatenate([s.motion() for s in slabs], axis=1)
        if errors:
            errs = [s.errors() for s in slabs]
            assert all(np.array_equal(e.view(np.uint32), errs[0].view(np.uint32)) for e in errs)
            return m, done, errs[0]
        return m, done
    finally:
        for s in slabs:
            s.close()
        g.close()


def run_single(ref, mov, alpha, niter, fixed, fp64=0):
    dimx, dimy = ref.shape
    s = SlabSolver(dimx, dimy, alpha)
    try:
        s.set_option("logger_fp64", fp64)
        s.set_images(ref, mov)
        it = s.run(niter, fixed_iters=fixed)
        return s.motion(), it
    finally:
        s.close()


@pytest.mark.parametrize("dimx,dimy,nranks,niter", [
    (256, 256, 2, 100),   # 33-iteration chunks: triples, then a single
    (200, 301, 3, 40),    # ragged grid, slabs of 101 / 100 / 100 j-lines
    (256, 600, 2, 70),    # 300 j-lines per slab: the exchange overlaps interior bands
    (130, 97, 4, 35),     # 24-25 j-lines per slab: one band, exchange then launch
    (256, 512, 8, 50),    # eight ranks
    (64, 12, 4, 20),      # three j-lines per slab, the minimum
])
@pytest.mark.parametrize("gi", [0, 1])
def test_slab_group_fixed_iterations_bitwise(gpu, dimx, dimy, nranks, niter, gi):
    """gi = 1: the triple kernel derives the gradients of the halo rows from the
    image halo rows the slab took at set_images (three j-lines each side)."""
    ref, mov = S.texture_pair(dimx, seed=5, ny=dimy)
    m1, it1 = run_single(ref, mov, 0.1, niter, True)
    mN, itN = run_group(ref, mov, 0.1, nranks, niter, True, gi)
    assert it1 == niter and itN == [niter] * nranks
    assert np.abs(m1).max() > 0.01  # the motion has crossed the slab seams
    assert np.array_equal(_bits(mN), _bits(m1))


@pytest.mark.parametrize("fp64", [0, 1])
@pytest.mark.parametrize("nranks", [2, 3])
def test_slab_group_break_replay(gpu, nranks, fp64):
    """Convergence on: every rank sees the global Logger sums (fp64 = 0: the
    last rank's chained float running sums; 1: the all-reduced fp64 sums),
    breaks at the same iteration and replays single steps (with their one-line
    exchanges) from the chunk's start buffer."""
    ref, mov = S.texture_pair(192, seed=7)
    m1, it1 = run_single(ref, mov, 0.1, 1000, False, fp64)
    assert it1 < 1000
    mN, itN = run_group(ref, mov, 0.1, nranks, 1000, False, fp64=fp64)
    assert itN == [it1] * nranks
    assert np.array_equal(_bits(mN), _bits(m1))


@pytest.mark.parametrize("nranks", [1, 2, 3, 8])
def test_slab_group_reference_logger_4096(gpu, nranks):
    """The reference's Logger across slabs: one float running sum in linear
    order, chained through the ranks' walks (Motion.cpp:42-49), so the slab
    group breaks where the one-grid reference does.  Bar: the 4096^2 texture
    fixture (tests/golden/convergence_hs_texture4096.json, the oracle's record
    of the reference semantics): 102 iterations, the motion's sha256 and every
    iteration's error bit for bit, on 1, 2, 3 and 8 slabs."""
    import json
    import hashlib
    import os
    from conftest import GOLDEN
    fx = json.load(open(os.path.join(GOLDEN, "convergence_hs_texture4096.json")))
    ref, mov = S.texture_pair(fx["n"])
    m, done, errs = run_group(ref, mov, fx["alpha"], nranks, fx["niter"][0], False,
                              errors=True)
    assert done == fx["iterations_executed"] * nranks
    f = np.asarray(m, np.float32)
    planar = np.concatenate([f[:, :, 0].reshape(-1, order="F"),
                             f[:, :, 1].reshape(-1, order="F")])
    assert hashlib.sha256(planar.tobytes()).hexdigest() == fx["motion_sha256_f32_planar"]
    want = np.asarray(fx["errors"], np.float32)
    assert errs.view(np.uint32).tolist() == want.view(np.uint32).tolist()

"""The row-slab decomposition (opticalflow2d_amd/csrc/slab.cpp) on ONE GPU.

RCCL refuses two ranks on one device, so the multi-rank path runs here as an
in-process slab group (``of2d_slab_group``): N slabs of one grid, one host
thread per rank, the same launches and halo lines as over RCCL, moved by device
copies.  This checks the slab code itself — halo offsets, the K-line exchange
before every fused launch, the global row index of the border rule, the halo
rows of the gradients, the per-chunk all-reduce of the Logger sums and the
break replay — where the gloo tests (test_dist_gloo.py) check the protocol on
a numpy model.

Slabs whose neighbours share their device run whole triples (slab_geometry:
the split only pays when the exchange crosses devices).  The launch order that
ranks on distinct devices and RCCL ranks run — each triple as an interior
launch on the compute stream beside the exchange and two 16-line edge launches
on the comm stream, ordered by the ev_int / ev_edge events — is forced here
with the slab option "split" = 1 (asserted through info()["split"]).

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


def can_split(dimy, nranks):
    """Every slab has >= 48 j-lines (two 16-line edges and an interior)."""
    return nranks > 1 and dimy // nranks >= 48


def run_group(ref, mov, alpha, nranks, niter, fixed, gi=-1, fp64=0, errors=False, split=-1):
    dimx, dimy = ref.shape
    g = SlabGroup(nranks)
    slabs = [SlabSolver(dimx, dimy, alpha, r, nranks, group=g) for r in range(nranks)]
    try:
        for s in slabs:
            s.set_option("hs_gradients_from_image", gi)
            s.set_option("logger_fp64", fp64)
            s.set_option("split", split)
            lo, hi = halo_rows(dimy, s.rank, nranks)
            s.set_images(ref[:, lo:hi], mov[:, lo:hi])
        # co-located slabs run unsplit unless the split is forced
        want = 1 if (split == 1 and can_split(dimy, nranks)) else 0
        assert [s.info()["split"] for s in slabs] == [want] * nranks
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
    (256, 600, 2, 70),    # 300 j-lines per slab: split, several interior bands
    (130, 97, 4, 35),     # 24-25 j-lines per slab: too short to split
    (256, 512, 8, 50),    # eight ranks (64 j-lines: split with a 32-line interior)
    (64, 12, 4, 20),      # three j-lines per slab, the minimum
])
@pytest.mark.parametrize("gi", [0, 1])
@pytest.mark.parametrize("split", [-1, 1])
def test_slab_group_fixed_iterations_bitwise(gpu, dimx, dimy, nranks, niter, gi, split):
    """gi = 1: the triple kernel derives the gradients of the halo rows from the
    image halo rows the slab took at set_images (three j-lines each side).
    split = 1: the interior / edge launches of ranks on distinct devices."""
    ref, mov = S.texture_pair(dimx, seed=5, ny=dimy)
    m1, it1 = run_single(ref, mov, 0.1, niter, True)
    mN, itN = run_group(ref, mov, 0.1, nranks, niter, True, gi, split=split)
    assert it1 == niter and itN == [niter] * nranks
    assert np.abs(m1).max() > 0.01  # the motion has crossed the slab seams
    assert np.array_equal(_bits(mN), _bits(m1))


@pytest.mark.parametrize("fp64,split", [(0, -1), (1, -1), (1, 1)])
@pytest.mark.parametrize("nranks", [2, 3])
def test_slab_group_break_replay(gpu, nranks, fp64, split):
    """Convergence on: every rank sees the global Logger sums (fp64 = 0: the
    last rank's chained float running sums; 1: the all-reduced fp64 sums),
    breaks at the same iteration and replays single steps (with their one-line
    exchanges) from the chunk's start buffer.  With fp64 = 1 the chunks' triples
    run split when forced (the reference-exact loop stores every iterate and
    runs whole triples)."""
    ref, mov = S.texture_pair(192, seed=7)
    m1, it1 = run_single(ref, mov, 0.1, 1000, False, fp64)
    assert it1 < 1000
    mN, itN = run_group(ref, mov, 0.1, nranks, 1000, False, fp64=fp64, split=split)
    assert itN == [it1] * nranks
    assert np.array_equal(_bits(mN), _bits(m1))


@pytest.fixture(scope="module")
def pair16384():
    return S.procedural_pair(16384, 0, 16384)


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_config5_split_slabs_16384(gpu, pair16384, nranks):
    """BASELINE config 5's grid (16384^2) as 2, 4 and 8 split in-process slabs:
    30 fixed iterations bit-identical to the one-rank SlabSolver (itself
    crop-pinned to the oracle at this size, test_gpu_hs.py::
    test_hs_16384_interior_matches_cropped_oracle).  The slabs' triples take
    the gradients from the image (past the MALL) and run as interior + edge
    launches, the order the driver's 8-GPU RCCL run executes."""
    ref, mov = pair16384
    n, niter = 16384, 30
    one = SlabSolver(n, n, 0.1)
    try:
        one.set_images(ref, mov)
        assert one.run(niter, fixed_iters=True) == niter
        want = _bits(one.motion())
    finally:
        one.close()
    g = SlabGroup(nranks)
    slabs = [SlabSolver(n, n, 0.1, r, nranks, group=g) for r in range(nranks)]
    try:
        for s in slabs:
            s.set_option("split", 1)
            lo, hi = halo_rows(n, s.rank, nranks)
            s.set_images(ref[:, lo:hi], mov[:, lo:hi])
            info = s.info()
            assert info["split"] == 1 and info["gradients_from_image"] == 1
        done, errs = [None] * nranks, [None] * nranks

        def work(r):
            try:
                done[r] = slabs[r].run(niter, fixed_iters=True)
            except Exception as e:  # reported below
                errs[r] = e

        th = [threading.Thread(target=work, args=(r,)) for r in range(nranks)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=180)
        assert not any(t.is_alive() for t in th), "a rank did not finish"
        assert errs == [None] * nranks, errs
        assert done == [niter] * nranks
        for s in slabs:
            got = _bits(s.motion())
            assert np.array_equal(got, want[:, s.row_begin:s.row_end]), s.rank
    finally:
        for s in slabs:
            s.close()
        g.close()


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

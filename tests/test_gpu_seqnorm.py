"""The Logger's norms on the MI355X, bit for bit against the reference's
float running sum (src/Motion.cpp:42-49 as Logger::update_error takes it,
src/Logger.cpp:32-51): of2d_motion_norms against oracle_motion_norm_sum.

Bar: the float32 bit patterns of both sums equal.  Cases cover the walk's
branches: ragged tiles and odd widths, a leading run of zero magnitudes (the
sum stays 0 across tiles), magnitudes that tie on every term once the sum's
ulp is 2 (a constant field of unit vectors past 2^24 terms), sums past 2^24
terms where the float sum saturates far below the exact one, tiny magnitudes
(the sum starts below 2^-100), NaN and infinite magnitudes.
"""
import numpy as np
import pytest

from opticalflow2d_amd.registration import motion_norms

pytestmark = pytest.mark.gpu


def oracle_sums(oracle, cur, prev):
    L = oracle.lib()
    n = cur.size // 2
    diff = np.ascontiguousarray((cur - prev).astype(np.float32).reshape(-1))
    p = np.ascontiguousarray(prev.astype(np.float32).reshape(-1))
    return np.array([L.oracle_motion_norm_sum(diff, n), L.oracle_motion_norm_sum(p, n)],
                     np.float32)


def check(oracle, cur, prev, dims):
    cur = np.asarray(cur, np.float32).reshape(-1, 2)
    prev = np.asarray(prev, np.float32).reshape(-1, 2)
    got, res = motion_norms(cur, prev, dims)
    want = oracle_sums(oracle, cur, prev)
    nan = np.isnan(want)
    assert np.array_equal(np.isnan(got), nan), (got, want)  # NaN payloads may differ
    assert got[~nan].view(np.uint32).tolist() == want[~nan].view(np.uint32).tolist(), \
        (got, want, res)
    return res


@pytest.mark.parametrize("dims", [(1, 1), (3, 5), (7, 1), (1, 9), (64, 64), (255, 257),
                                  (4096, 1), (1000, 1000), (1024, 4097)])
def test_random_fields(gpu, oracle, dims):
    rng = np.random.default_rng(sum(dims))
    n = dims[0] * dims[1]
    prev = rng.normal(0, 1.5, (n, 2)).astype(np.float32)
    cur = prev + rng.normal(0, 1e-3, (n, 2)).astype(np.float32)
    check(oracle, cur, prev, dims)


def test_config_scale_4096(gpu, oracle):
    """16.7 M terms: the float sum drifts a few % from the exact one."""
    rng = np.random.default_rng(7)
    n = 4096 * 4096
    prev = rng.normal(0, 1.0, (n, 2)).astype(np.float32)
    cur = prev * np.float32(1.001) + rng.normal(0, 1e-4, (n, 2)).astype(np.float32)
    res = check(oracle, cur, prev, (4096, 4096))
    # a cost figure, not a result: the prediction should leave few tiles to resolve
    assert res[:2].max() < 200, res


def test_past_2_24_terms_saturates(gpu, oracle):
    """5000 x 4000 terms of magnitude ~1: past 2^24 the float sum's ulp
    exceeds the terms and the reference's sum stalls."""
    rng = np.random.default_rng(3)
    n = 5000 * 4000
    prev = rng.uniform(0.5, 1.5, (n, 2)).astype(np.float32)
    cur = prev + rng.uniform(-1e-2, 1e-2, (n, 2)).astype(np.float32)
    check(oracle, cur, prev, (5000, 4000))


def test_ties_every_term(gpu, oracle):
    """|(1, 0)| = 1 on every pixel: from S = 2^24 on each addition is an exact
    tie (half an ulp), rounded to even."""
    n = 4500 * 4000
    prev = np.zeros((n, 2), np.float32)
    prev[:, 0] = 1.0
    cur = prev.copy()
    cur[::3, 1] = 0.75
    check(oracle, cur, prev, (4500, 4000))


@pytest.mark.parametrize("base", [1.5, 0.75])
def test_near_half_ulps(gpu, oracle, base):
    """Magnitudes within a few float ulps of a half-ulp of the running sum:
    |(base, y)| with y in [0, 2^-8] is base + [0, 2^-17.6], so d / ulp(S)
    lies just above a half-integer by less than, about and more than the
    fp32 estimate's decision margin (seqnorm_kernels.hip sn_incr_est): both
    the estimate and the exact fp64 sequence decide terms there, with ties
    (y = 0) and the 2^23 / 2^24 binades of S among them."""
    rng = np.random.default_rng(31 if base == 1.5 else 32)
    dims = (4096, 4096)
    n = dims[0] * dims[1]
    prev = np.zeros((n, 2), np.float32)
    prev[:, 0] = np.float32(base)
    prev[:, 0] -= rng.integers(0, 3, n).astype(np.float32) * np.float32(2.0 ** -23)
    prev[:, 1] = rng.uniform(0, 2.0 ** -8, n).astype(np.float32)
    prev[rng.random(n) < 0.1, 1] = 0.0
    cur = np.zeros_like(prev)
    cur[:, 0] = prev[:, 0] * np.float32(2.0)
    cur[:, 1] = prev[:, 1] * np.float32(3.0)
    check(oracle, cur, prev, dims)


@pytest.mark.parametrize("sigma", [2.0, 4.0])
def test_heavy_tailed_magnitudes(gpu, oracle, sigma):
    """Lognormal magnitudes: terms from far below half an ulp of the running
    sum to thousands of ulps (t = d / ulp(S) up to and past 2^13 and 2^18,
    where the fp32 estimate's margin shrinks and then vanishes), so both the
    estimate and the exact fp64 sequence decide many terms of every tile."""
    rng = np.random.default_rng(int(sigma * 10))
    dims = (2048, 1500)
    n = dims[0] * dims[1]
    mag = rng.lognormal(0.0, sigma, n).astype(np.float32)
    ang = rng.uniform(0, 2 * np.pi, n)
    prev = np.stack([mag * np.cos(ang), mag * np.sin(ang)], -1).astype(np.float32)
    cur = prev + (rng.lognormal(-3.0, sigma, (n, 1)) * rng.normal(0, 1, (n, 2))).astype(np.float32)
    check(oracle, cur, prev, dims)


def test_leading_zeros_and_tiny(gpu, oracle):
    rng = np.random.default_rng(11)
    dims = (3000, 200)
    n = dims[0] * dims[1]
    prev = rng.normal(0, 1, (n, 2)).astype(np.float32)
    prev[: 50 * 3000] = 0.0          # 37 zero tiles before anything
    prev[50 * 3000: 50 * 3000 + 7] = np.float32(1e-38)  # sum below 2^-100, then tiny steps
    prev[50 * 3000 + 7: 50 * 3000 + 9] = np.float32(1e-45)  # denormal components
    cur = prev.copy()
    cur[: 60 * 3000] = 0.0
    check(oracle, cur, prev, dims)


def test_all_zero(gpu, oracle):
    z = np.zeros((640 * 480, 2), np.float32)
    check(oracle, z, z, (640, 480))


@pytest.mark.parametrize("special", ["nan", "inf", "overflow"])
def test_nonfinite(gpu, oracle, special):
    rng = np.random.default_rng(5)
    dims = (2048, 300)
    n = dims[0] * dims[1]
    prev = rng.normal(0, 1, (n, 2)).astype(np.float32)
    cur = prev + np.float32(0.01)
    k = n // 3
    if special == "nan":
        prev[k, 1] = np.nan
    elif special == "inf":
        cur[k, 0] = np.inf
        prev[2 * k, 0] = np.inf
    else:  # magnitudes near FLT_MAX: the float sum overflows to inf
        prev[k: k + 5] = np.float32(3e38)
    check(oracle, cur, prev, dims)


def check_seq(oracle, curs, prevs, dims):
    curs = np.asarray(curs, np.float32)
    prevs = np.asarray(prevs, np.float32)
    got, res = motion_norms(curs, prevs, dims)
    for k in range(curs.shape[0]):
        want = oracle_sums(oracle, curs[k], prevs[k])
        assert got[k].view(np.uint32).tolist() == want.view(np.uint32).tolist(), (k, got[k], want)
    return res


def test_logger_sequence_profile(gpu, oracle):
    """A Logger loop's updates on one workspace: u_k converging, prev of the
    first update zero (Logger.cpp:13).  Each walk predicts the next."""
    rng = np.random.default_rng(21)
    dims = (1024, 1030)
    n = dims[0] * dims[1]
    u = [np.zeros((n, 2), np.float32)]
    step = rng.normal(0, 1.0, (n, 2)).astype(np.float32)
    for k in range(6):
        u.append((u[-1] + step * np.float32(0.5 ** k)).astype(np.float32))
    res = check_seq(oracle, u[1:], u[:-1], dims)
    # cost figures, not results: the walk resolves the tiles a profile missed
    # itself (|prev| grows 1.5x, then 1.17x: the trend of the totals
    # overshoots once), and a walk that resolved many tiles sends the next
    # call through the fp64 check, so the later updates resolve little more
    # than their crossings
    assert res[:, :2].max() < 120, res
    assert res[4:, :2].max() < 40, res


def test_profile_misprediction(gpu, oracle):
    """Consecutive pairs whose sums differ by 2^20: every tile's predicted
    binades miss, the fp64 check marks them pending, the result stays exact."""
    rng = np.random.default_rng(22)
    dims = (700, 900)
    n = dims[0] * dims[1]
    curs, prevs = [], []
    for scale in (1.0, 2.0 ** 20, 2.0 ** -20, 1.0):
        p = (rng.normal(0, 1, (n, 2)) * scale).astype(np.float32)
        curs.append(p + (rng.normal(0, 1e-3, (n, 2)) * scale).astype(np.float32))
        prevs.append(p)
    check_seq(oracle, curs, prevs, dims)


def hs_like_chain(dims, niter, seed):
    """u_k = A (1 - 0.8^k) + noise: smooth fields converging geometrically, as
    a registration loop's iterates do (|u_k - u_{k-1}| shrinks each update)."""
    rng = np.random.default_rng(seed)
    dimx, dimy = dims
    x = np.arange(dimx, dtype=np.float32)[None, :] / dimx
    y = np.arange(dimy, dtype=np.float32)[:, None] / dimy
    A = np.stack([1.5 * np.sin(6.3 * x + 2.0 * y) + 0.4 * np.cos(17.0 * y),
                  1.2 * np.cos(5.1 * y - 3.0 * x) + 0.3 * np.sin(23.0 * x)], -1)
    A = A.astype(np.float32).reshape(-1, 2)
    u = np.zeros((niter + 1, dimx * dimy, 2), np.float32)
    for k in range(1, niter + 1):
        w = np.float32(1.0 - 0.8 ** k)
        u[k] = A * w + rng.normal(0, 1e-3, A.shape).astype(np.float32)
    return u


@pytest.mark.parametrize("batch", [1, 2, 3])
@pytest.mark.parametrize("dims,niter", [((4096, 4096), 7), ((1000, 1003), 8), ((37, 5), 4)])
def test_batched_chain(gpu, oracle, batch, dims, niter):
    """The registration loop's batches (one pass over K + 1 iterates for K
    updates, the check / fix / walk of the K updates in one launch each, two
    workspace sets predicting each other's successors): every update's sums
    bit for bit, ragged last batches included."""
    from opticalflow2d_amd.registration import motion_norms_chain
    u = hs_like_chain(dims, niter, 40 + batch)
    got, res = motion_norms_chain(u, dims, batch)
    for k in range(niter):
        want = oracle_sums(oracle, u[k + 1], u[k])
        assert got[k].view(np.uint32).tolist() == want.view(np.uint32).tolist(), (k, got[k], want)
    if dims == (4096, 4096):
        # a cost figure, not a result: predicted updates resolve few tiles
        assert res[2:, :2].max() < 200, res

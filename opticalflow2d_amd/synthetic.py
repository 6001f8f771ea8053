"""Synthetic image pairs for parity tests and benchmarks.

There is no network and the reference's demo images (DIR-Lab TIFFs,
test_opticalflow2d.m:8-9) are not in the repository, so every workload is a
deterministic synthetic pair.  Arrays are [dimx, dimy] float64 in the
reference's convention (x first).
"""
from __future__ import annotations

import numpy as np


def translated_square(n: int = 256, shift=(2, 1), lo: int | None = None, hi: int | None = None):
    """Config 1: ref = 1 on [n/4, 3n/4)^2, else 0; mov = the square shifted by
    (+2, +1) px (x, y)."""
    lo = n // 4 if lo is None else lo
    hi = 3 * n // 4 if hi is None else hi
    ref = np.zeros((n, n))
    ref[lo:hi, lo:hi] = 1.0
    mov = np.zeros((n, n))
    sx, sy = shift
    mov[lo + sx:hi + sx, lo + sy:hi + sy] = 1.0
    return ref, mov


def _blur(a: np.ndarray, sigma: float) -> np.ndarray:
    """Separable Gaussian (reflect borders) in float64, numpy only."""
    r = int(np.ceil(4 * sigma))
    x = np.arange(-r, r + 1, dtype=np.float64)
    k = np.exp(-0.5 * (x / sigma) ** 2)
    k /= k.sum()
    out = a
    for axis in (0, 1):
        pad = [(0, 0), (0, 0)]
        pad[axis] = (r, r)
        p = np.pad(out, pad, mode="reflect")
        acc = np.zeros_like(out)
        for t in range(2 * r + 1):
            sl = [slice(None), slice(None)]
            sl[axis] = slice(t, t + out.shape[axis])
            acc += k[t] * p[tuple(sl)]
        out = acc
    return out


def _bilinear_shift(a: np.ndarray, sx: float, sy: float) -> np.ndarray:
    """b(x, y) = a(x - sx, y - sy), bilinear, edge-clamped."""
    nx, ny = a.shape
    X = np.arange(nx)[:, None] - sx
    Y = np.arange(ny)[None, :] - sy
    x0 = np.floor(X).astype(np.int64)
    y0 = np.floor(Y).astype(np.int64)
    fx = X - x0
    fy = Y - y0
    x0c, x1c = np.clip(x0, 0, nx - 1), np.clip(x0 + 1, 0, nx - 1)
    y0c, y1c = np.clip(y0, 0, ny - 1), np.clip(y0 + 1, 0, ny - 1)
    return ((1 - fx) * (1 - fy) * a[x0c, y0c] + fx * (1 - fy) * a[x1c, y0c]
            + (1 - fx) * fy * a[x0c, y1c] + fx * fy * a[x1c, y1c])


def texture_pair(n: int = 256, seed: int = 0, sigma: float = 2.0, shift=(1.5, -0.75),
                 ny: int | None = None):
    """Configs 2/3/5: uniform(0,1) noise (seed) blurred with a Gaussian of
    `sigma`, normalised to [0, 1]; mov = ref shifted bilinearly by `shift`."""
    ny = n if ny is None else ny
    rng = np.random.default_rng(seed)
    a = _blur(rng.random((n, ny)), sigma)
    a = (a - a.min()) / (a.max() - a.min())
    return a, _bilinear_shift(a, *shift)


def shifted_disk(n: int = 256, shift=(4, 2), radius: float | None = None):
    """Config 4 (Fluid): a sharp-edged disk of diameter n/2 shifted by (4, 2) px;
    Fluid needs strong edges (SURVEY.md §7 'Synthetic inputs')."""
    radius = n / 4 if radius is None else radius
    x = np.arange(n)[:, None] + 0.5
    y = np.arange(n)[None, :] + 0.5
    c = n / 2
    ref = (((x - c) ** 2 + (y - c) ** 2) < radius ** 2).astype(np.float64)
    mov = (((x - c - shift[0]) ** 2 + (y - c - shift[1]) ** 2) < radius ** 2).astype(np.float64)
    return ref, mov


def procedural_pair(dimx: int, row_lo: int, row_hi: int, seed: int = 0, waves: int = 24,
                    shift=(1.5, -0.75)):
    """Rows [row_lo, row_hi) of a smooth procedural texture (sum of random plane
    waves, normalised to about [0, 1]) and of the same texture translated by
    `shift`.  Any slab of any global grid is generated independently and
    consistently, so every rank builds only its own rows (benchmarks, weak
    scaling).  Returns ([dimx, rows], [dimx, rows]) float64."""
    rng = np.random.default_rng(seed)
    k = rng.uniform(0.02, 0.35, size=waves)
    th = rng.uniform(0, 2 * np.pi, size=waves)
    ph = rng.uniform(0, 2 * np.pi, size=waves)
    amp = rng.uniform(0.5, 1.0, size=waves)
    kx, ky = k * np.cos(th), k * np.sin(th)
    x = np.arange(dimx, dtype=np.float64)[:, None]
    y = np.arange(row_lo, row_hi, dtype=np.float64)[None, :]
    norm = 0.5 / amp.sum()

    def tex(X, Y):
        # sin(u x + v y + p) = sin(u x) cos(v y + p) + cos(u x) sin(v y + p): one GEMM
        A = np.concatenate([amp * np.sin(X * kx), amp * np.cos(X * kx)], axis=1)
        B = np.concatenate([np.cos(ky[:, None] * Y + ph[:, None]),
                            np.sin(ky[:, None] * Y + ph[:, None])], axis=0)
        return 0.5 + norm * (A @ B)

    return tex(x, y), tex(x - shift[0], y - shift[1])

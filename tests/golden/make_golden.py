"""Generate the golden fixtures under tests/golden/ (run in the build container).

1. ``ref_prims.npz`` — inputs and outputs of the reference's OWN primitives
   (src/gradients.h, src/coord2d.h, src/Kernel.cpp compiled from
   /root/reference by oracle/Makefile into oracle/_ref/libref_prims.so).
2. ``oracle_paths.npz`` — whole-registration outputs of the oracle
   (oracle/of2d_oracle.c) on small synthetic pairs, for regression of the
   oracle itself and for GPU parity without re-running the oracle.
3. ``reference_known_answers.json`` is hand-written (reference outputs recorded
   in SURVEY.md §8c / §7) and not produced here.

Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from opticalflow2d_amd import synthetic as S  # noqa: E402

GAUSS_CASES = [(5, 2.0), (5, 1.0), (3, 0.5), (7, 1.3), (1, 1.0), (4, 2.0), (9, 3.5)]


def make_ref_prims(path):
    O.build(ref=True)
    R = O.ref_lib()
    assert R is not None, "oracle/_ref/libref_prims.so missing (needs /root/reference)"
    rng = np.random.default_rng(1234)
    out = {}
    for k, (kw, s) in enumerate(GAUSS_CASES):
        w = np.zeros(kw * kw)
        R.ref_gaussian(kw, s, w)
        out[f"gauss_{k}"] = w
    out["gauss_cases"] = np.array(GAUSS_CASES, dtype=np.float64)
    dx, dy = 37, 23
    I = rng.random(dx * dy).astype(np.float32)
    dI = np.zeros(2 * dx * dy, np.float32)
    R.ref_spatial_derivative(I, dx, dy, dI)
    u = (3 * rng.standard_normal(2 * dx * dy)).astype(np.float32)
    q = np.zeros_like(u)
    R.ref_qlaplacian(u, dx, dy, q)
    dudx, dudy = np.zeros_like(u), np.zeros_like(u)
    R.ref_motion_partials(u, dx, dy, dudx, dudy)
    g = rng.standard_normal(2 * dx * dy).astype(np.float32)
    It = rng.standard_normal(dx * dy).astype(np.float32)
    hs = np.zeros_like(u)
    R.ref_hs_pointwise(q, g, It, dx * dy, 0.1, hs)
    out.update(dims=np.array([dx, dy]), I=I, dI=dI, u=u, q=q, dudx=dudx, dudy=dudy, g=g, It=It,
               hs_alpha=np.float32(0.1), hs=hs,
               norm=np.float32(R.ref_norm_probe(u, dx * dy)),
               maxabs=np.float32(R.ref_maxabs_probe(u, dx * dy)))
    np.savez_compressed(path, **out)


PATH_CASES = {
    # name: (pair, dims, niter, nscales, reg, params, nrefine)
    "hs_square64": ("square", 64, [60], 0, 0, [0.1], 1),
    "hs_texture64_pyr": ("texture", 64, [40, 30], 1, 0, [0.2], 2),
    "demons_texture64": ("texture", 64, [20], 0, 3, [1.0, 0.25, 2.0, 2.0, 5, 0], 1),
    "demons_add_texture64": ("texture", 64, [15], 0, 3, [1.0, 0.25, 2.0, 1.0, 3, 1], 1),
    "fluid_disk64": ("disk", 64, [30, 30], 1, 5, [0.25, 0.0], 1),
    "elastic_texture64": ("texture", 64, [25], 0, 2, [0.5, 0.25], 1),
}


def pair(kind, n):
    if kind == "square":
        return S.translated_square(n, lo=n // 4, hi=3 * n // 4)
    if kind == "texture":
        return S.texture_pair(n, seed=7)
    return S.shifted_disk(n)


def make_oracle_paths(path):
    O.lib().oracle_capture_output(1)
    out = {}
    for name, (kind, n, niter, nscales, reg, params, nrefine) in PATH_CASES.items():
        ref, mov = pair(kind, n)
        r = O.Registration((n, n), niter, nscales, reg, params, nrefine, 0)
        r.register(ref, mov)
        out[f"{name}/ref"] = ref
        out[f"{name}/mov"] = mov
        out[f"{name}/motion"] = r.motion()
        out[f"{name}/warped"] = r.warp(mov)
        out[f"{name}/iters"] = np.array(r.iterations(), np.int32)
        r.close()
    O.lib().oracle_clear_output()
    np.savez_compressed(path, **out)


if __name__ == "__main__":
    make_ref_prims(os.path.join(HERE, "ref_prims.npz"))
    make_oracle_paths(os.path.join(HERE, "oracle_paths.npz"))
    print("wrote", os.listdir(HERE))

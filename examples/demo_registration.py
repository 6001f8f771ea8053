#!/usr/bin/env python3
"""End-to-end registration through the MEX call sequence, the way a reference
user drives it from test_opticalflow2d.m (init -> register -> get motion ->
warp -> close, test_opticalflow2d.m:42-59), but from Python through
``opticalflow2d_amd.OpticalFlow2d`` (same modes, same argument meaning).

The reference demo reads two DIR-lab slices that are not part of the
repository; this one builds a synthetic pair (a disk shifted by a few pixels,
or a smooth texture pair for Demons,
replicate-padded by 11 pixels along x like the demo) so it runs anywhere an MI355X is.

    python examples/demo_registration.py [--reg 5] [--size 256]

Prints the motion statistics the reference demo prints (mean / std, maxabs)
plus the residual before and after warping and the minimum Jacobian of the
motion (the quantity the demo plots).
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from opticalflow2d_amd import OpticalFlow2d, Regularisation  # noqa: E402
from opticalflow2d_amd import synthetic as S  # noqa: E402

# per regularisation: niter per scale, nscales, parameters (SolverOptions order)
PRESETS = {
    Regularisation.Diffusion: ([200, 200], 1, [0.1]),
    Regularisation.Elastic: ([100, 100], 1, [0.25, 0.0]),
    Regularisation.ThirionsDemons: ([50, 50], 1, [1.0, 0.25, 2.0, 2.0, 5, 0]),
    Regularisation.Curvature: ([100, 100], 1, [0.1]),
    # (5 parameters: no accumulation mode.  With per-iteration updates below
    # 0.5 px, Motion::exp takes no squaring step and the result equals Thirion's
    # with Composition; the oracle agrees)
    Regularisation.DiffeomorphicDemons: ([50, 50], 1, [1.0, 0.25, 2.0, 2.0, 5]),
    Regularisation.Fluid: ([25, 25, 200], 2, [0.25, 0.0]),
}


def jacobian_min(motion: np.ndarray) -> float:
    """min over the grid of det(I + grad u), numpy.gradient differences."""
    dudx, dudy = np.gradient(motion[:, :, 0])
    dvdx, dvdy = np.gradient(motion[:, :, 1])
    return float(((1.0 + dudx) * (1.0 + dvdy) - dudy * dvdx).min())


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reg", type=int, default=int(Regularisation.Fluid))
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--verbose", type=int, default=0)
    args = ap.parse_args()
    reg = Regularisation(args.reg)
    if reg not in PRESETS:
        print(f"no preset for {reg.name}", file=sys.stderr)
        return 2
    niter, nscales, params = PRESETS[reg]

    if reg in (Regularisation.ThirionsDemons, Regularisation.DiffeomorphicDemons):
        # Demons divides by |grad I|^2 + It^2 s: a flat background makes that 0 and
        # the reference throws "Divide by zero exception" (Demons.cpp:57), so the
        # Demons presets register a smooth texture pair instead of the disk
        ref, mov = S.texture_pair(args.size)
    else:
        ref, mov = S.shifted_disk(args.size)
    ref = (ref - ref.min()) / (ref.max() - ref.min())
    mov = (mov - mov.min()) / (mov.max() - mov.min())
    # replicate-pad the first (x) dimension by 11, as the demo's padarray(.., [11 0])
    pad = 11
    ref = np.pad(ref, ((pad, pad), (0, 0)), mode="edge")
    mov = np.pad(mov, ((pad, pad), (0, 0)), mode="edge")
    dimx, dimy = ref.shape

    OpticalFlow2d([dimx, dimy], niter, nscales, int(reg), params, len(params), 1, args.verbose)
    t0 = time.perf_counter()
    OpticalFlow2d(ref, mov)
    elapsed = time.perf_counter() - t0
    motion = OpticalFlow2d(nargout=1)
    ireg = OpticalFlow2d(mov, nargout=1)
    OpticalFlow2d()

    # the demo crops 11 pixels off both dimensions (test_opticalflow2d.m:62-65)
    core = (slice(pad, -pad), slice(pad, -pad))
    ref_c, mov_c, reg_c = ref[core], mov[core], ireg[core]
    motion_c = motion[pad:-pad, pad:-pad, :]
    print(f"{reg.name}: {dimx}x{dimy}, niter {niter}, nscales {nscales}, {elapsed:.3f} s")
    print(f"Distribution: {motion_c.mean():.3f} +/ {motion_c.std():.3f}")
    print(f"Maxabs: {np.abs(motion_c).max():.3f}")
    print(f"mean |Iref - Imov| {np.abs(ref_c - mov_c).mean():.4f} -> "
          f"mean |Iref - Ireg| {np.abs(ref_c - reg_c).mean():.4f}")
    print(f"min Jacobian {jacobian_min(motion_c):.3f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())

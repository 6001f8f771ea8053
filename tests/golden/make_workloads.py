#!/usr/bin/env python3
"""Golden records of each BASELINE.json GPU configuration's FULL workload.

The GPU suite compares most kernels with the oracle over a few iterations; these
records pin the whole benchmarked work instead.  Each is the oracle (the C
restatement of the reference path, oracle/of2d_oracle.c, itself pinned by the
reference's compiled primitives and known answers) run once, here, on exactly
the inputs and options the benchmark uses, reduced to SHA-256 digests so that a
GPU test can compare a full-size run without running the oracle again:

  cfg2  Horn-Schunck 4096^2, procedural pair, alpha 0.1, 1000 fixed Jacobi
        iterations: bench.py's step (SlabSolver, zero initial motion, one level,
        one refine), oracle_hs_loop_mt (bit-identical to the one-thread loop,
        tests/test_oracle.py) on the gradients of the moving image
        (IterativeSolver.cpp:22-56), then motion->accumulate(motion_est) onto the
        zero motion (ImageRegistrationOpticalFlow.cpp:138)
  cfg3  Thirion's Demons 4096^2, procedural pair, params [1, 0.25, 2, 2, 5, 0]
        (Composition, kw 5), 100 fixed iterations (bench_configs.py cfg3;
        DemonsThirions.cpp:18-42)
  cfg4  viscous fluid 8192^2, shifted disk, 3-level pyramid x 200 fixed
        iterations, params [0.25, 0.0] (bench_configs.py cfg4;
        ImageRegistrationFluid.cpp:67-142) with every printed Dumax /
        Regridding line (OpticalFlowFluid.cpp:94, ImageRegistrationFluid.cpp:110)

    python tests/golden/make_workloads.py [cfg2 cfg3 cfg4]   (cfg4: ~30 min)
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from opticalflow2d_amd import synthetic as S  # noqa: E402

OUT = os.path.join(HERE, "workloads.json")

CFG2 = {"n": 4096, "alpha": 0.1, "niter": 1000, "pair": "procedural_pair(n, 0, n)"}
CFG3 = {"n": 4096, "params": [1.0, 0.25, 2.0, 2.0, 5, 0], "niter": [100],
        "pair": "procedural_pair(n, 0, n)"}
CFG4 = {"n": 8192, "params": [0.25, 0.0], "niter": [200, 200, 200], "nscales": 2,
        "pair": "shifted_disk(n)"}


def digest_planar(m):
    """SHA-256 of a [dimx, dimy, 2] motion as float32 planar [x; y] bits (the
    double output is an exact widening of the float field)."""
    f = np.asarray(m, np.float32)
    planar = np.concatenate([f[:, :, 0].reshape(-1, order="F"), f[:, :, 1].reshape(-1, order="F")])
    return hashlib.sha256(planar.tobytes()).hexdigest()


def digest_image(w):
    f = np.asarray(w, np.float32).reshape(-1, order="F")
    return hashlib.sha256(f.tobytes()).hexdigest()


def printed_body(text):
    """The lines a fluid loop prints after the banner (tests/test_gpu_fluid.py)."""
    return [l for l in text.splitlines() if l.startswith(("Dumax", "Regridding", "Iteration"))]


def digest_lines(lines):
    return hashlib.sha256("\n".join(lines).encode()).hexdigest()


def cfg2():
    n, it = CFG2["n"], CFG2["niter"]
    ref, mov = S.procedural_pair(n, 0, n)
    L = O.lib()
    I = np.ascontiguousarray(mov.reshape(-1, order="F").astype(np.float32))
    Ir = np.ascontiguousarray(ref.reshape(-1, order="F").astype(np.float32))
    dI = np.zeros(2 * n * n, np.float32)
    It = np.zeros(n * n, np.float32)
    L.oracle_spatial_derivative(I, n, n, dI)
    L.oracle_temporal_derivative(Ir, I, n * n, It)
    u = np.zeros(2 * n * n, np.float32)
    errs = np.zeros(it, np.float32)
    t0 = time.time()
    assert L.oracle_hs_loop_mt(u, dI, It, n, n, CFG2["alpha"], it, os.cpu_count() or 1, errs) == it
    dt = time.time() - t0
    motion = np.zeros_like(u)
    L.oracle_accumulate(motion, u, n, n)
    m = motion.reshape(n * n, 2)
    planar = np.concatenate([m[:, 0], m[:, 1]])
    return dict(CFG2, motion_sha256_f32_planar=hashlib.sha256(planar.tobytes()).hexdigest(),
                sum_motion=float(m.astype(np.float64).sum()),
                max_abs_motion=float(np.abs(m).max()), oracle_seconds=round(dt, 1),
                oracle="oracle_hs_loop_mt + oracle_accumulate")


def registration(dims, niter, nscales, reg, params, ref, mov):
    L = O.lib()
    L.oracle_capture_output(1)
    L.oracle_clear_output()
    t0 = time.time()
    o = O.Registration(dims, niter, nscales, reg, params, 1, 0, fixed_iters=True)
    o.register(ref, mov)
    m, it = o.motion(), o.iterations()
    w = o.warp(mov)
    o.close()
    text = L.oracle_captured_output().decode()
    L.oracle_clear_output()
    return m, it, w, text, time.time() - t0


def cfg3():
    n = CFG3["n"]
    ref, mov = S.procedural_pair(n, 0, n)
    m, it, w, _, dt = registration((n, n), CFG3["niter"], 0, 3, CFG3["params"], ref, mov)
    return dict(CFG3, iterations=it, motion_sha256_f32_planar=digest_planar(m),
                warped_sha256_f32=digest_image(w), sum_motion=float(m.sum()),
                max_abs_motion=float(np.abs(m).max()), oracle_seconds=round(dt, 1),
                oracle="oracle Registration (fixed_iters)")


def cfg4():
    n = CFG4["n"]
    ref, mov = S.shifted_disk(n)
    m, it, w, text, dt = registration((n, n), CFG4["niter"], CFG4["nscales"], 5, CFG4["params"],
                                      ref, mov)
    body = printed_body(text)
    return dict(CFG4, iterations=it, motion_sha256_f32_planar=digest_planar(m),
                warped_sha256_f32=digest_image(w), printed_lines=len(body),
                printed_sha256=digest_lines(body),
                regridding_lines=sum(l.startswith("Regridding") for l in body),
                timestep_skips=sum(1 for l in body if "Timestep:" in l
                                   and float(l.split("Timestep:")[1]) >= 65.0),
                first_lines=body[:3], sum_motion=float(m.sum()),
                max_abs_motion=float(np.abs(m).max()), oracle_seconds=round(dt, 1),
                oracle="oracle Registration (fixed_iters)")


def main(names):
    rec = json.load(open(OUT)) if os.path.exists(OUT) else {
        "_source": "oracle/of2d_oracle.c via tests/golden/make_workloads.py"}
    for name in names or ["cfg2", "cfg3", "cfg4"]:
        r = {"cfg2": cfg2, "cfg3": cfg3, "cfg4": cfg4}[name]()
        rec[name] = r
        with open(OUT, "w") as f:
            json.dump(rec, f, indent=1)
        print(name, r.get("iterations"), r["oracle_seconds"], "s", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])

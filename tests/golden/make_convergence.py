#!/usr/bin/env python3
"""Golden fixtures for convergence-on (default semantics) Horn-Schunck at
config scale: the oracle (the C restatement of the reference path, pinned by
the reference's known answers, tests/golden/reference_known_answers.json) run
init -> register -> get with niter = 1000 and the reference's break test
`err < 0.001f && iter > 1` (ImageRegistrationOpticalFlow.cpp:131-134) on the
Logger's sequential fp32 norm (Motion.cpp:42-49, Logger.cpp:32-51).

Each fixture records the iterations executed, every iteration's Logger error
and a SHA-256 of the final motion's float32 bits, so a GPU test can compare a
4096^2 run without running the oracle again.  "exact_norms" holds the same
for the oracle with the Logger's norms summed in double (oracle_set_logger_fp64):
at 4096^2 the reference's sequential FLOAT running sum (Motion.cpp:42-49)
rounds each of its 16.7 M additions at ~1 ulp of the sum, so its error can
cross 0.001 an iteration away from where the exactly summed error does.  The
GPU's default Logger reproduces the float running sum bit for bit
(seqnorm_kernels.hip) and is checked against the reference-semantics records;
its `logger_fp64` mode sums in fp64 and is checked against "exact_norms".

    python tests/golden/make_convergence.py [--exact-only] [name ...]
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

CASES = {
    # name: (generator, n, niter)
    "hs_texture1024": ("texture_pair", 1024, 1000),
    "hs_texture4096": ("texture_pair", 4096, 1000),
    "hs_procedural4096": ("procedural_pair", 4096, 1000),
}


def inputs(gen, n):
    if gen == "texture_pair":
        return S.texture_pair(n)
    return S.procedural_pair(n, 0, n)


def motion_digest(m):
    """SHA-256 of the motion as float32 planar [x-plane; y-plane] bits (the
    double output is an exact widening of the float field)."""
    f = np.asarray(m, np.float32)
    planar = np.concatenate([f[:, :, 0].reshape(-1, order="F"), f[:, :, 1].reshape(-1, order="F")])
    return hashlib.sha256(planar.tobytes()).hexdigest()


def run(gen, n, niter, fp64):
    ref, mov = inputs(gen, n)
    O.lib().oracle_capture_output(1)
    O.lib().oracle_set_logger_fp64(1 if fp64 else 0)
    t0 = time.time()
    try:
        o = O.Registration((n, n), [niter], 0, 0, [0.1], 1, 0)
        o.register(ref, mov)
        m, it, errs = o.motion(), o.iterations(), o.last_errors()
        o.close()
    finally:
        O.lib().oracle_set_logger_fp64(0)
        O.lib().oracle_clear_output()
    return m, it, errs, time.time() - t0


def add_exact(name):
    gen, n, niter = CASES[name]
    path = os.path.join(HERE, f"convergence_{name}.json")
    rec = json.load(open(path))
    m, it, errs, dt = run(gen, n, niter, True)
    rec["exact_norms"] = {
        "iterations_executed": it,
        "errors": [float(e) for e in errs],
        "motion_sha256_f32_planar": motion_digest(m),
        "oracle_seconds": round(dt, 1),
    }
    with open(path, "w") as f:
        json.dump(rec, f, indent=1)
    print(name, "exact norms:", it, "reference norms:", rec["iterations_executed"], flush=True)


def main(names):
    if names and names[0] == "--exact-only":
        for name in names[1:] or CASES:
            add_exact(name)
        return
    for name in names or CASES:
        gen, n, niter = CASES[name]
        ref, mov = inputs(gen, n)
        O.lib().oracle_capture_output(1)
        t0 = time.time()
        o = O.Registration((n, n), [niter], 0, 0, [0.1], 1, 0)
        o.register(ref, mov)
        m = o.motion()
        it = o.iterations()
        errs = o.last_errors()
        o.close()
        O.lib().oracle_clear_output()
        rec = {
            "_source": "oracle/of2d_oracle.c via tests/golden/make_convergence.py",
            "generator": gen, "n": n, "niter": [niter], "alpha": 0.1, "reg": 0,
            "iterations_executed": it,
            "errors": [float(e) for e in errs],
            "motion_sha256_f32_planar": motion_digest(m),
            "sum_motion": float(m.sum()),
            "max_abs_motion": float(np.abs(m).max()),
            "oracle_seconds": round(time.time() - t0, 1),
        }
        with open(os.path.join(HERE, f"convergence_{name}.json"), "w") as f:
            json.dump(rec, f, indent=1)
        print(name, it, rec["oracle_seconds"], "s", flush=True)
        add_exact(name)


if __name__ == "__main__":
    main(sys.argv[1:])

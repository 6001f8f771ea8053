#!/usr/bin/env python3
"""SOR wavefront probe: a single strip (step latency) and a single row band
(strip-to-strip lag) of the viscous-fluid solver, timed under rocprofv3."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from opticalflow2d_amd import ImageRegistration, set_print_sink
from opticalflow2d_amd import synthetic as S

set_print_sink(lambda s: None)
for dims in [(64, 8192), (8192, 64), (8192, 8192)]:
    n = max(dims)
    rng = np.random.default_rng(0)
    ref = rng.random(dims) * 100
    mov = np.roll(ref, 1, axis=0)
    with ImageRegistration(dims, [10], 0, 5, [0.25, 0.0], 1, fixed_iters=1) as r:
        r.register(ref, mov)
        r.register(ref, mov)
    print(dims, "done", flush=True)

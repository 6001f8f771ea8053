"""Wall time of convergence-on registrations in the two Logger modes
(reference-exact float norms, default; fp64 sums, `logger_fp64`).

    python tools/time_convergence.py [n] [reps]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opticalflow2d_amd import ImageRegistration, set_print_sink  # noqa: E402
from opticalflow2d_amd import synthetic as S  # noqa: E402

set_print_sink(lambda s: None)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
only = os.environ.get("OF2D_CONV_CASE")  # one of the pairs (traces)
cases = {k: g() for k, g in (("texture", lambda: S.texture_pair(n)),
                             ("procedural", lambda: S.procedural_pair(n, 0, n)))
         if not only or k == only}
for name, (ref, mov) in cases.items():
    for fp64 in ((0,) if os.environ.get("OF2D_CONV_ONLY") else (0, 1)):
        extra = {}
        if os.environ.get("OF2D_CONV_CHUNK"):  # iterations per host decision block
            extra["chunk"] = int(os.environ["OF2D_CONV_CHUNK"])
        if os.environ.get("OF2D_CONV_GI"):  # the triple's gradients from Iaux
            extra["hs_gradients_from_image"] = int(os.environ["OF2D_CONV_GI"])
        if os.environ.get("OF2D_CONV_FRESH"):
            # a fresh registration per estimate (as a MEX register call after
            # init: bench.py default_semantics), the first one a warm-up
            ts = []
            for rep in range(reps + 1):
                with ImageRegistration((n, n), [1000], 0, 0, [0.1], logger_fp64=fp64,
                                       **extra) as r:
                    r.set_images(ref, mov)
                    t0 = time.perf_counter()
                    r.estimate()
                    if rep:
                        ts.append(time.perf_counter() - t0)
                    it = r.iterations()[0]
                    mot = r.motion()
        else:
            with ImageRegistration((n, n), [1000], 0, 0, [0.1], logger_fp64=fp64, **extra) as r:
                r.set_images(ref, mov)
                r.estimate()  # warm-up
                ts = []
                for _ in range(reps):
                    t0 = time.perf_counter()
                    r.estimate()
                    ts.append(time.perf_counter() - t0)
                it = r.iterations()[0]
                mot = r.motion()
        # the second estimate warm-starts from the first's motion (reference
        # semantics): iterations of the timed calls, not of the first
        t = min(ts)
        h = ""
        if os.environ.get("OF2D_CONV_HASH"):  # the last estimate's motion
            import hashlib
            h = " motion " + hashlib.sha256(np.ascontiguousarray(mot).tobytes()).hexdigest()[:16]
        print(f"{name:10s} {n}^2 logger_fp64={fp64}: {it} iterations, {t*1e3:.2f} ms "
              f"({t*1e6/it:.1f} us/iteration){h}", flush=True)

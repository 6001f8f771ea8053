"""One warm convergence-on registration of the 4096^2 texture pair (for a
kernel trace of the exact loop's start and end):
    python tools/time_texture_loop.py [n]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opticalflow2d_amd import ImageRegistration, set_print_sink  # noqa: E402
from opticalflow2d_amd import synthetic as S  # noqa: E402

set_print_sink(lambda s: None)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
ref, mov = S.texture_pair(n)
with ImageRegistration((n, n), [1000], 0, 0, [0.1]) as r:
    r.set_images(ref, mov)
    r.estimate()
    t0 = time.perf_counter()
    r.estimate()
    t = time.perf_counter() - t0
    print(f"texture {n}^2: {r.iterations()[0]} iterations, {t * 1e3:.2f} ms", flush=True)

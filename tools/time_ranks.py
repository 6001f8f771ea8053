"""Wall time per iteration of the in-process multi-device HS path
(of2d_set_option "ngpus", csrc/ranks.cpp) at 4096^2 against one rank: fixed
iterations and convergence on (the reference-exact Logger).  Each count runs
with the default (ranks beyond the device count merge: on a one-GPU box the
one-device loop) and with "ngpus_share" (every rank on device 0 of a one-GPU
box: the decomposition's overhead at equal total work).

    python tools/time_ranks.py [n] [reps] [modes] [ngpus]

modes: "fixed,conv" (default both); ngpus: comma list (default 1,2,8).
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opticalflow2d_amd import ImageRegistration, set_print_sink  # noqa: E402
from opticalflow2d_amd import synthetic as S  # noqa: E402

set_print_sink(lambda s: None)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
modes = sys.argv[3].split(",") if len(sys.argv) > 3 else ["fixed", "conv"]
ngs = [int(v) for v in sys.argv[4].split(",")] if len(sys.argv) > 4 else [1, 2, 8]
ref, mov = S.texture_pair(n)
for mode, opts, niter in (("fixed 999", {"fixed_iters": 1}, 999), ("convergence", {}, 1000)):
    if mode.split()[0][:4] not in [m[:4] for m in modes]:
        continue
    base = None
    for ng, share in [(g, sh) for g in ngs for sh in ((0,) if g == 1 else (0, 1))]:
        if os.environ.get("OF2D_MAPS_DUMP"):  # to symbolise a crash's frames afterwards
            with open("/proc/self/maps") as f, open(os.environ["OF2D_MAPS_DUMP"], "w") as g:
                g.write(f.read())
        with ImageRegistration((n, n), [niter], 0, 0, [0.1], ngpus=ng, ngpus_share=share,
                               **opts) as r:
            r.set_images(ref, mov)
            r.estimate()  # warm-up (allocations, the ranks' threads' first launches)
            ts = []
            for _ in range(reps):
                r.set_images(ref, mov)
                t0 = time.perf_counter()
                r.estimate()
                ts.append(time.perf_counter() - t0)
            it = r.iterations()[0]
        t = min(ts)
        us = t * 1e6 / it
        base = base or us
        print(f"{mode:12s} {n}^2 ngpus={ng} share={share}: {it} iterations, {t*1e3:.2f} ms "
              f"({us:.1f} us/iteration, {us / base:.3f}x of ngpus=1)", flush=True)

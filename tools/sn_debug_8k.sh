#!/bin/bash
# Exact-Logger cost counters of a warm-started 8192^2 texture registration
# (OF2D_SN_DEBUG: per-iteration walk resolves / raw segments / listed tiles).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OF2D_SN_DEBUG=1 timeout -k 10 600 python3 -u - <<'PY' > gpurun_out/r03ah_sndebug.log 2>&1
import os, sys, time
sys.path.insert(0, os.getcwd())
from opticalflow2d_amd import ImageRegistration, set_print_sink
from opticalflow2d_amd import synthetic as S
set_print_sink(lambda s: None)
n = 8192
ref, mov = S.texture_pair(n)
with ImageRegistration((n, n), [1000], 0, 0, [0.1]) as r:
    r.set_images(ref, mov)
    t0 = time.perf_counter(); r.estimate(); t1 = time.perf_counter()
    print("first", r.iterations(), t1 - t0, file=sys.stderr, flush=True)
    t0 = time.perf_counter(); r.estimate(); t1 = time.perf_counter()
    print("second", r.iterations(), t1 - t0, file=sys.stderr, flush=True)
PY
rc=$?
grep -E "first|second" gpurun_out/r03ah_sndebug.log
exit $rc

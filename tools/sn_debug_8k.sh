#!/bin/bash
# Exact-Logger cost counters of warm-started registrations (OF2D_SN_DEBUG:
# per-iteration walk resolves / raw segments / listed tiles / clocks / tiles
# given the walk's own entries).  usage: tools/sn_debug_8k.sh <tag> [n] [case]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-r03ah}; n=${2:-8192}; case=${3:-texture}
log=gpurun_out/${tag}_sndebug${n}${case}.log
[ "$n" = 8192 ] && [ "$case" = texture ] && log=gpurun_out/${tag}_sndebug.log
OF2D_SN_DEBUG=1 timeout -k 10 600 python3 -u - $n $case <<'PY' > $log 2>&1
import os, sys, time
sys.path.insert(0, os.getcwd())
from opticalflow2d_amd import ImageRegistration, set_print_sink
from opticalflow2d_amd import synthetic as S
set_print_sink(lambda s: None)
n, case = int(sys.argv[1]), sys.argv[2]
ref, mov = S.texture_pair(n) if case == "texture" else S.procedural_pair(n, 0, n)
with ImageRegistration((n, n), [1000], 0, 0, [0.1]) as r:
    r.set_images(ref, mov)
    t0 = time.perf_counter(); r.estimate(); t1 = time.perf_counter()
    print("first", r.iterations(), t1 - t0, file=sys.stderr, flush=True)
    t0 = time.perf_counter(); r.estimate(); t1 = time.perf_counter()
    print("second", r.iterations(), t1 - t0, file=sys.stderr, flush=True)
PY
rc=$?
grep -E "first|second" $log
exit $rc

cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
OF2D_SN_DEBUG=1 timeout -k 10 300 python3 -u - <<'PY' > gpurun_out/r03bo_sndebug_cfg1.log 2>&1
import os, sys, time
sys.path.insert(0, os.getcwd())
from opticalflow2d_amd import ImageRegistration, set_print_sink
from opticalflow2d_amd import synthetic as S
set_print_sink(lambda s: None)
ref, mov = S.translated_square(256)
with ImageRegistration((256, 256), [200], 0, 0, [0.1]) as r:
    r.register(ref, mov)
    t0 = time.perf_counter(); r.register(ref, mov); t1 = time.perf_counter()
    print("second", r.iterations(), t1 - t0, file=sys.stderr, flush=True)
PY
rc=$?; grep -c seqnorm gpurun_out/r03bo_sndebug_cfg1.log; grep second gpurun_out/r03bo_sndebug_cfg1.log; exit $rc

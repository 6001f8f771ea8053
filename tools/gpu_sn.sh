#!/bin/bash
# Exact-Logger check on the GPU box: the seqnorm / convergence tests, then
# convergence timings at 4096^2 and 8192^2 and the 8192^2 walk counters.
# usage: tools/gpu_sn.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:?tag}
step() {
    local name=$1; shift
    echo "== $name: $*"
    timeout -k 10 600 "$@" > gpurun_out/${tag}_$name.log 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -n 12 gpurun_out/${tag}_$name.log
    return $rc
}
step sntests python -u -m pytest tests/test_gpu_seqnorm.py tests/test_gpu_convergence.py -x -q \
    --timeout 300 --timeout-method thread &&
step conv python -u tools/time_convergence.py 4096 3 &&
bash tools/sn_debug_8k.sh ${tag} &&
step conv8k python -u tools/time_convergence.py 8192 1

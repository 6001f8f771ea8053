#!/bin/bash
# Convergence-on timings at several host block sizes ("chunk" option), interleaved:
#   tools/gpu_ab_chunk.sh <rounds> <chunk>...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rounds=$1; shift
for r in $(seq 1 $rounds); do
    for c in "$@"; do
        echo "== round $r chunk $c"
        OF2D_CONV_CHUNK=$c OF2D_CONV_ONLY=1 timeout -k 10 300 python -u tools/time_convergence.py 4096 3 2>&1 | grep -v amdgpu || exit 1
    done
done

#!/bin/bash
# convergence-on timings, the in-tree library and tools/ab/<variant>s,
# interleaved: tools/gpu_ab_conv3.sh <rounds> <variant>...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rounds=$1; shift
for r in $(seq 1 $rounds); do
    for v in tree "$@"; do
        lp=""; [ "$v" != tree ] && lp="$PWD/tools/abx/$v/libof2d.so"
        echo "== round $r $v"
        OF2D_LIB_PATH=$lp OF2D_CONV_ONLY=1 timeout -k 10 300 python -u tools/time_convergence.py 4096 3 2>&1 | grep -v amdgpu || exit 1
    done
done

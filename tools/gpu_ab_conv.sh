#!/bin/bash
# Convergence-on timings (tools/time_convergence.py) of the in-tree library
# ("base") and A/B builds (tools/build_variant.sh), interleaved:
#   tools/gpu_ab_conv.sh <rounds> <n> <variant>...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rounds=$1 n=$2; shift 2
for r in $(seq 1 $rounds); do
    for v in base "$@"; do
        echo "== round $r $v"
        if [ "$v" = base ]; then
            timeout -k 10 300 python -u tools/time_convergence.py $n 2 || exit $?
        else
            OF2D_LIB_PATH=tools/ab/$v/libof2d.so timeout -k 10 300 python -u tools/time_convergence.py $n 2 || exit $?
        fi
    done
done

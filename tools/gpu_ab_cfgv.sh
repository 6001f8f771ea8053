#!/bin/bash
# bench_configs.py configuration A/B: the in-tree library ("base") and
# tools/abx/<variant> builds (tools/build_variant.sh), interleaved, each
# variant's parity tests (a pytest file, or -) first:
#   tools/gpu_ab_cfgv.sh <rounds> <config: 1, 2c, 3, 4 or 5> <pytest file|-> <variant>...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rounds=$1 cfg=$2 tf=$3; shift 3
lib() { [ "$1" = base ] && echo "" || echo "$PWD/tools/abx/$1/libof2d.so"; }
if [ "$tf" != "-" ]; then
    for v in "$@"; do
        echo "== tests $v"
        OF2D_LIB_PATH=$(lib $v) timeout -k 10 600 python -u -m pytest $tf -x -q --timeout 300 --timeout-method thread 2>&1 | tail -n 2 || exit $?
    done
fi
for r in $(seq 1 $rounds); do
    for v in base "$@"; do
        out=$(OF2D_LIB_PATH=$(lib $v) timeout -k 10 300 python -u bench_configs.py --configs $cfg --no-cpu) || exit $?
        echo "round $r $v: $(echo "$out" | grep '^{' | tail -1)"
    done
done

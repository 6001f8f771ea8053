#!/bin/bash
# Round-2 GPU session c: GI (gradients from Iaux) A/B harness, the GPU suite,
# bench (driver command, both gradient sources, default), rocprofv3 stats.
# Stops at the first step that faults / aborts / times out (rc > 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r02c}
OUT=gpurun_out/$TAG
mkdir -p $OUT
R=$PWD
step() {  # step <name> <timeout> <cmd...>
    local name=$1 to=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 8 "$OUT/$name.log"
    return $rc
}
step ab 180 tools/hs_gi_ab 4096 300 5; rc=$?; [ $rc -le 1 ] || exit $rc
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread; rc=$?
[ $rc -le 1 ] || exit $rc
step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
step bench_field 300 python bench.py --gpus 1 --steps 20 --warmup 5 --gradients field --no-cpu-baseline || exit $?
step bench_cfg5 600 python bench.py --grid 16384 --steps 3 --warmup 1 --no-cpu-baseline || exit $?
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof" -o hs -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
echo ALL-DONE

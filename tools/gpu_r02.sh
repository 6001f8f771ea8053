#!/bin/bash
# Round-2 GPU session: gpu tests -> smoke -> bench (driver's command, default,
# config 5 one-GPU point) -> rocprofv3 kernel stats of the driver's command.
# Stops at the first step that faults / aborts / times out (rc > 1).
#   tools/gpu_r02.sh [tag] [pytest -k expr]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r02}
K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
R=$PWD
step() {  # step <name> <timeout> <cmd...>
    local name=$1 to=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 4 "$OUT/$name.log"
    return $rc
}
if [ -n "$K" ]; then
    step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K"; rc=$?
else
    step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread; rc=$?
fi
[ $rc -le 1 ] || exit $rc
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
step bench_default 300 python bench.py || exit $?
step bench_cfg5 600 python bench.py --grid 16384 --steps 600 --warmup 150 --no-cpu-baseline || exit $?
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof" -o hs -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
echo ALL-DONE

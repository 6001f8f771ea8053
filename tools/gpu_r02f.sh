#!/bin/bash
# Round-2 GPU session f: dI vs GI at the config-5 per-rank slab shapes, the
# GPU suite, bench (driver command) + rocprofv3 kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r02f
mkdir -p $OUT
R=$PWD
step() {  # step <name> <timeout> <cmd...>
    local name=$1 to=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 5 "$OUT/$name.log"
    return $rc
}
step ab_4096x4096 120 tools/hs_gi_ab 4096 300 3 -1 4096 || exit $?
step ab_16384x2048 120 tools/hs_gi_ab 16384 150 3 -1 2048 || exit $?
step ab_16384x4096 120 tools/hs_gi_ab 16384 80 3 -1 4096 || exit $?
step ab_8192x4096 120 tools/hs_gi_ab 8192 150 3 -1 4096 || exit $?
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread; rc=$?
[ $rc -le 1 ] || exit $rc
step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
step bench_cfg5 600 python bench.py --grid 16384 --steps 3 --warmup 1 --no-cpu-baseline || exit $?
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof" -o hs -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
echo ALL-DONE

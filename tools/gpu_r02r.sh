#!/bin/bash
# Round-2 GPU session r: final-state check (GPU suite, smoke, bench driver command,
# rocprofv3 kernel stats of the
# driver command, the secondary configurations with their kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${R02_TAG:-r02r}
mkdir -p $OUT
R=$PWD
step() {  # step <name> <timeout> <cmd...>
    local name=$1 to=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 3 "$OUT/$name.log"
    return $rc
}
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread; rc=$?
[ $rc -le 1 ] || exit $rc
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof" -o hs -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
step configs 900 python bench_configs.py || exit $?
step prof_cfg 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_cfg" -o cfg -- python3 "$R/bench_configs.py" --configs 3,4 --iters 20 || exit $?
echo ALL-DONE

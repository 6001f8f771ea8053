#!/bin/bash
# One GPU session: gpu tests -> smoke -> bench -> rocprofv3 kernel stats.
# Stops at the first step that faults / aborts / times out (rc > 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
step() {  # step <name> <timeout> <cmd...>
    local name=$1 to=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 5 "$OUT/$name.log"
    return $rc
}
step tests 600 python -m pytest tests -m gpu -x -q ; rc=$?
[ $rc -le 1 ] || exit $rc
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 600 python bench.py || exit $?
R=$PWD
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof" -o hs -- python3 "$R/bench.py" --no-cpu-baseline || exit $?
echo ALL-DONE

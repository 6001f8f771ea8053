#!/bin/bash
# Round-2 GPU session g: the GPU suite (gradient source parametrised), bench
# driver command, PMC traffic of the config-5 (16384^2, Iaux gradients) launch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r02g
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
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread; rc=$?
[ $rc -le 1 ] || exit $rc
step bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
step ab16384 200 tools/hs_gi_ab 16384 60 3 -1 16384 || exit $?
pass() {  # pass <counter> <tag> <cmd...>
    local c=$1 t=$2; shift 2
    echo "== pmc $c $t"
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$R/$OUT/$t" -o p -- "$@" > $OUT/$t.log 2>&1
}
pass FETCH_SIZE pf "$R/tools/hs_gi_ab" 16384 3 1 -2 16384 || exit $?
pass WRITE_SIZE pw "$R/tools/hs_gi_ab" 16384 3 1 -2 16384 || exit $?
B="$R/bench.py --grid 16384 --steps 1 --warmup 0 --iters-per-step 33 --no-cpu-baseline --timing-launches 3"
pass FETCH_SIZE bf python3 $B || exit $?
pass WRITE_SIZE bw python3 $B || exit $?
csv() { find $OUT/$1 -name '*counter_collection.csv' | head -1; }
python3 tools/pmc_traffic_mix.py --grid 16384 16384 --pitch 16384 --mix image --probe $(csv pf) $(csv pw) --kernel $(csv bf) $(csv bw) --out $OUT/hs_traffic_16384.json
echo ALL-DONE

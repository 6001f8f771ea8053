#!/bin/bash
# PMC traffic of the product HS triple kernel as bench.py launches it: FETCH_SIZE and
# WRITE_SIZE in separate passes (kernel trace only), over the harness (the probe
# kernel's known bytes calibrate the counters) and over bench.py itself.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/pmcb
mkdir -p $O
pass() {  # pass <counter> <tag> <cmd...>
    local c=$1 t=$2; shift 2
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$R/$O/$t" -o p -- "$@" > $O/$t.log 2>&1
}
pass FETCH_SIZE hf "$R/tools/hs_variants" 4096 42 triple || exit $?
pass WRITE_SIZE hw "$R/tools/hs_variants" 4096 42 triple || exit $?
B="python3 $R/bench.py --steps 33 --warmup 0 --no-cpu-baseline --timing-launches 20"
pass FETCH_SIZE bf $B || exit $?
pass WRITE_SIZE bw $B || exit $?
csv() { find $O/$1 -name '*counter_collection.csv' | head -1; }
python3 tools/pmc_traffic.py --out $O/hs_traffic.json $(csv hf) $(csv hw) 4096 --bench $(csv bf) $(csv bw)

#!/bin/bash
# Round-2 GPU session j: SOR wavefront timeline (per-strip start lag, ns per step).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r02j
mkdir -p $OUT
timeout -k 10 60 tools/sor_harness 8192 8192 4 > $OUT/sor8192.log 2>&1 || exit $?
timeout -k 10 60 tools/sor_harness 4096 4096 4 > $OUT/sor4096.log 2>&1 || exit $?
timeout -k 10 60 tools/sor_harness 2048 2048 4 > $OUT/sor2048.log 2>&1 || exit $?
cat $OUT/*.log

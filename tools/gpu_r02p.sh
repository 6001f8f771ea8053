#!/bin/bash
# Round-2 GPU session p: SOR cycles per step and shader clock (strip 0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r02p
mkdir -p $OUT
timeout -k 10 60 tools/sor_harness 64 65536 3 > $OUT/sor64x65536.log 2>&1 || exit $?
timeout -k 10 60 tools/sor_harness 8192 8192 3 > $OUT/sor8192.log 2>&1 || exit $?
timeout -k 10 60 tools/sor_harness 2048 2048 3 > $OUT/sor2048.log 2>&1 || exit $?
grep -E "^glead|strip 0" $OUT/*.log

#!/bin/bash
# Round-2 GPU session k: SOR block kernel (4 strips per block, LDS hand-off):
# fluid/elastic parity tests, then the wavefront timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r02k
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_fluid.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -n 25 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 60 tools/sor_harness 8192 8192 4 > $OUT/sor8192.log 2>&1 || exit $?
timeout -k 10 60 tools/sor_harness 4096 4096 4 > $OUT/sor4096.log 2>&1 || exit $?
timeout -k 10 60 tools/sor_harness 2048 2048 4 > $OUT/sor2048.log 2>&1 || exit $?
cat $OUT/sor*.log

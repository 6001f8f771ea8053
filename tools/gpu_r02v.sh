#!/bin/bash
# Round-2 GPU session v: fluid tests (8192^2 with two iterations per level, the
# dt >= 65 skip), Demons SQ counters after the branch-free gathers.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r02v
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_fluid.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -n 4 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_pmc_groups.sh demons_r02v --configs 3 --iters 5 > $OUT/pmc.log 2>&1 || exit $?
grep -A1 "demons_fused\|smooth_norm" gpurun_out/pmc_demons_r02v/summary.txt

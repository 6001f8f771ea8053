#!/bin/bash
# Round-2 GPU session o: Demons force pass at the warped tile's pitch (LDS bank
# conflicts): Demons + example parity tests, config 3 timing, SQ counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r02o
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_demons.py tests/test_gpu_examples.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -n 4 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench_configs.py --configs 3 > $OUT/cfg3.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/cfg3.log
bash tools/gpu_pmc_groups.sh demons_r02o --configs 3 --iters 5 > $OUT/pmc.log 2>&1 || exit $?
grep -A1 "demons_fused\|smooth_norm" gpurun_out/pmc_demons_r02o/summary.txt

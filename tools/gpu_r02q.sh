#!/bin/bash
# Round-2 GPU session q: smooth_norm with the Logger prev prefetched before the
# tile barrier: Demons tests, config 3 timing and kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
OUT=gpurun_out/r02q
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_demons.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -n 2 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench_configs.py --configs 3 > $OUT/cfg3.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/cfg3.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof" -o cfg -- python3 "$R/bench_configs.py" --configs 3 --iters 50 > $OUT/prof.log 2>&1 || exit $?
cut -c1-110 $OUT/prof/cfg_kernel_stats.csv | head -8

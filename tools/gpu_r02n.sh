#!/bin/bash
# Round-2 GPU session n: fused fluid step (integrate + Logger + Jacobian + next
# force pack): fluid parity tests, config 4 timing, config 3/4 kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
OUT=gpurun_out/r02n
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_fluid.py -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -n 18 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench_configs.py --configs 4 > $OUT/cfg4.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/cfg4.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_cfg" -o cfg -- python3 "$R/bench_configs.py" --configs 4 --iters 20 > $OUT/prof_cfg.log 2>&1 || exit $?
cut -c1-160 $OUT/prof_cfg/cfg_kernel_stats.csv | head -14

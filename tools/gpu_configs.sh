#!/bin/bash
# Secondary configurations + kernel stats for Demons / Fluid.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
mkdir -p gpurun_out
timeout -k 10 900 python bench_configs.py "$@" > gpurun_out/configs.log 2>&1; rc=$?
cat gpurun_out/configs.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_cfg" -o cfg -- python3 "$R/bench_configs.py" --configs 3,4 --iters 20 > gpurun_out/prof_cfg.log 2>&1 || exit $?
cut -c1-160 gpurun_out/prof_cfg/cfg_kernel_stats.csv

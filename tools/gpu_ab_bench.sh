#!/bin/bash
# One-call A/B of bench.py (driver command, no CPU baseline) between the
# in-tree library (A) and tools/lib_alt.so (B), interleaved; B's parity tests first.
#   tools/gpu_ab_bench.sh <tag> <rounds> [pytest file] [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1 N=${2:-2} TF=$3
shift 3
ARGS=${@:-"--gpus 1 --steps 20 --warmup 5"}
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
B=$PWD/tools/lib_alt.so
if [ -n "$TF" ] && [ "$TF" != "-" ]; then
  OF2D_LIB_PATH=$B timeout -k 10 600 python -u -m pytest $TF -x -q --timeout 300 --timeout-method thread > $OUT/tests_B.log 2>&1 || { tail -n 20 $OUT/tests_B.log; exit 1; }
  tail -n 1 $OUT/tests_B.log
fi
for r in $(seq $N); do
  timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline > $OUT/A$r.log 2>&1 || exit $?
  OF2D_LIB_PATH=$B timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline > $OUT/B$r.log 2>&1 || exit $?
  for v in A B; do
    python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/$v$r.log') if l.startswith('{')][-1]); print('$v$r', d['value'], d['roofline']['avg_launch_us'], d['roofline']['isolated_launch_us'], d['roofline']['loop_us_per_3_iterations'])"
  done
done

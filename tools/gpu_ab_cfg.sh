#!/bin/bash
# One-call A/B of a secondary configuration between the in-tree library (A)
# and tools/lib_alt.so (B), interleaved; B's parity tests first.
#   tools/gpu_ab_cfg.sh <tag> <config> <rounds> [pytest file]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1 CFG=$2 N=${3:-2} TF=$4
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
B=$PWD/tools/lib_alt.so
if [ -n "$TF" ] && [ "$TF" != "-" ]; then
  OF2D_LIB_PATH=$B timeout -k 10 600 python -u -m pytest $TF -x -q --timeout 300 --timeout-method thread > $OUT/tests_B.log 2>&1 || { tail -n 20 $OUT/tests_B.log; exit 1; }
  tail -n 1 $OUT/tests_B.log
fi
for r in $(seq $N); do
  timeout -k 10 300 python bench_configs.py --configs $CFG > $OUT/A$r.log 2>&1 || exit $?
  OF2D_LIB_PATH=$B timeout -k 10 300 python bench_configs.py --configs $CFG > $OUT/B$r.log 2>&1 || exit $?
  echo "A$r $(grep -o '"value": [0-9.]*' $OUT/A$r.log)   B$r $(grep -o '"value": [0-9.]*' $OUT/B$r.log)"
done

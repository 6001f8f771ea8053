#!/bin/bash
# One-call A/B/C.. of a secondary configuration: the in-tree library (A) and
# the builds given after the config (tools/lib_*.so), interleaved; each
# build's parity tests first.
#   tools/gpu_abn_cfg.sh <tag> <config> <rounds> <pytest file|-> <lib> [lib ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1 CFG=$2 N=$3 TF=$4
shift 4
OUT=gpurun_out/abn_$TAG
mkdir -p $OUT
for L in "$@"; do
  if [ "$TF" != "-" ]; then
    OF2D_LIB_PATH=$PWD/$L timeout -k 10 600 python -u -m pytest $TF -x -q --timeout 300 --timeout-method thread > $OUT/tests_$(basename $L).log 2>&1 || { tail -n 20 $OUT/tests_$(basename $L).log; exit 1; }
    echo "$L $(tail -n 1 $OUT/tests_$(basename $L).log)"
  fi
done
for r in $(seq $N); do
  timeout -k 10 300 python bench_configs.py --configs $CFG > $OUT/A$r.log 2>&1 || exit $?
  line="A$r $(grep -o '"value": [0-9.]*' $OUT/A$r.log | head -1)"
  for L in "$@"; do
    b=$(basename $L .so)
    OF2D_LIB_PATH=$PWD/$L timeout -k 10 300 python bench_configs.py --configs $CFG > $OUT/$b$r.log 2>&1 || exit $?
    line="$line   $b $(grep -o '"value": [0-9.]*' $OUT/$b$r.log | head -1)"
  done
  echo "$line"
done

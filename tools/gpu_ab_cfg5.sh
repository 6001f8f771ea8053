#!/bin/bash
# A/B of the 16384^2 one-GPU config 5 (HS GI triple kernel) and the 4096^2
# bench between the in-tree library (A) and tools/lib_alt.so (B), after A's HS tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/ab5_$TAG
mkdir -p $OUT
B=$PWD/tools/lib_alt.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_hs.py tests/test_gpu_convergence.py -x -q --timeout 300 --timeout-method thread > $OUT/tests_A.log 2>&1 || { tail -n 20 $OUT/tests_A.log; exit 1; }
tail -n 1 $OUT/tests_A.log
for r in 1 2; do
  timeout -k 10 300 python -u bench_configs.py --configs 5 --no-cpu --iters 300 > $OUT/c5A$r.log 2>&1 || exit $?
  OF2D_LIB_PATH=$B timeout -k 10 300 python -u bench_configs.py --configs 5 --no-cpu --iters 300 > $OUT/c5B$r.log 2>&1 || exit $?
  echo "A$r $(grep -o '"value": [0-9.]*\|"kernel_us": [0-9.]*' $OUT/c5A$r.log | tr '\n' ' ')   B$r $(grep -o '"value": [0-9.]*\|"kernel_us": [0-9.]*' $OUT/c5B$r.log | tr '\n' ' ')"
done

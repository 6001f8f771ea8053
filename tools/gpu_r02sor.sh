#!/bin/bash
# SOR harness A/B: tools/sor_harness_new against tools/sor_harness_old at
# 8192^2, 4096^2, 2048^2 (interleaved; field hashes must agree).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SOR_TAG:-sor_ab}
mkdir -p $OUT
for n in 8192 4096 2048; do
  for v in old new old new; do
    timeout -k 10 60 tools/sor_harness_$v $n $n 4 > $OUT/sor${n}_$v.log 2>&1 || exit $?
  done
  for v in old new; do
    echo "$n $v $(grep -E '^glead' $OUT/sor${n}_$v.log | awk '{print $6}' | tr '\n' ' ') $(grep -E 'strip 0:' $OUT/sor${n}_$v.log | tail -1) $(grep hash $OUT/sor${n}_$v.log | awk '{print $NF}')"
  done
done

#!/bin/bash
# Round-2 GPU session x: SOR row-load lead (batches per group 4/5/6 = 32/40/48
# rows) at 8192^2, 4096^2, 2048^2; field hashes must agree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r02x
mkdir -p $OUT
for n in 8192 4096 2048; do
  for v in 4 5 6 4; do
    timeout -k 10 60 tools/sor_harness_nb$v $n $n 4 > $OUT/sor${n}_nb$v.log 2>&1 || exit $?
    echo "$n nb$v $(grep -E '^glead' $OUT/sor${n}_nb$v.log | awk '{print $6}' | tr '\n' ' ') $(grep -E 'strip 0:' $OUT/sor${n}_nb$v.log | tail -1) $(grep hash $OUT/sor${n}_nb$v.log | awk '{print $NF}')"
  done
done

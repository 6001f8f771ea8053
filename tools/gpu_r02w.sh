#!/bin/bash
# Round-2 GPU session w: SOR row-load / value-store cache policy A/B (aux bits:
# 2 = nt) at 8192^2 and 4096^2, field hashes must agree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r02w
mkdir -p $OUT
for n in 8192 4096; do
  for v in 00 20 02 22 00; do
    timeout -k 10 60 tools/sor_harness_a$v $n $n 4 > $OUT/sor${n}_a$v.log 2>&1 || exit $?
    echo "$n aux$v $(grep -E '^glead' $OUT/sor${n}_a$v.log | tail -2 | awk '{print $6}' | tr '\n' ' ') $(grep hash $OUT/sor${n}_a$v.log | awk '{print $NF}')"
  done
done

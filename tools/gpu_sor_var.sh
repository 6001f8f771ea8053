#!/bin/bash
# SOR harness A/B over several builds: tools/sor_harness_<v> for each v in
# $SOR_VARS (default "old new"), interleaved at 8192^2, 4096^2, 2048^2; the
# field hashes must agree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SOR_TAG:-sor_var}
VARS=${SOR_VARS:-old new}
mkdir -p $OUT
for n in 8192 4096 2048; do
  for r in 1 2; do
    for v in $VARS; do
      timeout -k 10 60 tools/sor_harness_$v $n $n 4 > $OUT/sor${n}_${v}_$r.log 2>&1 || exit $?
    done
  done
  for v in $VARS; do
    echo "$n $v $(cat $OUT/sor${n}_${v}_*.log | grep -E '^glead' | awk '{print $6}' | tr '\n' ' ') $(grep -h 'strip 0:' $OUT/sor${n}_${v}_*.log | tail -1) $(grep -h hash $OUT/sor${n}_${v}_1.log | awk '{print $NF}')"
  done
done

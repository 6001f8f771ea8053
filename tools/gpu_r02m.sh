#!/bin/bash
# Round-2 GPU session m: SOR granule-vector lead (1-4 batches) A/B with field hashes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r02m
mkdir -p $OUT
for n in 8192 4096; do
  for g in 2 1 3 4; do
    timeout -k 10 60 tools/sor_harness_g$g $n $n 5 > $OUT/sor${n}_g$g.log 2>&1 || exit $?
  done
done
for f in $OUT/sor*.log; do grep -E "^glead" $f | tail -3; grep -E "^ +0:" $f; done

#!/bin/bash
# Round-2 GPU session l: SOR strips per block (1, 2, 4) A/B with field hashes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r02l
mkdir -p $OUT
for n in 8192 4096 2048; do
  for w in 1 2 4; do
    timeout -k 10 60 tools/sor_harness $n $n 4 $w > $OUT/sor${n}_w$w.log 2>&1 || exit $?
  done
done
for f in $OUT/sor*.log; do grep -E "^waves" $f | tail -2; grep -E "^ +0:" $f; done

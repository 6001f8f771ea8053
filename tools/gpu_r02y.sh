#!/bin/bash
# Round-2 GPU session y: SOR A/B, tools/sor_harness_new against tools/sor_harness_old
# in the harness, then config 4 A/B (tools/lib_alt.so) + fluid tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R02_TAG:-r02y}
mkdir -p $OUT
for n in 8192 4096 2048; do
  for v in old new old new; do
    timeout -k 10 60 tools/sor_harness_$v $n $n 4 > $OUT/sor${n}_$v.log 2>&1 || exit $?
    echo "$n $v $(grep -E '^glead' $OUT/sor${n}_$v.log | awk '{print $6}' | tr '\n' ' ') $(grep -E 'strip 0:' $OUT/sor${n}_$v.log | tail -1)"
  done
done
tools/gpu_ab_cfg.sh ${AB_TAG:-granule_layout} 4 2 tests/test_gpu_fluid.py || exit $?
for f in A1 A2 B1 B2; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/ab_${AB_TAG:-granule_layout}/$f.log | head -1)"; done

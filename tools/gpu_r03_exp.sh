#!/bin/bash
# round-3 experiments in one call: SOR strip order, slab launch events, Demons stage ablation
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > gpurun_out/r03q_$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; cat gpurun_out/r03q_$name.log; return $rc; }
step sor bash tools/sor_xcd_ab.sh && step gap bash tools/gpu_ab_bench.sh r03q_launchgap 3 - && step abl bash tools/demons_abl.sh run r03q_abl

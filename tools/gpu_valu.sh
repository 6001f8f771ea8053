#!/bin/bash
# Issue-side counters of the HS triple kernel (tools/hs_variants triple): one
# counter per rocprofv3 pass (kernel trace only, no sys/runtime trace).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
mkdir -p gpurun_out/valu
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/valu/avail.txt 2>&1 || true
for c in SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_ANY; do
  timeout -k 10 200 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/valu/$c" -o v -- "$R/tools/hs_variants" 4096 42 triple > gpurun_out/valu/$c.log 2>&1
  rc=$?
  echo "$c rc=$rc"
  [ $rc -le 1 ] || exit $rc
done

#!/bin/bash
# SOR step ablations (fluid_kernels.hip OF2D_SOR_ABL, timing only): strip 0's
# cycles per step and the sweep time of each harness build, interleaved:
#   tools/gpu_sor_abl.sh <rounds> <dimx> <dimy> <abl>...   (builds in tools/abx/sor/abl<N>)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rounds=$1 dx=$2 dy=$3; shift 3
for r in $(seq 1 $rounds); do
    for a in "$@"; do
        echo "== round $r abl $a ${dx}x${dy}"
        timeout -k 10 120 tools/abx/sor/abl$a $dx $dy 3 | grep -E "glead|strip 0" | tail -2 || exit $?
    done
done

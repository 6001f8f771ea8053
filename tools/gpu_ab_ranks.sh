#!/bin/bash
# ngpus_share timings (tools/time_ranks.py, fixed iterations, 1 / 2 / 8 ranks) of
# the in-tree library and tools/abx/<variant>s, interleaved:
#   tools/gpu_ab_ranks.sh <rounds> <variant>...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rounds=$1; shift
for r in $(seq 1 $rounds); do
    for v in tree "$@"; do
        lp=""; [ "$v" != tree ] && lp="$PWD/tools/abx/$v/libof2d.so"
        echo "== round $r $v"
        OF2D_LIB_PATH=$lp timeout -k 10 300 python -u tools/time_ranks.py 4096 2 fixed 1,2,8 2>&1 | grep -v amdgpu || exit 1
    done
done

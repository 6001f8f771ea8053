#!/bin/bash
# seqnorm_bench against each A/B library (tools/build_variant.sh), interleaved:
#   tools/gpu_ab_sn.sh <rounds> <args to seqnorm_bench> -- <variant>...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rounds=$1; shift
args=()
while [ "$1" != "--" ]; do args+=("$1"); shift; done
shift
for r in $(seq 1 $rounds); do
    for v in "$@"; do
        echo "== round $r $v"
        LD_LIBRARY_PATH=tools/ab/$v:/opt/rocm/lib timeout -k 10 120 tools/seqnorm_bench "${args[@]}" | tail -1 || exit $?
    done
done

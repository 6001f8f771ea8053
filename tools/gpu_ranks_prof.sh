#!/bin/bash
# ngpus path on one device: timings with the default and a larger hardware
# queue count, and a kernel trace of the fixed-iteration N=8 run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; tag=${1:?tag}
timeout -k 10 300 python -u tools/time_ranks.py 4096 3 fixed,conv 1,2,8 > $O/${tag}_ranks_q4.log 2>&1 || exit 1
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python -u tools/time_ranks.py 4096 3 fixed,conv 1,2,8 > $O/${tag}_ranks_q16.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/${tag}_ranksprof -o k -- python3 -u $PWD/tools/time_ranks.py 4096 1 fixed 8 > $O/${tag}_ranksprof.log 2>&1 || exit 1
echo done

#!/bin/bash
# PMC traffic of the HS triple kernel: two separate counter passes (kernel trace only,
# no sys/runtime trace), then calibration + profiles/hs_traffic.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
mkdir -p gpurun_out/pmc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc/fetch" -o f -- "$R/tools/hs_variants" 4096 42 triple > gpurun_out/pmc/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc/write" -o w -- "$R/tools/hs_variants" 4096 42 triple > gpurun_out/pmc/write.log 2>&1 || exit $?
find gpurun_out/pmc -name '*.csv' | head
python3 tools/pmc_traffic.py --out gpurun_out/hs_traffic.json $(find gpurun_out/pmc/fetch -name '*counter_collection.csv' | head -1) $(find gpurun_out/pmc/write -name '*counter_collection.csv' | head -1) 4096

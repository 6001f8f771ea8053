#!/bin/bash
# One-call A/B of one bench_configs.py configuration between the in-tree
# library (A) and tools/lib_alt.so (B), interleaved, after A's parity tests.
#   tools/gpu_ab_cfg.sh <tag> <config> <rounds> [pytest file|-]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1 CFG=$2 N=${3:-3} TF=${4:--}
OUT=gpurun_out/abc_$TAG
mkdir -p $OUT
B=$PWD/tools/lib_alt.so
if [ "$TF" != "-" ]; then
  timeout -k 10 600 python -u -m pytest $TF -x -q --timeout 300 --timeout-method thread > $OUT/tests_A.log 2>&1 || { tail -n 20 $OUT/tests_A.log; exit 1; }
  tail -n 1 $OUT/tests_A.log
fi
for r in $(seq $N); do
  timeout -k 10 300 python -u bench_configs.py --configs $CFG --no-cpu > $OUT/A$r.log 2>&1 || exit $?
  OF2D_LIB_PATH=$B timeout -k 10 300 python -u bench_configs.py --configs $CFG --no-cpu > $OUT/B$r.log 2>&1 || exit $?
  for v in A B; do
    python3 -c "import json; d=json.loads([l for l in open('$OUT/$v$r.log') if l.startswith('{')][-1]); print('$v$r', d['value'], d.get('ms_per_iter'))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$OUT/prof -o k -- python3 $PWD/bench_configs.py --configs $CFG --no-cpu --iters 30 > $OUT/prof.log 2>&1 || exit $?
python3 - "$PWD/$OUT/prof/k_kernel_stats.csv" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:8]:
    print(r['Name'][:70], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
PY

#!/bin/bash
# GPU session runner (one gpurun call): tools/gpu_session.sh <tag> <step>...
#   steps: tests (all gpu tests), sntests / ranks (Logger-norm / multi-device
#          tests), diag (tools/seqnorm_diag.py), conv (tools/time_convergence.py),
#          convprof (rocprofv3 kernel stats of conv), smoke, bench, prof (bench
#          under rocprofv3), cfgs (bench_configs.py), cfg3prof / cfg4prof
#          (rocprofv3 kernel trace of one secondary config, 50 iterations)
# Stops at the first step that faults / aborts / times out (rc > 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
tag=$1; shift
R=$PWD
step() {  # step <name> <timeout> <cmd...>
    local name=$1 to=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$to" "$@" > "$OUT/${tag}_$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 12 "$OUT/${tag}_$name.log"
    return $rc
}
for s in "$@"; do
    case $s in
        ranks) step ranks 600 python -u -m pytest tests/test_gpu_ranks.py -x -v --timeout 300 --timeout-method thread; rc=$?; [ $rc -le 1 ] || exit $rc ;;
        sntests) step sntests 600 python -u -m pytest tests/test_gpu_seqnorm.py tests/test_gpu_convergence.py -x -q --timeout 300 --timeout-method thread; rc=$?; [ $rc -le 1 ] || exit $rc ;;
        tests) step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread; rc=$?; [ $rc -le 1 ] || exit $rc ;;
        diag) step diag 600 python -u tools/seqnorm_diag.py 4096 8 || exit $? ;;
        conv) step conv 600 python -u tools/time_convergence.py 4096 3 || exit $? ;;
        convprof) step convprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/${tag}_convprof" -o conv -- python3 -u "$R/tools/time_convergence.py" 4096 1 || exit $? ;;
        smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
        bench) step bench 600 python bench.py || exit $? ;;
        prof) step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/${tag}_prof" -o hs -- python3 "$R/bench.py" --no-cpu-baseline || exit $? ;;
        cfgs) step cfgs 900 python -u bench_configs.py || exit $? ;;
        cfg4prof) step cfg4prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/${tag}_cfg4prof" -o k -- python3 -u "$R/bench_configs.py" --configs 4 --no-cpu --iters 50 || exit $? ;;
        cfg3prof) step cfg3prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/${tag}_cfg3prof" -o k -- python3 -u "$R/bench_configs.py" --configs 3 --no-cpu --iters 50 || exit $? ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo ALL-DONE

#!/bin/bash
# Fluid sweep with the increment behind it (SorInc): fluid GPU tests, then
# config 4 under environment settings (interleaved), then kernel traces.
#   tools/sor_inc_ab.sh <tag> [setting ...]   setting: VAR=value[,VAR=value]
#   (OF2D_SOR_NCONS=0: separate increment pass; N: N worker workgroups; the
#    timing-only OF2D_SOR_INC_SKIP of profiles/r03bf_* lived at commit 246f03d)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
tag=$1; shift
settings=${*:-"OF2D_SOR_NCONS=0 OF2D_SOR_NCONS=384 OF2D_SOR_NCONS=0 OF2D_SOR_NCONS=384"}
R=$PWD
timeout -k 10 600 python -u -m pytest tests/test_gpu_fluid.py -x -q --timeout 300 --timeout-method thread \
    > $OUT/${tag}_fluid_tests.log 2>&1
rc=$?; tail -n 3 $OUT/${tag}_fluid_tests.log; [ $rc -eq 0 ] || exit $rc
for st in $settings; do
    env ${st//,/ } timeout -k 10 300 python -u bench_configs.py --configs 4 --no-cpu \
        > $OUT/${tag}_one.log 2>&1 || { cat $OUT/${tag}_one.log; exit 1; }
    echo "$st $(grep '^{' $OUT/${tag}_one.log | tail -n 1)" | tee -a $OUT/${tag}_ab.log
done
for st in ${PROF:-}; do
    n=${st//[=,]/_}
    env ${st//,/ } timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/${tag}_prof_$n" -o k \
        -- python3 -u "$R/bench_configs.py" --configs 4 --no-cpu --iters 50 > $OUT/${tag}_prof_$n.log 2>&1 || exit $?
done
echo ALL-DONE

cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r02b
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r02b/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 5 gpurun_out/r02b/tests.log
[ $rc -le 1 ] || exit $rc
bash tools/gpu_pmc_groups.sh demons --configs 3 --iters 5 || exit $?
bash tools/gpu_pmc_groups.sh fluid --configs 4 --iters 5 || exit $?
echo ALL-DONE

set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05ai_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_convergence.py tests/test_gpu_rccl.py tests/test_gpu_workloads.py > gpurun_out/r05ai_tests.log 2>&1
echo rc=$?

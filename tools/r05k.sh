set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OF2D_LIB_PATH=$PWD/tools/abx/parts4/libof2d.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_convergence.py tests/test_gpu_hs.py > gpurun_out/r05k_parts4_tests.log 2>&1; rc=$?; echo "parts4 tests rc=$rc"
[ $rc -ge 124 ] && exit $rc
bash tools/gpu_ab_conv3.sh 2 parts2 parts4 > gpurun_out/r05k_parts_ab.log 2>&1 || exit $?
OF2D_CONV_FRESH=1 OF2D_CONV_ONLY=1 timeout -k 10 300 python -u tools/time_convergence.py 4096 2 > gpurun_out/r05k_fresh.log 2>&1 || exit $?
bash tools/gpu_ab_ranks.sh 1 sq1 sq2 > gpurun_out/r05k_ranks_ab.log 2>&1 || exit $?
bash tools/gpu.sh r05k freshprof > gpurun_out/r05k_freshprof_step.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_rccl.py > gpurun_out/r05k_rccl.log 2>&1; echo "rccl rc=$?"

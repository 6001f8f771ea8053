set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OF2D_LIB_PATH=$PWD/tools/abx/keep/libof2d.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_convergence.py tests/test_gpu_hs.py tests/test_gpu_examples.py > gpurun_out/r05ab_keep_tests.log 2>&1 || exit $?
bash tools/gpu_ab_conv3.sh 3 keep > gpurun_out/r05ab_keep_ab.log 2>&1
echo rc=$?

set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OF2D_LIB_PATH=$PWD/tools/abx/chkpass/libof2d.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_convergence.py > gpurun_out/r05ag_chkpass_tests.log 2>&1 || exit $?
bash tools/gpu_ab_conv3.sh 3 chkpass > gpurun_out/r05ag_chkpass_ab.log 2>&1 || exit $?
for v in tree chkpass; do lp=""; [ $v != tree ] && lp=$PWD/tools/abx/$v/libof2d.so; echo "== $v"; OF2D_LIB_PATH=$lp OF2D_CONV_FRESH=1 OF2D_CONV_ONLY=1 timeout -k 10 300 python -u tools/time_convergence.py 4096 2 || exit $?; done > gpurun_out/r05ag_fresh.log 2>&1
echo rc=$?

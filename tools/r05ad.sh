set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OF2D_LIB_PATH=$PWD/tools/abx/nshape/libof2d.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_convergence.py tests/test_gpu_seqnorm.py tests/test_gpu_hs.py > gpurun_out/r05ad_nshape_tests.log 2>&1 || exit $?
for r in 1 2; do for v in tree nshape; do lp=""; [ $v != tree ] && lp=$PWD/tools/abx/$v/libof2d.so; echo "== round $r $v"; OF2D_LIB_PATH=$lp OF2D_CONV_FRESH=1 OF2D_CONV_ONLY=1 timeout -k 10 300 python -u tools/time_convergence.py 4096 2 || exit $?; done; done > gpurun_out/r05ad_fresh.log 2>&1
bash tools/gpu_ab_conv3.sh 2 nshape > gpurun_out/r05ad_warm.log 2>&1
echo rc=$?

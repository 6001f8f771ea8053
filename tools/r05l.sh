set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OF2D_LIB_PATH=$PWD/tools/abx/prio3/libof2d.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_convergence.py tests/test_gpu_seqnorm.py > gpurun_out/r05l_prio3_tests.log 2>&1 || exit $?
bash tools/gpu_ab_conv3.sh 2 prio3 prio2 cuwalk > gpurun_out/r05l_prio_ab.log 2>&1 || exit $?
OF2D_LIB_PATH=$PWD/tools/abx/prio3/libof2d.so OF2D_CONV_FRESH=1 OF2D_CONV_ONLY=1 timeout -k 10 300 python -u tools/time_convergence.py 4096 2 > gpurun_out/r05l_prio3_fresh.log 2>&1 || exit $?
OF2D_LIB_PATH=$PWD/tools/abx/prio3/libof2d.so bash tools/gpu.sh r05l freshprof > gpurun_out/r05l_freshprof_step.log 2>&1 || exit $?
echo done

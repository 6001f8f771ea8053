set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu.sh r05p tests conv || exit $?
OF2D_CONV_FRESH=1 OF2D_CONV_ONLY=1 timeout -k 10 300 python -u tools/time_convergence.py 4096 2 > gpurun_out/r05p_fresh.log 2>&1
echo rc=$?

set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_ab_conv3.sh 2 cuwalk cw8 cw24 cw32 > gpurun_out/r05m_cuwalk_ab.log 2>&1 || exit $?
echo done

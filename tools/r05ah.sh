set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_ab_conv3.sh 2 chkpass chkpass_nonear > gpurun_out/r05ah_ab.log 2>&1 || exit $?
OF2D_LIB_PATH=$PWD/tools/abx/chkpass/libof2d.so OF2D_CONV_CASE=texture OF2D_CONV_ONLY=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/r05ah_texprof" -o k -- python3 -u tools/time_convergence.py 4096 1 > gpurun_out/r05ah_texprof.log 2>&1
echo rc=$?

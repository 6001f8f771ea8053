set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
bash tools/gpu.sh r05ac freshprof || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r05ac_cfg3prof" -o k -- python3 -u "$R/bench_configs.py" --configs 3 --no-cpu > gpurun_out/r05ac_cfg3prof.log 2>&1
echo rc=$?
